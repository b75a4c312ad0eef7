// internal.hh -- symbols shared by the library's translation units only.
#pragma once
#include "../../include/click_amd_cksum.h"

extern "C" int clk_ctx_set_error_internal(clk_ctx *ctx, const char *msg);
