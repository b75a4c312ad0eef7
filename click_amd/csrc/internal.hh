// internal.hh -- symbols shared by the library's translation units only.
#pragma once
#include "../../include/click_amd_cksum.h"

extern "C" int clk_ctx_set_error_internal(clk_ctx *ctx, const char *msg);
// Changes whenever a host region is registered or unregistered (the glue's
// zero-copy lookup cache is valid for one generation).
extern "C" uint64_t clk_host_generation_internal(void);
