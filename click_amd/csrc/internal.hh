// internal.hh -- symbols shared by the library's translation units only.
#pragma once
#include <atomic>
#include <stdint.h>
#include "../../include/click_amd_cksum.h"

extern "C" int clk_ctx_set_error_internal(clk_ctx *ctx, const char *msg);
// Changes whenever a host region is registered or unregistered (the glue's
// zero-copy lookup cache is valid for one generation).
extern "C" uint64_t clk_host_generation_internal(void);
namespace clk {
extern std::atomic<uint64_t> host_regions_gen;     // (the counter itself: read inline per packet)
inline uint64_t host_generation() { return host_regions_gen.load(std::memory_order_acquire); }
}
// Test hook: the n-th checked HIP call of the element glue's flush path
// from now on fails (tests/test_gpu_glue_faults.py); 0 disarms it.
extern "C" void clk_glue_inject_fault_internal(int nth);
