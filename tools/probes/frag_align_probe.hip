// frag_align_probe.hip -- what do the fragmenter's unaligned 16 B payload
// accesses cost? (diagnostic, not product)
// C3 shape: 16M packets in 1536 B slots; each copies 928 B of payload (the
// appended fragments' bytes at MTU 576) into a packed output region, one
// 16-lane group per packet, four 16 B chunks per lane loaded before any
// store (as frag_write_kernel).  Variants by (source offset in the slot,
// destination offset in the region, region stride):
//   prod      572 / 20 / 976   source 12 mod 16, destination 4 mod 16 (the product's case)
//   aligned   576 / 16 / 976   both 16 B aligned
//   ld_al     576 / 20 / 976   aligned loads, unaligned stores
//   st_al     572 / 16 / 976   unaligned loads, aligned stores
//   al_1024   576 / 64 / 1024  aligned, each region its own 64 B blocks
// Build: hipcc --offload-arch=gfx950 -O3 -o frag_align_probe frag_align_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef __attribute__((address_space(1))) u32x4_a4 g4;

__global__ void __launch_bounds__(256) copy_payload(const uint8_t *src, uint8_t *dst, uint64_t n, uint32_t soff,
                                                    uint32_t doff, uint32_t dstride)
{
    const uint32_t gl = threadIdx.x & 15;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / 16;
    for (uint64_t p = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 16; p < n; p += groups) {
        const uint8_t *s = src + p * 1536 + soff;
        uint8_t *d = dst + p * dstride + doff;
        u32x4_a4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t c = gl + 16 * u;
            v[u] = c < 58 ? __builtin_nontemporal_load((const g4 *)(s + 16 * c)) : u32x4_a4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t c = gl + 16 * u;
            if (c < 58)
                *(g4 *)(d + 16 * c) = v[u];
        }
    }
}

int main()
{
    const uint64_t n = 16ull << 20;
    uint8_t *src, *dst;
    if (hipMalloc(&src, n * 1536) != hipSuccess || hipMalloc(&dst, n * 1024) != hipSuccess)
        return 2;
    hipMemset(src, 1, n * 1536);
    hipMemset(dst, 0, n * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct V {
        const char *name;
        uint32_t soff, doff, stride;
    } vs[] = {{"prod", 572, 20, 976}, {"aligned", 576, 16, 976}, {"ld_al", 576, 20, 976},
              {"st_al", 572, 16, 976}, {"al_1024", 576, 64, 1024}, {"prod_again", 572, 20, 976}};
    for (int grid : {16384, 65536}) {
        for (const V &v : vs) {
            float best = 1e9;
            for (int r = 0; r < 7; r++) {
                hipEventRecord(a);
                copy_payload<<<grid, 256>>>(src, dst, n, v.soff, v.doff, v.stride);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (r > 0 && ms < best)
                    best = ms;
            }
            printf("{\"variant\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"TBs_rw\": %.3f}\n", v.name, grid, best,
                   n * 928.0 * 2 / (best * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    hipFree(src);
    hipFree(dst);
    return 0;
}
