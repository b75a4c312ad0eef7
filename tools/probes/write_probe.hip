// write_probe.hip -- scattered-store microbenchmark (diagnostic, not product):
// one store per 1536 B slot over a 25 GB arena, as the two-phase Set's
// field_scatter_kernel does, at several store widths.  Answers whether the
// partial-sector write itself (ECC read-modify-write) is the limiter.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) probe(uint8_t *base, uint64_t n, uint64_t stride)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nt) {
        uint8_t *p = base + i * stride;
        if (MODE == 0)                       // 2 B at +26 (uh_sum)
            *(uint16_t *)(p + 26) = (uint16_t)i;
        else if (MODE == 1)                  // 4 B dword at +24
            *(uint32_t *)(p + 24) = (uint32_t)i;
        else if (MODE == 2) {                // full 32 B sector [0, 32)
            *(u32x4 *)(p) = u32x4{(uint32_t)i, 1, 2, 3};
            *(u32x4 *)(p + 16) = u32x4{4, 5, 6, (uint32_t)i};
        } else if (MODE == 3) {              // full 64 B [0, 64)
            for (int k = 0; k < 4; k++)
                *(u32x4 *)(p + 16 * k) = u32x4{(uint32_t)i, 1, 2, (uint32_t)k};
        } else if (MODE == 4) {              // 16 B at [16, 32)
            *(u32x4 *)(p + 16) = u32x4{4, 5, 6, (uint32_t)i};
        } else {                             // read 32 B + write 2 B (RMW in the kernel)
            u32x4 a = *(volatile u32x4 *)(p + 16);
            *(uint16_t *)(p + 26) = (uint16_t)(a[0] + i);
        }
    }
}

int main()
{
    const uint64_t n = 16ull << 20, stride = 1536;
    uint8_t *base;
    if (hipMalloc(&base, n * stride) != hipSuccess) return 1;
    hipMemset(base, 0, n * stride);
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    const char *names[] = {"2B@26", "4B@24", "32B sector", "64B", "16B@16", "read32+write2"};
    for (int grid : {16384, 65536}) {
        for (int mode = 0; mode < 6; mode++) {
            float best = 1e9;
            for (int r = 0; r < 5; r++) {
                hipEventRecord(s);
                switch (mode) {
                case 0: probe<0><<<grid, 256>>>(base, n, stride); break;
                case 1: probe<1><<<grid, 256>>>(base, n, stride); break;
                case 2: probe<2><<<grid, 256>>>(base, n, stride); break;
                case 3: probe<3><<<grid, 256>>>(base, n, stride); break;
                case 4: probe<4><<<grid, 256>>>(base, n, stride); break;
                default: probe<5><<<grid, 256>>>(base, n, stride); break;
                }
                hipEventRecord(e);
                hipEventSynchronize(e);
                float ms;
                hipEventElapsedTime(&ms, s, e);
                if (ms < best) best = ms;
            }
            printf("{\"grid\": %d, \"mode\": \"%s\", \"ms\": %.4f, \"Gstores_per_s\": %.1f}\n", grid, names[mode], best,
                   n / (best * 1e-3) / 1e9);
        }
    }
    hipFree(base);
    return 0;
}
