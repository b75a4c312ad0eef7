// frag_pipe_probe.hip -- would the fragmenter gain from issuing a packet's
// payload loads before the previous packet's stores? (diagnostic, not
// product)
// C3 shape as frag_align_probe.hip: 16M packets in 1536 B slots, 928 B of
// payload each (source 12 mod 16) copied into a packed region (976 B
// stride, destination 4 mod 16), one 16-lane group per packet, four 16 B
// chunks per lane.  gfx9 counts stores in vmcnt, so a group that loads
// packet j+1 only after storing packet j waits for j's stores at its next
// load wait: one load and one store round trip per packet.
//   serial   per packet: loads, then stores (frag_write_kernel today)
//   pipe     packet j+1's loads issued before packet j's stores
//   pair     two packets per step: both packets' loads, then both stores
// Occupancy is pinned with dynamic LDS per 256-thread workgroup (WG/CU =
// 160 KB / LDS): 4 waves per SIMD (the product kernel's 118 VGPRs), 3 (what
// a pipelined kernel's extra registers would leave) and the probe's own.
// Build: hipcc --offload-arch=gfx950 -O3 -o frag_pipe_probe frag_pipe_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef __attribute__((address_space(1))) u32x4_a4 g4;

constexpr uint32_t SOFF = 572, DOFF = 20, DSTRIDE = 976, NCH = 58;

__device__ __forceinline__ void load4(const uint8_t *s, uint32_t gl, u32x4_a4 *v)
{
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t c = gl + 16 * u;
        v[u] = c < NCH ? *(const g4 *)(s + 16 * c) : u32x4_a4{0, 0, 0, 0};
    }
}
__device__ __forceinline__ void store4(uint8_t *d, uint32_t gl, const u32x4_a4 *v)
{
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t c = gl + 16 * u;
        if (c < NCH)
            *(g4 *)(d + 16 * c) = v[u];
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) copy_payload(const uint8_t *src, uint8_t *dst, uint64_t n)
{
    extern __shared__ uint32_t pad[];                    // occupancy only
    if (n == 0)
        pad[threadIdx.x] = 0;
    const uint32_t gl = threadIdx.x & 15;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / 16;
    uint64_t p = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 16;
    if (MODE == 0) {
        for (; p < n; p += groups) {
            u32x4_a4 v[4];
            load4(src + p * 1536 + SOFF, gl, v);
            store4(dst + p * DSTRIDE + DOFF, gl, v);
        }
    } else if (MODE == 1) {
        if (p >= n)
            return;
        u32x4_a4 v[4];
        load4(src + p * 1536 + SOFF, gl, v);
        for (;;) {
            const uint64_t q = p + groups;
            u32x4_a4 w[4];
            if (q < n)
                load4(src + q * 1536 + SOFF, gl, w);
            store4(dst + p * DSTRIDE + DOFF, gl, v);
            if (q >= n)
                break;
#pragma unroll
            for (int u = 0; u < 4; u++)
                v[u] = w[u];
            p = q;
        }
    } else {
        for (; p < n; p += 2 * groups) {
            const uint64_t q = p + groups;
            u32x4_a4 v[4], w[4];
            load4(src + p * 1536 + SOFF, gl, v);
            if (q < n)
                load4(src + q * 1536 + SOFF, gl, w);
            store4(dst + p * DSTRIDE + DOFF, gl, v);
            if (q < n)
                store4(dst + q * DSTRIDE + DOFF, gl, w);
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
    const char *names[] = {"serial", "pipe", "pair"};
    for (int wps : {4, 3, 0}) {                           // waves per SIMD pinned by LDS (0: not pinned)
        const size_t lds = wps ? (160 * 1024) / wps - 1024 : 0;
        for (int grid : {16384, 65536}) {
            for (int mode = 0; mode < 3; mode++) {
                float best = 1e9;
                for (int r = 0; r < 7; r++) {
                    hipEventRecord(a);
                    if (mode == 0)
                        copy_payload<0><<<grid, 256, lds>>>(src, dst, n);
                    else if (mode == 1)
                        copy_payload<1><<<grid, 256, lds>>>(src, dst, n);
                    else
                        copy_payload<2><<<grid, 256, lds>>>(src, dst, n);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    if (r > 0 && ms < best)
                        best = ms;
                }
                if (hipGetLastError() != hipSuccess) {
                    printf("{\"error\": \"launch\", \"lds\": %zu}\n", lds);
                    return 3;
                }
                printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"grid\": %d, \"ms\": %.4f, \"TBs_rw\": %.3f}\n",
                       names[mode], wps, grid, best, n * 928.0 * 2 / (best * 1e-3) / 1e12);
                fflush(stdout);
            }
        }
    }
    hipFree(src);
    hipFree(dst);
    return 0;
}
