// copy_probe.hip -- read+write bandwidth probes (diagnostic, not product):
// what a kernel that reads and writes HBM can reach on MI355X, as the
// ceiling for IPFragmenter (reads ~ writes) and for the Set kernels (a
// read stream with one write per packet).
//   copy:    dst[i] = src[i], 16 B per lane, U loads in flight, load/store
//            cache policy default or nontemporal
//   stream+block: read a 16M x 1536 B arena (C3 layout) and write the first
//            64 B block of every slot back (the fused whole-block Set), in
//            the same kernel
//   stream, then block: the same reads in one kernel, the block writes in a
//            second kernel (the two-phase Set)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/copy_probe tools/probes/copy_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) copy_kernel(const u32x4 *src, u32x4 *dst, uint64_t n16)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * nt < n16; i += U * nt) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            v[u] = NTL ? __builtin_nontemporal_load((const gu32x4 *)(src + i + u * nt)) : ((const gu32x4 *)src)[i + u * nt];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NTS)
                __builtin_nontemporal_store(v[u], (gu32x4 *)(dst + i + u * nt));
            else
                ((gu32x4 *)dst)[i + u * nt] = v[u];
        }
    }
    for (; i < n16; i += nt)
        dst[i] = src[i];
}

// 16 lanes per 1536 B slot, 6 chunks of 16 B each per lane (96 chunks =
// 1536 B), nontemporal reads; WRITE: the lanes holding chunks 0..3 store them
// back (a whole 64 B block) after the group's reduction.
template <bool WRITE>
__global__ void __launch_bounds__(256) stream_slots(u32x4 *base, uint64_t nslots, unsigned long long *out)
{
    const uint32_t gl = threadIdx.x & 15;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / 16;
    uint32_t acc = 0;
    for (uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 16; s < nslots; s += groups) {
        u32x4 *p = base + s * 96;
        u32x4 v[6];
#pragma unroll
        for (int k = 0; k < 6; k++)
            v[k] = __builtin_nontemporal_load((const gu32x4 *)(p + 16 * k + gl));
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 6; k++)
            x += v[k][0] + v[k][1] + v[k][2] + v[k][3];
        for (int m = 1; m < 16; m <<= 1)
            x += __shfl_xor(x, m, 64);
        if (WRITE && gl < 4) {
            u32x4 w = v[0];
            w[1] = x;
            ((gu32x4 *)p)[gl] = w;
        }
        acc += x;
    }
    if (acc == 0x12345678u)
        atomicAdd(out, 1ull);
}

// one lane per slot: store the slot's first 64 B block (4 x 16 B), or 2 B
template <bool FULL>
__global__ void __launch_bounds__(256) block_writes(u32x4 *base, uint64_t nslots)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += nt) {
        u32x4 *p = base + s * 96;
        if (FULL) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                ((gu32x4 *)p)[q] = u32x4{(uint32_t)s, 1, 2, (uint32_t)q};
        } else {
            *(uint16_t *)((uint8_t *)p + 26) = (uint16_t)s;
        }
    }
}

template <typename F>
static float best_ms(F f, int reps = 5)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    float best = 1e9;
    for (int r = 0; r < reps; r++) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best)
            best = ms;
    }
    return best;
}

int main()
{
    const uint64_t bytes = 8ull << 30, n16 = bytes / 16;
    u32x4 *src, *dst;
    if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&dst, bytes) != hipSuccess)
        return 1;
    hipMemset(src, 1, bytes);
    hipMemset(dst, 0, bytes);
    const int grid = 65536;
#define COPY(U, L, S, name)                                                                                   \
    {                                                                                                         \
        float ms = best_ms([&] { copy_kernel<U, L, S><<<grid, 256>>>(src, dst, n16); });                       \
        printf("{\"probe\": \"copy %s\", \"ms\": %.4f, \"rw_TBs\": %.3f}\n", name, ms, 2.0 * bytes / ms / 1e9); \
    }
    COPY(4, false, false, "U4 default")
    COPY(4, true, false, "U4 nt-load")
    COPY(4, false, true, "U4 nt-store")
    COPY(4, true, true, "U4 nt-both")
    COPY(8, false, false, "U8 default")
    COPY(8, true, true, "U8 nt-both")
    COPY(2, false, false, "U2 default")
    hipFree(dst);
    // C3 layout: 16M slots of 1536 B (25.8 GB)
    const uint64_t nslots = 16ull << 20;
    u32x4 *arena;
    unsigned long long *out;
    hipFree(src);
    if (hipMalloc(&arena, nslots * 1536) != hipSuccess || hipMalloc(&out, 8) != hipSuccess)
        return 2;
    hipMemset(arena, 3, nslots * 1536);
    const int sgrid = 262144;
    float r0 = best_ms([&] { stream_slots<false><<<sgrid, 256>>>(arena, nslots, out); });
    float r1 = best_ms([&] { stream_slots<true><<<sgrid, 256>>>(arena, nslots, out); });
    float w64 = best_ms([&] { block_writes<true><<<grid, 256>>>(arena, nslots); });
    float w2 = best_ms([&] { block_writes<false><<<grid, 256>>>(arena, nslots); });
    printf("{\"probe\": \"stream 16M x 1536 B, read only\", \"ms\": %.4f, \"read_TBs\": %.3f}\n", r0,
           nslots * 1536.0 / r0 / 1e9);
    printf("{\"probe\": \"stream + whole 64 B block write per slot (fused)\", \"ms\": %.4f}\n", r1);
    printf("{\"probe\": \"64 B block write per slot alone\", \"ms\": %.4f}\n", w64);
    printf("{\"probe\": \"2 B write per slot alone\", \"ms\": %.4f}\n", w2);
    printf("{\"probe\": \"stream, then block writes (two kernels)\", \"ms\": %.4f}\n", r0 + w64);
    printf("{\"probe\": \"stream, then 2 B writes (two kernels)\", \"ms\": %.4f}\n", r0 + w2);
    hipFree(arena);
    return 0;
}
