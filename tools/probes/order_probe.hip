// order_probe.hip -- does the ORDER of the two-phase Set's scattered field
// writes change their cost? (diagnostic, not product)
// The same 16M two-byte stores, one per 1536 B slot at +26 (C3's uh_sum), as
// field_scatter_kernel issues them, with the slot of global thread t taken
// from a bijection of [0, n):
//   linear     t                                   (the product's order)
//   tileAxB    within tiles of A*B slots, lane r -> (r % A) * B + r / A
//              (a wave's 64 stores spread B slots apart instead of adjacent)
//   hash       t * 0x9E3779B1 mod 2^24             (no locality at all)
//   xcd        workgroup b -> block (b % 8) * nb/8 + b / 8: each XCD writes one
//              contiguous eighth of the arena
// Each order with plain and with nontemporal stores; linear also as the
// grid-stride loop at 16K workgroups the product launches.
// Build: hipcc --offload-arch=gfx950 -O3 -o order_probe order_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __attribute__((address_space(1))) uint16_t gu16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum { LINEAR, T64x64, T64x16, T16x64, T64x4, HASH, XCD, NORD };

template <int ORD>
__device__ __forceinline__ uint64_t slot_of(uint64_t t, uint64_t n)
{
    if (ORD == LINEAR)
        return t;
    if (ORD == HASH)
        return (t * 0x9E3779B1ull) & (n - 1);
    if (ORD == XCD) {
        const uint64_t nb = n / 256, b = t / 256;
        return ((b % 8) * (nb / 8) + b / 8) * 256 + t % 256;
    }
    constexpr uint64_t A = ORD == T16x64 ? 16 : 64, B = ORD == T64x64 || ORD == T16x64 ? 64 : ORD == T64x16 ? 16 : 4;
    const uint64_t tile = t / (A * B), r = t % (A * B);
    return tile * (A * B) + (r % A) * B + r / A;
}

template <int ORD, bool NT>
__global__ void __launch_bounds__(256) scatter(uint8_t *base, uint64_t n)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += nt) {
        const uint64_t s = slot_of<ORD>(t, n);
        gu16 *p = (gu16 *)(base + s * 1536 + 26);
        if (NT)
            __builtin_nontemporal_store((uint16_t)s, p);
        else
            *p = (uint16_t)s;
    }
}

// a read of the whole arena between timed launches, so that no launch finds
// the previous one's dirty lines in L2 / the memory-side cache
__global__ void __launch_bounds__(256) sweep(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        x += v[0] ^ v[3];
    }
    if (x == 0x12345678u)
        atomicAdd(out, 1ull);
}

template <int ORD, bool NT>
static float run(uint8_t *base, uint64_t n, unsigned grid, unsigned long long *out)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 6; r++) {
        sweep<<<65536, 256>>>((const u32x4 *)base, n * 1536 / 16, out);
        hipEventRecord(a);
        scatter<ORD, NT><<<grid, 256>>>(base, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r > 0 && ms < best)
            best = ms;
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    return best;
}

template <int ORD>
static void both(const char *name, uint8_t *base, uint64_t n, unsigned grid, unsigned long long *out)
{
    const float p = run<ORD, false>(base, n, grid, out), q = run<ORD, true>(base, n, grid, out);
    printf("{\"order\": \"%s\", \"grid\": %u, \"plain_ms\": %.4f, \"nt_ms\": %.4f, \"nt_Gstores_per_s\": %.1f}\n", name,
           grid, p, q, n / (q * 1e-3) / 1e9);
    fflush(stdout);
}

int main()
{
    const uint64_t n = 16ull << 20;
    uint8_t *base;
    unsigned long long *out;
    if (hipMalloc(&base, n * 1536) != hipSuccess || hipMalloc(&out, 8) != hipSuccess)
        return 2;
    hipMemset(base, 0, n * 1536);
    const unsigned full = (unsigned)(n / 256);
    both<LINEAR>("linear_grid16k", base, n, 16384, out);
    both<LINEAR>("linear", base, n, full, out);
    both<T64x64>("tile64x64", base, n, full, out);
    both<T64x16>("tile64x16", base, n, full, out);
    both<T16x64>("tile16x64", base, n, full, out);
    both<T64x4>("tile64x4", base, n, full, out);
    both<HASH>("hash", base, n, full, out);
    both<XCD>("xcd", base, n, full, out);
    both<LINEAR>("linear_again", base, n, full, out);
    hipFree(base);
    return 0;
}
