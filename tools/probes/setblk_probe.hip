// setblk_probe.hip -- where does a fused Set's whole-block write cost go?
// (the C3 layout: 16M slots of 1536 B, each slot's first 64 B block written
// back whole, as a fused SetUDPChecksum would).
//
// gfx9 counts stores in vmcnt with the loads, in order: a wave that stores
// and then loads again waits, at its next load wait, for the stores too.
// The variants separate that coupling from the HBM cost of the writes:
//   read       the read stream alone (16 lanes x 6 nontemporal 16 B loads per slot)
//   fused      each group stores its block right after its slot (as copy_probe.hip)
//   runblk1    a workgroup owns ONE run of 64 slots; the blocks are parked in
//              LDS and stored after the run's reads -- the workgroup ends
//              there, so no load ever waits behind a store
//   runblkN    the same with N runs per workgroup (stores between runs)
//   two        the read stream, then a second kernel writing the blocks
// Build: hipcc --offload-arch=gfx950 -O3 -o setblk_probe setblk_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ uint32_t slot_sum(const u32x4 *p, uint32_t gl, u32x4 &first)
{
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
    first = v[0];
    return x;
}

template <bool WRITE>
__global__ void __launch_bounds__(256) fused(u32x4 *base, uint64_t nslots, unsigned long long *out)
{
    const uint32_t gl = threadIdx.x & 15;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / 16;
    uint32_t acc = 0;
    for (uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 16; s < nslots; s += groups) {
        u32x4 w;
        const uint32_t x = slot_sum(base + s * 96, gl, w);
        if (WRITE && gl < 4) {
            w[1] = x;
            ((gu32x4 *)(base + s * 96))[gl] = w;
        }
        acc += x;
    }
    if (acc == 0x12345678u)
        atomicAdd(out, 1ull);
}

// runs of 64 slots (4 passes of 16), blocks parked in LDS, stored whole after
// the run: thread t stores quarter t & 3 of block t >> 2 (coalesced)
template <bool NTS>
__global__ void __launch_bounds__(256) runblk(u32x4 *base, uint64_t nslots, unsigned long long *out)
{
    __shared__ u32x4 blk[64][4];
    const uint32_t gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint64_t nruns = nslots / 64;
    uint32_t acc = 0;
    for (uint64_t run = blockIdx.x; run < nruns; run += gridDim.x) {
#pragma unroll 1
        for (uint32_t p = 0; p < 4; p++) {
            const uint64_t s = run * 64 + p * 16 + grp;
            u32x4 w;
            const uint32_t x = slot_sum(base + s * 96, gl, w);
            if (gl < 4) {
                w[1] = x;
                blk[p * 16 + grp][gl] = w;
            }
            acc += x;
        }
        __syncthreads();
        const uint32_t b = threadIdx.x >> 2, q = threadIdx.x & 3;
        gu32x4 *dst = (gu32x4 *)(base + (run * 64 + b) * 96 + q);
        if (NTS)
            __builtin_nontemporal_store(blk[b][q], dst);
        else
            *dst = blk[b][q];
        __syncthreads();
    }
    if (acc == 0x12345678u)
        atomicAdd(out, 1ull);
}

__global__ void __launch_bounds__(256) block_writes(u32x4 *base, uint64_t nslots)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslots * 4; t += nt) {
        const uint64_t s = t >> 2;
        ((gu32x4 *)(base + s * 96))[t & 3] = u32x4{(uint32_t)s, 1, 2, (uint32_t)t};
    }
}

template <typename F>
static float best_ms(F f, int reps = 7)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
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
    const uint64_t nslots = 16ull << 20, nruns = nslots / 64;
    u32x4 *arena;
    unsigned long long *out;
    if (hipMalloc(&arena, nslots * 1536) != hipSuccess || hipMalloc(&out, 8) != hipSuccess)
        return 2;
    hipMemset(arena, 3, nslots * 1536);
    const int sgrid = 262144;
    for (int round = 0; round < 2; round++) {
        const float r0 = best_ms([&] { fused<false><<<sgrid, 256>>>(arena, nslots, out); });
        const float f1 = best_ms([&] { fused<true><<<sgrid, 256>>>(arena, nslots, out); });
        const float b1 = best_ms([&] { runblk<false><<<(unsigned)nruns, 256>>>(arena, nslots, out); });
        const float b1n = best_ms([&] { runblk<true><<<(unsigned)nruns, 256>>>(arena, nslots, out); });
        const float b4 = best_ms([&] { runblk<false><<<(unsigned)(nruns / 4), 256>>>(arena, nslots, out); });
        const float b16 = best_ms([&] { runblk<false><<<(unsigned)(nruns / 16), 256>>>(arena, nslots, out); });
        const float w = best_ms([&] { block_writes<<<65536, 256>>>(arena, nslots); });
        const float two = best_ms([&] {
            fused<false><<<sgrid, 256>>>(arena, nslots, out);
            block_writes<<<65536, 256>>>(arena, nslots);
        });
        printf("{\"round\": %d, \"read_ms\": %.4f, \"read_TBs\": %.3f, \"fused_ms\": %.4f, \"runblk1_ms\": %.4f, "
               "\"runblk1_nt_ms\": %.4f, \"runblk4_ms\": %.4f, \"runblk16_ms\": %.4f, \"block_writes_ms\": %.4f, "
               "\"two_kernels_ms\": %.4f}\n",
               round, r0, nslots * 1536.0 / r0 / 1e9, f1, b1, b1n, b4, b16, w, two);
        fflush(stdout);
    }
    hipFree(arena);
    return 0;
}
