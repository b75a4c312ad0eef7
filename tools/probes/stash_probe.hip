// stash_probe.hip -- can a Set avoid both the in-stream scattered writes and
// the memory controller's read-modify-write of a 2-byte field store?
// (diagnostic, not product).  C3 layout: 16M slots of 1536 B.
//   read:          the Check stream alone (16 lanes per slot, 6 chunks/lane)
//   read+work:     + one dense 4 B word per slot (today's two-phase pass 1)
//   read+stash:    + the slot's first 64 B block copied to a dense buffer
//                  (lanes 0-3 of the group, 1 KB contiguous per wave store)
//   read+work64:   the dense 4 B words of 16 consecutive slots gathered in one
//                  wave (4 slots per pass, 4 passes) and stored as one whole
//                  64 B block
//   scatter2:      one lane per slot writes 2 B into the slot (pass 2 today)
//   stash->block:  4 lanes per slot read the dense stash and write the whole
//                  64 B block back into the slot (no read of the arena)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/stash_probe tools/probes/stash_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

// MODE 0 read only, 1 + dense 4 B word, 2 + dense 64 B stash
template <int MODE>
__global__ void __launch_bounds__(256) stream_slots(const u32x4 *base, uint64_t nslots, uint32_t *work, u32x4 *stash,
                                                    unsigned long long *out)
{
    const uint32_t gl = threadIdx.x & 15;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / 16;
    uint32_t acc = 0;
    for (uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 16; s < nslots; s += groups) {
        const u32x4 *p = base + s * 96;
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
        if (MODE == 1 && gl == 0)
            work[s] = x;
        if (MODE == 2 && gl < 4) {
            u32x4 w = v[0];
            if (gl == 1)
                w[2] = (w[2] & 0xFFFF0000u) | (x & 0xFFFFu);
            ((gu32x4 *)stash)[s * 4 + gl] = w;
        }
        acc += x;
    }
    if (acc == 0x12345678u)
        atomicAdd(out, 1ull);
}

// a wave owns 16 consecutive slots: pass j takes slots 16w + 4j + group
__global__ void __launch_bounds__(256) stream_work64(const u32x4 *base, uint64_t nslots, uint32_t *work,
                                                     unsigned long long *out)
{
    const uint32_t lane = threadIdx.x & 63, gl = lane & 15, grp = lane >> 4;
    const uint64_t nwaves = (uint64_t)gridDim.x * blockDim.x / 64;
    uint32_t acc = 0;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; w * 16 < nslots; w += nwaves) {
        u32x4 mine = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t s = w * 16 + 4 * j + grp;
            const u32x4 *p = base + s * 96;
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
            // slots 16w + 4j + 0..3 are words 4j..4j+3 of the block: lane j's
            const uint32_t y0 = __shfl(x, 0, 64), y1 = __shfl(x, 16, 64), y2 = __shfl(x, 32, 64), y3 = __shfl(x, 48, 64);
            if (lane == (uint32_t)j)
                mine = u32x4{y0, y1, y2, y3};
            acc += x;
        }
        if (lane < 4)          // one store instruction: the whole 64 B block
            ((gu32x4 *)work)[w * 4 + lane] = mine;
    }
    if (acc == 0x12345678u)
        atomicAdd(out, 1ull);
}

__global__ void __launch_bounds__(256) scatter2(u32x4 *base, const uint32_t *work, uint64_t nslots)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += nt)
        *(uint16_t *)((uint8_t *)(base + s * 96) + 26) = (uint16_t)work[s];
}

__global__ void __launch_bounds__(256) stash_to_block(u32x4 *base, const u32x4 *stash, uint64_t nslots)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots * 4; i += nt) {
        u32x4 w = __builtin_nontemporal_load((const gu32x4 *)(stash + i));
        ((gu32x4 *)base)[(i >> 2) * 96 + (i & 3)] = w;
    }
}

template <typename F>
static float best_ms(F f, int reps = 7)
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
    const uint64_t nslots = 16ull << 20;
    u32x4 *arena, *stash;
    uint32_t *work;
    unsigned long long *out;
    if (hipMalloc(&arena, nslots * 1536) != hipSuccess || hipMalloc(&stash, nslots * 64) != hipSuccess ||
        hipMalloc(&work, nslots * 4) != hipSuccess || hipMalloc(&out, 8) != hipSuccess)
        return 2;
    hipMemset(arena, 3, nslots * 1536);
    hipMemset(work, 0, nslots * 4);
    const int sgrid = 262144, grid = 65536;
    for (int round = 0; round < 2; round++) {
        float r0 = best_ms([&] { stream_slots<0><<<sgrid, 256>>>(arena, nslots, work, stash, out); });
        float r1 = best_ms([&] { stream_slots<1><<<sgrid, 256>>>(arena, nslots, work, stash, out); });
        float r2 = best_ms([&] { stream_slots<2><<<sgrid, 256>>>(arena, nslots, work, stash, out); });
        float r3 = best_ms([&] { stream_work64<<<sgrid, 256>>>(arena, nslots, work, out); });
        float s2 = best_ms([&] { scatter2<<<grid, 256>>>(arena, work, nslots); });
        float sb = best_ms([&] { stash_to_block<<<grid, 256>>>(arena, stash, nslots); });
        float t1 = best_ms([&] {
            stream_slots<1><<<sgrid, 256>>>(arena, nslots, work, stash, out);
            scatter2<<<grid, 256>>>(arena, work, nslots);
        });
        float t2 = best_ms([&] {
            stream_slots<2><<<sgrid, 256>>>(arena, nslots, work, stash, out);
            stash_to_block<<<grid, 256>>>(arena, stash, nslots);
        });
        printf("{\"round\": %d, \"read\": %.4f, \"read_work\": %.4f, \"read_stash\": %.4f, \"scatter2\": %.4f, "
               "\"stash_block\": %.4f, \"two_phase_2B\": %.4f, \"two_phase_stash\": %.4f, \"read_work64\": %.4f}\n",
               round, r0, r1, r2, s2, sb, t1, t2, r3);
    }
    return 0;
}
