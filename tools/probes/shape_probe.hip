// shape_probe.hip -- does the packet-stream kernel's load shape, by itself,
// cap its read rate?  (diagnostic, not product)  Every variant reads the
// same 8 GiB once per launch with 16 B loads (default policy; _nt: nontemporal), U per lane per
// step, waves stepping round-robin, and folds it so nothing is elided:
//   lc<U>   lane l loads chunks l*U .. l*U+U-1 of the wave's 64*U-chunk step
//           (the stream kernel's ownership: each instruction spans 64*16*U B)
//   co<U>   lane l loads chunks u*64 + l (each instruction reads 1 KiB
//           contiguous)
// Occupancy is capped by dynamic LDS per workgroup (the stream kernel is at
// 6 waves per SIMD), so "w6" = 6 workgroups of 4 waves per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/shape_probe tools/probes/shape_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

template <int U, bool LC, bool NT = false>
__global__ void __launch_bounds__(256) shape(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    extern __shared__ uint32_t pad[];
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t nsteps = n16 / (64 * U);
    uint32_t acc = 0;
    for (uint64_t s = w0; s < nsteps; s += nwaves) {
        const u32x4 *q = p + s * 64 * U;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
        {
            const gu32x4 *a = (const gu32x4 *)(q + (LC ? lane * U + u : u * 64 + lane));
            v[u] = NT ? __builtin_nontemporal_load(a) : *a;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    for (int m = 32; m >= 1; m >>= 1)
        acc += __shfl_xor(acc, m, 64);
    if (lane == 0 && acc == 0x12345678u) {
        pad[0] = acc;
        atomicAdd(out, (unsigned long long)pad[0]);
    }
}

int main()
{
    const uint64_t bytes = 8ull << 30, n16 = bytes / 16;
    u32x4 *p;
    unsigned long long *out;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess)
        return 1;
    (void)hipMemset(p, 0x5A, bytes);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct V {
        const char *name;
        void (*k)(const u32x4 *, uint64_t, unsigned long long *);
        unsigned wpe;          // waves per SIMD (LDS-capped); 0: uncapped
    };
    const V vs[] = {
        {"lc2_w8", shape<2, true>, 8},  {"co2_w8", shape<2, false>, 8}, {"lc3_w6", shape<3, true>, 6},
        {"co3_w6", shape<3, false>, 6}, {"lc3_w8", shape<3, true>, 8},  {"co3_w8", shape<3, false>, 8},
        {"lc4_w6", shape<4, true>, 6},  {"co4_w6", shape<4, false>, 6}, {"lc6_w4", shape<6, true>, 4},
        {"co6_w4", shape<6, false>, 4}, {"co8_w4", shape<8, false>, 4}, {"lc3_w4", shape<3, true>, 4},
        {"lc3_nt_w6", shape<3, true, true>, 6}, {"co3_nt_w6", shape<3, false, true>, 6},
        {"lc2_nt_w8", shape<2, true, true>, 8}, {"co2_nt_w8", shape<2, false, true>, 8},
        {"co4_nt_w6", shape<4, false, true>, 6}, {"co6_nt_w4", shape<6, false, true>, 4},
        {"co3_nt_w4", shape<3, false, true>, 4}, {"co2_nt_w6", shape<2, false, true>, 6},
    };
    const int R = 5, L = 10;
    const unsigned grid = 8192;
    double best[sizeof(vs) / sizeof(vs[0])] = {0};
    for (int r = 0; r < R; r++)
        for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); v++) {
            // LDS per workgroup so that wpe workgroups of 4 waves fit a CU (160 KiB)
            const size_t lds = vs[v].wpe ? (160u * 1024u) / vs[v].wpe - 1024 : 0;
            hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(256), lds, 0, p, n16, out);   // warm
            (void)hipEventRecord(a, 0);
            for (int l = 0; l < L; l++)
                hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(256), lds, 0, p, n16, out);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            const double tbs = bytes / (ms / L * 1e-3) / 1e12;
            if (tbs > best[v])
                best[v] = tbs;
        }
    printf("{");
    for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); v++)
        printf("%s\"%s\": %.3f", v ? ", " : "", vs[v].name, best[v]);
    printf("}\n");
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
