// read_probe.hip -- read-bandwidth ceiling probes (diagnostic, not product):
// is the 6.9 TB/s of read_stream_kernel the chip's read ceiling, or does
// another access shape read HBM faster?  Every variant reads the same 8 GiB
// once per launch and folds it into a checksum so nothing is elided.
//   gs<U,NT>     grid-stride, U 16 B loads per lane in flight (the product's
//                read_stream_kernel is gs<4,nt>)
//   wave<U,NT>   each wave reads U KiB contiguous per step (lane l loads
//                16 B at l*16 + u*1024), steps assigned round-robin to waves
//   tile<KB>     each workgroup owns a contiguous KB-KiB tile per step
//                (4 waves x 16 B x 64 lanes x KB/4 loads)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/read_probe tools/probes/read_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p)
{
    if (NT)
        return __builtin_nontemporal_load((const gu32x4 *)p);
    return *(const gu32x4 *)p;
}

__device__ __forceinline__ void fold(uint32_t acc, unsigned long long *out)
{
    for (int m = 32; m >= 1; m >>= 1)
        acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0 && acc == 0x12345678u)
        atomicAdd(out, 1ull);
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) gs(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + (U - 1) * nt < n16; i += U * nt) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            v[u] = ld<NT>(p + i + u * nt);
#pragma unroll
        for (int u = 0; u < U; u++)
            acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    fold(acc, out);
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) wave(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t nsteps = n16 / (64 * U);
    uint32_t acc = 0;
    for (uint64_t s = w0; s < nsteps; s += nwaves) {
        const u32x4 *q = p + s * 64 * U + lane;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            v[u] = ld<NT>(q + 64 * u);
#pragma unroll
        for (int u = 0; u < U; u++)
            acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    fold(acc, out);
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
        unsigned grid;
    };
    const V vs[] = {
        {"gs4_nt_g256k", gs<4, true>, 262144},   {"gs4_nt_g8k", gs<4, true>, 8192},
        {"gs8_nt_g8k", gs<8, true>, 8192},       {"gs8_nt_g4k", gs<8, true>, 4096},
        {"gs4_def_g8k", gs<4, false>, 8192},     {"gs16_nt_g2k", gs<16, true>, 2048},
        {"wave4_nt_g8k", wave<4, true>, 8192},   {"wave8_nt_g4k", wave<8, true>, 4096},
        {"wave8_nt_g2k", wave<8, true>, 2048},   {"wave16_nt_g2k", wave<16, true>, 2048},
        {"wave6_nt_g4k", wave<6, true>, 4096},   {"wave8_def_g4k", wave<8, false>, 4096},
    };
    const int R = 5, L = 10;
    double best[sizeof(vs) / sizeof(vs[0])] = {0};
    for (int r = 0; r < R; r++)
        for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); v++) {
            hipLaunchKernelGGL(vs[v].k, dim3(vs[v].grid), dim3(256), 0, 0, p, n16, out);   // warm
            (void)hipEventRecord(a, 0);
            for (int l = 0; l < L; l++)
                hipLaunchKernelGGL(vs[v].k, dim3(vs[v].grid), dim3(256), 0, 0, p, n16, out);
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
