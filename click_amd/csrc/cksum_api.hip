// cksum_api.hip -- the C ABI (include/click_amd_cksum.h) over the gfx950
// kernels in cksum_kernels.hh.  Host side: argument checks, geometry
// selection (lanes per packet), launches on the context's stream.
#include "cksum_kernels.hh"
#include "frag_kernels.hh"
#include "../../include/click_amd_cksum.h"
#include "internal.hh"

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

struct clk_ctx {
    int device;
    hipStream_t own;
    hipStream_t cur;
    // speed-only tuning (clk_ctx_tune; never read from the environment):
    // every setting gives bit-identical results
    int max_blocks;      // grid cap
    int force_group;     // lanes per packet of the fixed-geometry kernels (0: by max_len)
    int set_mode;        // -1 auto; 0: Set kernels store the field; 1: two-phase
    int scatter_blocks;  // grid cap of field_scatter_kernel: fewer, longer-lived waves
                         // (C3 scatter 0.57 vs 0.67 ms at 16K vs 64K blocks)
    uint64_t stream_min; // len[] batches of >= stream_min packets run by the packet-stream kernel
    uint64_t frag_flat_min; // clk_ip_fragment: batches of >= this many packets use the flat payload pass
    int frag_chunks;        // ... in this many tile ranges, each range's flat pass overlapping the next one's plan
    int set_chunks;      // two-phase Set: packet ranges whose scatter overlaps the next range's compute
    int read_shape;      // clk_read_stream's load shape (CLK_TUNE_READ_SHAPE)
    hipStream_t side;    // the scatters' stream (created on first use)
    hipEvent_t ev_pass, ev_side;
    void *scratch;       // two-phase work array (grown on demand)
    size_t scratch_bytes;
    uint32_t *dev_flags;   // device word kernels report internal faults in (fragmenter look-back timeout)
    bool check_flags;      // a launch since the last clk_ctx_sync may have set dev_flags
    char err[512];
};

namespace {

thread_local char tls_err[512];

int fail(clk_ctx *ctx, int code, const char *fmt, ...)
{
    char *buf = ctx ? ctx->err : tls_err;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, 512, fmt, ap);
    va_end(ap);
    return code;
}

int hip_fail(clk_ctx *ctx, hipError_t e, const char *what)
{
    return fail(ctx, CLK_EHIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

int enter(clk_ctx *ctx)
{
    if (!ctx)
        return fail(nullptr, CLK_EINVAL, "null context");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess)
        return hip_fail(ctx, e, "hipSetDevice");
    return CLK_SUCCESS;
}

int check_launch(clk_ctx *ctx, const char *what)
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(ctx, e, what);
    return CLK_SUCCESS;
}

// Device scratch for the two-phase Set (one u32 per packet).  Grown with a
// synchronous hipMalloc the first time a larger batch arrives; steady-state
// calls allocate nothing.
int ensure_scratch(clk_ctx *ctx, size_t bytes)
{
    if (ctx->scratch_bytes >= bytes)
        return CLK_SUCCESS;
    if (ctx->scratch) {
        hipError_t e = hipStreamSynchronize(ctx->cur);
        if (e != hipSuccess)
            return hip_fail(ctx, e, "hipStreamSynchronize");
        (void)hipFree(ctx->scratch);
        ctx->scratch = nullptr;
        ctx->scratch_bytes = 0;
    }
    hipError_t e = hipMalloc(&ctx->scratch, bytes);
    if (e != hipSuccess)
        return hip_fail(ctx, e, "hipMalloc(scratch)");
    ctx->scratch_bytes = bytes;
    return CLK_SUCCESS;
}

// The side stream and events of the chunked two-phase Set (first use).
int ensure_side(clk_ctx *ctx)
{
    hipError_t e = hipSuccess;
    if (!ctx->side && (e = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(ctx, e, "hipStreamCreateWithFlags(side)");
    for (hipEvent_t *ev : {&ctx->ev_pass, &ctx->ev_side})
        if (!*ev && (e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(ctx, e, "hipEventCreateWithFlags");
    return CLK_SUCCESS;
}

int check_batch(clk_ctx *ctx, const clk_batch *b, const char *fn)
{
    if (!b)
        return fail(ctx, CLK_EINVAL, "%s: null batch", fn);
    if (b->n && !b->base)
        return fail(ctx, CLK_EINVAL, "%s: null batch base", fn);
    if (b->n && !b->off && b->stride == 0 && b->n > 1)
        return fail(ctx, CLK_EINVAL, "%s: off == NULL needs a nonzero stride", fn);
    return CLK_SUCCESS;
}

clk::BatchArgs args_of(const clk_batch *b)
{
    clk::BatchArgs a;
    a.base = b->base;
    a.off = b->off;
    a.stride = b->stride;
    a.len = b->len;
    a.fixed_len = b->fixed_len;
    a.n = b->n;
    return a;
}

// packets [i0, i0 + m) of a batch
clk::BatchArgs sub_args(const clk_batch *b, uint64_t i0, uint64_t m)
{
    clk::BatchArgs a = args_of(b);
    if (a.off)
        a.off += i0;
    else
        a.base += i0 * a.stride;
    if (a.len)
        a.len += i0;
    a.n = m;
    return a;
}

constexpr int BLOCK = 256;
#ifndef CLK_K
#define CLK_K 8
#endif
constexpr int K = CLK_K;   // 16-byte chunk loads in flight per lane per pass
#ifndef CLK_K16
#define CLK_K16 6          // ... for 16 lanes per packet: 96 chunks cover a 1500 B packet (C3 Check -1.9 %)
#endif
// l4_kernel's loads per lane and pass at G lanes per packet.  pick_group
// sizes G by K; a G = 16 packet past 16 * CLK_K16 chunks takes two passes.
constexpr int k_for(int G) { return G == 16 ? CLK_K16 : K; }
#ifndef CLK_SKV
#define CLK_SKV 4          // chunks per lane per pass of the packet-stream kernel (Set; dense path: 3 / 5 chunks 5.18 / 5.11 vs 5.08 ms)
#endif
#ifndef CLK_SKV_CHECK
#define CLK_SKV_CHECK 4    // ... Check, at CLK_SWPE_CHECK waves per SIMD (C4 Check 3.74 vs 3.89 ms with 3 at 6)
#endif

// Lanes per packet: the fewest (of 1, 4, 16, 64) whose K-deep pass covers
// the largest packet in one pass; 64 beyond that (multi-pass).
int pick_group(const clk_ctx *ctx, const clk_batch *b)
{
    if (ctx->force_group)
        return ctx->force_group;
    uint32_t ml = b->len ? b->max_len : b->fixed_len;
    if (b->len && ml == 0)
        return 16;
    const uint64_t nch = (uint64_t)ml / 16 + 2;
    if (nch <= (uint64_t)K * 1) return 1;
    if (nch <= (uint64_t)K * 4) return 4;
    if (nch <= (uint64_t)K * 16) return 16;
    return 64;
}

unsigned grid_for(const clk_ctx *ctx, uint64_t threads)
{
    uint64_t g = (threads + BLOCK - 1) / BLOCK;
    if (g > (uint64_t)ctx->max_blocks)
        g = (uint64_t)ctx->max_blocks;
    return g ? (unsigned)g : 1u;
}

// Scratch for n packets: the two-phase Set's work words (u32 x n).
size_t work_bytes(uint64_t n) { return (n * 4 + 255) & ~size_t(255); }

// The packet-stream kernel keeps a run's chunk counts in 32 bits and a
// packet's in 27: it takes packets of known length up to 16 MiB.
bool use_stream(const clk_ctx *ctx, const clk_batch *b)
{
    return b->len && !ctx->force_group && b->n >= ctx->stream_min && b->max_len && b->max_len <= clk::STREAM_MAX_LEN;
}

template <int G>
void launch_range(clk_ctx *ctx, const clk::BatchArgs &a, unsigned grid, uint16_t *out)
{
    if (CLK_L4_RUNS)                 // runs per workgroup, as l4_kernel
        hipLaunchKernelGGL((clk::range_kernel<G, k_for(G), true>), dim3(grid), dim3(BLOCK), 0, ctx->cur, a, out);
    else
        hipLaunchKernelGGL((clk::range_kernel<G, k_for(G), false>), dim3(grid), dim3(BLOCK), 0, ctx->cur, a, out);
}

void launch_range_dispatch(clk_ctx *ctx, const clk::BatchArgs &a, unsigned grid, uint16_t *out, int g)
{
    switch (g) {
    case 1: launch_range<1>(ctx, a, grid, out); break;
    case 2: launch_range<2>(ctx, a, grid, out); break;
    case 4: launch_range<4>(ctx, a, grid, out); break;
    case 8: launch_range<8>(ctx, a, grid, out); break;
    case 16: launch_range<16>(ctx, a, grid, out); break;
    case 32: launch_range<32>(ctx, a, grid, out); break;
    default: launch_range<64>(ctx, a, grid, out); break;
    }
}

template <int PROTO, bool SET, int G>
void launch_l4_g(clk_ctx *ctx, const clk::BatchArgs &a, unsigned grid, int fixoff, uint8_t *code, uint16_t *sum,
                 uint32_t *work)
{
    // runs per workgroup (CLK_L4_RUNS) for Check and for Sets from
    // CLK_L4_RUNS_SET_G lanes per packet, else the grid-stride group loop
    constexpr bool RUNS = CLK_L4_RUNS && (!SET || G >= CLK_L4_RUNS_SET_G);
    if (SET && work)
        hipLaunchKernelGGL((clk::l4_kernel<PROTO, SET, G, k_for(G), true, RUNS>), dim3(grid), dim3(BLOCK), 0, ctx->cur, a,
                           fixoff, code, sum, work);
    else
        hipLaunchKernelGGL((clk::l4_kernel<PROTO, SET, G, k_for(G), false, RUNS>), dim3(grid), dim3(BLOCK), 0, ctx->cur, a,
                           fixoff, code, sum, work);
}

template <int PROTO, bool SET>
int launch_l4_dispatch(clk_ctx *ctx, const clk::BatchArgs &a, unsigned grid, int fixoff, uint8_t *code,
                       uint16_t *sum, uint32_t *work, int g)
{
    switch (g) {
    case 1: launch_l4_g<PROTO, SET, 1>(ctx, a, grid, fixoff, code, sum, work); break;
    case 2: launch_l4_g<PROTO, SET, 2>(ctx, a, grid, fixoff, code, sum, work); break;
    case 4: launch_l4_g<PROTO, SET, 4>(ctx, a, grid, fixoff, code, sum, work); break;
    case 8: launch_l4_g<PROTO, SET, 8>(ctx, a, grid, fixoff, code, sum, work); break;
    case 16: launch_l4_g<PROTO, SET, 16>(ctx, a, grid, fixoff, code, sum, work); break;
    case 32: launch_l4_g<PROTO, SET, 32>(ctx, a, grid, fixoff, code, sum, work); break;
    default: launch_l4_g<PROTO, SET, 64>(ctx, a, grid, fixoff, code, sum, work); break;
    }
    return 0;
}

template <int PROTO, bool SET>
int launch_l4(clk_ctx *ctx, const clk_batch *b, int fixoff, uint8_t *code, uint16_t *sum, const char *fn)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, fn))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    if (!code) return fail(ctx, CLK_EINVAL, "%s: null output", fn);
    uint32_t *work = nullptr;
    const bool stream = use_stream(ctx, b);
    // auto (-1): two-phase for the fixed-geometry Set kernels (a read-only
    // compute pass, then field_scatter_kernel), fused for the packet-stream
    // kernel (phase C stores the field's 64 B block from its LDS stash);
    // DESIGN.md §6
    const bool two = SET && (ctx->set_mode == 1 || (ctx->set_mode < 0 && !stream));
    if (two) {
        if ((r = ensure_scratch(ctx, work_bytes(b->n)))) return r;
        work = (uint32_t *)ctx->scratch;
    }
    if (stream) {
        constexpr int KV = SET ? CLK_SKV : CLK_SKV_CHECK;
        uint64_t blocks = (b->n + 255) / 256;            // 4 waves x 64 packets per block
        if (blocks > (uint64_t)ctx->max_blocks)
            blocks = (uint64_t)ctx->max_blocks;
        if (work)
            hipLaunchKernelGGL((clk::l4_stream_kernel<PROTO, SET, true, KV>), dim3((unsigned)blocks), dim3(BLOCK), 0,
                               ctx->cur, args_of(b), fixoff, code, sum, work);
        else
            hipLaunchKernelGGL((clk::l4_stream_kernel<PROTO, SET, false, KV>), dim3((unsigned)blocks), dim3(BLOCK), 0,
                               ctx->cur, args_of(b), fixoff, code, sum, work);
    } else {
        const int g = pick_group(ctx, b);
        auto compute = [&](const clk::BatchArgs &a, uint8_t *c_, uint16_t *s_, uint32_t *w_) {
            uint64_t threads = a.n * (uint64_t)g;
            if (CLK_L4_RUNS && (!SET || g >= CLK_L4_RUNS_SET_G)) {   // a workgroup per run
                const uint64_t run = 256 / g < 64 ? 64 : 256 / g;    // as l4_kernel's RB
                threads = (a.n + run - 1) / run * BLOCK;
            }
            launch_l4_dispatch<PROTO, SET>(ctx, a, grid_for(ctx, threads), fixoff, c_, s_, w_, g);
        };
        const uint64_t per = work && ctx->set_chunks > 1
                                 ? (((b->n + ctx->set_chunks - 1) / ctx->set_chunks + 255) & ~uint64_t(255))
                                 : b->n;
        if (per < b->n) {
            // the two-phase Set in packet ranges: each range's scatter (2 B
            // writes, read-modify-write bound) runs on the side stream while
            // the next range's compute pass (read bound) runs on this one
            if ((r = ensure_side(ctx))) return r;
            constexpr int FIELD = PROTO == clk::UDP ? 6 : 16;
            for (uint64_t i0 = 0; i0 < b->n; i0 += per) {
                const clk::BatchArgs a = sub_args(b, i0, std::min(per, b->n - i0));
                compute(a, code + i0, sum ? sum + i0 : nullptr, work + i0);
                (void)hipEventRecord(ctx->ev_pass, ctx->cur);
                (void)hipStreamWaitEvent(ctx->side, ctx->ev_pass, 0);
                hipLaunchKernelGGL((clk::field_scatter_kernel<FIELD>),
                                   dim3(std::min<unsigned>(grid_for(ctx, a.n), (unsigned)ctx->scatter_blocks)),
                                   dim3(BLOCK), 0, ctx->side, a, (const uint32_t *)(work + i0), code + i0,
                                   sum ? sum + i0 : nullptr);
            }
            (void)hipEventRecord(ctx->ev_side, ctx->side);
            (void)hipStreamWaitEvent(ctx->cur, ctx->ev_side, 0);
            return check_launch(ctx, fn);
        }
        compute(args_of(b), code, sum, work);
    }
    if (work) {
        constexpr int FIELD = PROTO == clk::UDP ? 6 : 16;
        hipLaunchKernelGGL((clk::field_scatter_kernel<FIELD>),
                           dim3(std::min<unsigned>(grid_for(ctx, b->n), (unsigned)ctx->scatter_blocks)), dim3(BLOCK), 0,
                           ctx->cur, args_of(b), (const uint32_t *)work, code, sum);
    }
    return check_launch(ctx, fn);
}

bool is_gfx950(int device)
{
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess)
        return false;
    return std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

} // namespace

extern "C" {

int clk_abi_version(void) { return CLK_ABI_VERSION; }

int clk_device_count(void)
{
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e == hipErrorNoDevice)
        return 0;
    if (e != hipSuccess)
        return hip_fail(nullptr, e, "hipGetDeviceCount");
    int n = 0;
    for (int d = 0; d < ndev; d++)
        n += is_gfx950(d) ? 1 : 0;
    return n;
}

int clk_ctx_create(int device, clk_ctx **out)
{
    if (!out)
        return fail(nullptr, CLK_EINVAL, "clk_ctx_create: null out");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess)
        return hip_fail(nullptr, e, "hipGetDeviceCount");
    if (device < 0 || device >= ndev)
        return fail(nullptr, CLK_ENODEV, "clk_ctx_create: device %d of %d", device, ndev);
    if (!is_gfx950(device))
        return fail(nullptr, CLK_ENODEV, "clk_ctx_create: device %d is not gfx950", device);
    e = hipSetDevice(device);
    if (e != hipSuccess)
        return hip_fail(nullptr, e, "hipSetDevice");
    clk_ctx *c = new (std::nothrow) clk_ctx;
    if (!c)
        return fail(nullptr, CLK_EINVAL, "clk_ctx_create: out of memory");
    c->device = device;
    c->err[0] = 0;
    c->max_blocks = 262144;
    c->scratch = nullptr;
    c->scratch_bytes = 0;
    c->set_mode = -1;
    c->set_chunks = 1;
    c->read_shape = 0;
    c->side = nullptr;
    c->ev_pass = c->ev_side = nullptr;
    c->scatter_blocks = 16384;
    c->stream_min = 65536;
    c->frag_flat_min = 8192;
    c->frag_chunks = 1;
    c->force_group = 0;
    e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(nullptr, e, "hipStreamCreateWithFlags");
    }
    c->cur = c->own;
    c->check_flags = false;
    c->dev_flags = nullptr;
    if ((e = hipMalloc(&c->dev_flags, 256)) != hipSuccess || (e = hipMemset(c->dev_flags, 0, 256)) != hipSuccess) {
        (void)hipStreamDestroy(c->own);
        delete c;
        return hip_fail(nullptr, e, "hipMalloc");
    }
    *out = c;
    return CLK_SUCCESS;
}

int clk_ctx_destroy(clk_ctx *ctx)
{
    if (!ctx)
        return CLK_SUCCESS;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->cur);
    (void)hipStreamDestroy(ctx->own);
    if (ctx->side) {
        (void)hipStreamSynchronize(ctx->side);
        (void)hipStreamDestroy(ctx->side);
    }
    for (hipEvent_t e : {ctx->ev_pass, ctx->ev_side})
        if (e)
            (void)hipEventDestroy(e);
    if (ctx->scratch)
        (void)hipFree(ctx->scratch);
    if (ctx->dev_flags)
        (void)hipFree(ctx->dev_flags);
    delete ctx;
    return CLK_SUCCESS;
}

int clk_ctx_set_stream(clk_ctx *ctx, void *hip_stream)
{
    if (!ctx)
        return fail(nullptr, CLK_EINVAL, "null context");
    ctx->cur = (hipStream_t)hip_stream;
    return CLK_SUCCESS;
}

void *clk_ctx_stream(clk_ctx *ctx) { return ctx ? (void *)ctx->cur : nullptr; }
void *clk_ctx_own_stream(clk_ctx *ctx) { return ctx ? (void *)ctx->own : nullptr; }
int clk_ctx_device(clk_ctx *ctx) { return ctx ? ctx->device : -1; }

int clk_ctx_reserve(clk_ctx *ctx, uint64_t max_packets)
{
    int r = enter(ctx);
    if (r) return r;
    return ensure_scratch(ctx, work_bytes(max_packets));
}

int clk_ctx_tune(clk_ctx *ctx, int knob, int64_t value)
{
    if (!ctx)
        return fail(nullptr, CLK_EINVAL, "null context");
    switch (knob) {
    case CLK_TUNE_MAX_BLOCKS:
        if (value < 1 || value > (1 << 30)) break;
        ctx->max_blocks = (int)value;
        return CLK_SUCCESS;
    case CLK_TUNE_SCATTER_BLOCKS:
        if (value < 1 || value > (1 << 30)) break;
        ctx->scatter_blocks = (int)value;
        return CLK_SUCCESS;
    case CLK_TUNE_SET_MODE:
        if (value < -1 || value > 1) break;
        ctx->set_mode = (int)value;
        return CLK_SUCCESS;
    case CLK_TUNE_STREAM_MIN:
        if (value < 1) break;
        ctx->stream_min = (uint64_t)value;
        return CLK_SUCCESS;
    case CLK_TUNE_SET_CHUNKS:
        if (value < 1 || value > 64) break;
        ctx->set_chunks = (int)value;
        return CLK_SUCCESS;
    case CLK_TUNE_READ_SHAPE:
        if (value < 0 || value > 5) break;
        ctx->read_shape = (int)value;
        return CLK_SUCCESS;
    case CLK_TUNE_FRAG_FLAT_MIN:
        if (value < 0) break;
        ctx->frag_flat_min = (uint64_t)value;
        return CLK_SUCCESS;
    case CLK_TUNE_FRAG_CHUNKS:
        if (value < 1 || value > 64) break;
        ctx->frag_chunks = (int)value;
        return CLK_SUCCESS;
    case CLK_TUNE_GROUP:
        if (!(value == 0 || value == 1 || value == 2 || value == 4 || value == 8 || value == 16 || value == 32 ||
              value == 64)) break;
        ctx->force_group = (int)value;
        return CLK_SUCCESS;
    default:
        return fail(ctx, CLK_EINVAL, "clk_ctx_tune: unknown knob %d", knob);
    }
    return fail(ctx, CLK_EINVAL, "clk_ctx_tune: knob %d: bad value %lld", knob, (long long)value);
}

int clk_ctx_sync(clk_ctx *ctx)
{
    int r = enter(ctx);
    if (r) return r;
    hipError_t e = hipStreamSynchronize(ctx->cur);
    if (e != hipSuccess)
        return hip_fail(ctx, e, "hipStreamSynchronize");
    if (ctx->check_flags) {              // a kernel's internal fault report (see dev_flags)
        ctx->check_flags = false;
        uint32_t f = 0;
        if ((e = hipMemcpy(&f, ctx->dev_flags, 4, hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(ctx, e, "hipMemcpy");
        if (f) {
            (void)hipMemset(ctx->dev_flags, 0, 4);
            return fail(ctx, CLK_EHIP, "clk_ip_fragment: the tile look-back timed out (internal error; "
                                       "fragment offsets of that call are wrong)");
        }
    }
    return CLK_SUCCESS;
}

const char *clk_last_error(clk_ctx *ctx) { return ctx ? ctx->err : tls_err; }

int clk_ctx_set_error_internal(clk_ctx *ctx, const char *msg)
{
    return fail(ctx, CLK_EINVAL, "%s", msg);
}

int clk_in_cksum(clk_ctx *ctx, const clk_batch *b, uint16_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_in_cksum"))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    if (!out_sum) return fail(ctx, CLK_EINVAL, "clk_in_cksum: null output");
    const int g = pick_group(ctx, b);
    uint64_t threads = b->n * (uint64_t)g;
    if (CLK_L4_RUNS) {                                        // a workgroup per run
        const uint64_t run = 256 / g < 64 ? 64 : 256 / g;
        threads = (b->n + run - 1) / run * BLOCK;
    }
    launch_range_dispatch(ctx, args_of(b), grid_for(ctx, threads), out_sum, g);
    return check_launch(ctx, "clk_in_cksum");
}

int clk_check_ip_header(clk_ctx *ctx, const clk_batch *b, const clk_ip_check_cfg *cfg, uint8_t *out_verdict)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_check_ip_header"))) return r;
    if (!cfg) return fail(ctx, CLK_EINVAL, "clk_check_ip_header: null cfg");
    if ((cfg->nbadsrc && !cfg->badsrc) || (cfg->ngooddst && !cfg->gooddst))
        return fail(ctx, CLK_EINVAL, "clk_check_ip_header: null address list");
    if (b->n == 0) return CLK_SUCCESS;
    if (!out_verdict) return fail(ctx, CLK_EINVAL, "clk_check_ip_header: null output");
    const unsigned grid = grid_for(ctx, (CLK_IPH_PAIR ? 2 : 1) * b->n);
    if (cfg->checksum)
        hipLaunchKernelGGL((clk::ip_header_kernel<clk::IP_CHECK>), dim3(grid), dim3(BLOCK), 0, ctx->cur,
                           args_of(b), cfg->offset, cfg->badsrc, cfg->nbadsrc, cfg->gooddst, cfg->ngooddst,
                           out_verdict, (uint16_t *)nullptr);
    else
        hipLaunchKernelGGL((clk::ip_header_kernel<clk::IP_CHECK_NOCKSUM>), dim3(grid), dim3(BLOCK), 0, ctx->cur,
                           args_of(b), cfg->offset, cfg->badsrc, cfg->nbadsrc, cfg->gooddst, cfg->ngooddst,
                           out_verdict, (uint16_t *)nullptr);
    return check_launch(ctx, "clk_check_ip_header");
}

int clk_set_ip_checksum(clk_ctx *ctx, const clk_batch *b, uint8_t *out_status, uint16_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_set_ip_checksum"))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    if (!out_status) return fail(ctx, CLK_EINVAL, "clk_set_ip_checksum: null output");
    hipLaunchKernelGGL((clk::ip_header_kernel<clk::IP_SET>), dim3(grid_for(ctx, b->n)), dim3(BLOCK), 0, ctx->cur,
                       args_of(b), 0u, (const uint32_t *)nullptr, 0u, (const uint32_t *)nullptr, 0u, out_status,
                       out_sum);
    return check_launch(ctx, "clk_set_ip_checksum");
}

int clk_check_udp_header(clk_ctx *ctx, const clk_batch *b, uint8_t *out_verdict)
{
    return launch_l4<clk::UDP, false>(ctx, b, 0, out_verdict, nullptr, "clk_check_udp_header");
}

int clk_set_udp_checksum(clk_ctx *ctx, const clk_batch *b, uint8_t *out_status, uint16_t *out_sum)
{
    return launch_l4<clk::UDP, true>(ctx, b, 0, out_status, out_sum, "clk_set_udp_checksum");
}

int clk_check_tcp_header(clk_ctx *ctx, const clk_batch *b, uint8_t *out_verdict)
{
    return launch_l4<clk::TCP, false>(ctx, b, 0, out_verdict, nullptr, "clk_check_tcp_header");
}

int clk_set_tcp_checksum(clk_ctx *ctx, const clk_batch *b, int fixoff, uint8_t *out_status, uint16_t *out_sum)
{
    return launch_l4<clk::TCP, true>(ctx, b, fixoff ? 1 : 0, out_status, out_sum, "clk_set_tcp_checksum");
}

int clk_check_icmp_header(clk_ctx *ctx, const clk_batch *b, uint8_t *out_verdict)
{
    return launch_l4<clk::ICMP, false>(ctx, b, 0, out_verdict, nullptr, "clk_check_icmp_header");
}

int clk_dec_ip_ttl(clk_ctx *ctx, const clk_batch *b, int multicast, uint8_t *out_status, uint16_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_dec_ip_ttl"))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    if (!out_status) return fail(ctx, CLK_EINVAL, "clk_dec_ip_ttl: null output");
    hipLaunchKernelGGL(clk::dec_ttl_kernel, dim3(grid_for(ctx, b->n)), dim3(BLOCK), 0, ctx->cur, args_of(b),
                       multicast ? 1 : 0, out_status, out_sum);
    return check_launch(ctx, "clk_dec_ip_ttl");
}

int clk_update_in_cksum(clk_ctx *ctx, const clk_batch *b, const clk_cksum_update_cfg *cfg, const uint16_t *new_hw,
                        uint8_t *out_status, uint16_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_update_in_cksum"))) return r;
    if (!cfg) return fail(ctx, CLK_EINVAL, "clk_update_in_cksum: null cfg");
    if (b->n == 0) return CLK_SUCCESS;
    if (!new_hw) return fail(ctx, CLK_EINVAL, "clk_update_in_cksum: null new_hw");
    clk::UpdateArgs u{cfg->sum_off, cfg->hw_off, cfg->zero_lo, cfg->zero_fix ? 1 : 0, 1};
    hipLaunchKernelGGL(clk::update_kernel, dim3(grid_for(ctx, b->n)), dim3(BLOCK), 0, ctx->cur, args_of(b), u,
                       new_hw, out_status, out_sum);
    return check_launch(ctx, "clk_update_in_cksum");
}

int clk_update_zero_in_cksum(clk_ctx *ctx, const clk_batch *b, uint32_t sum_off, uint32_t zero_lo,
                             uint8_t *out_status, uint16_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_update_zero_in_cksum"))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    clk::UpdateArgs u{sum_off, 0, zero_lo, 1, 0};
    hipLaunchKernelGGL(clk::update_kernel, dim3(grid_for(ctx, b->n)), dim3(BLOCK), 0, ctx->cur, args_of(b), u,
                       (const uint16_t *)nullptr, out_status, out_sum);
    return check_launch(ctx, "clk_update_zero_in_cksum");
}

}   // extern "C"

namespace {
template <int MODE>
int launch_ip_out(clk_ctx *ctx, const clk_batch *b, const clk_ip_out_cfg *cfg, const uint8_t *flags,
                  uint8_t *code, uint8_t *problem, uint16_t *sum, const char *fn)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, fn))) return r;
    if (!cfg) return fail(ctx, CLK_EINVAL, "%s: null cfg", fn);
    if (cfg->n_my_addrs && !cfg->my_addrs) return fail(ctx, CLK_EINVAL, "%s: null address list", fn);
    if (b->n == 0) return CLK_SUCCESS;
    uint8_t *c = code;
    if (!c) {                                   // FixIPSrc has no per-packet outcome
        if ((r = ensure_scratch(ctx, b->n))) return r;
        c = (uint8_t *)ctx->scratch;
    }
    clk::IpOutArgs a;
    a.my_ip = cfg->my_ip;
    a.ts = cfg->ts;
    a.n_my_addrs = cfg->n_my_addrs;
    a.mtu = cfg->mtu;
    a.my_addrs = cfg->my_addrs;
    a.flags = flags;
    hipLaunchKernelGGL((clk::ip_out_kernel<MODE>), dim3(grid_for(ctx, b->n)), dim3(BLOCK), 0, ctx->cur, args_of(b),
                       a, c, problem, sum);
    return check_launch(ctx, fn);
}
}   // namespace

extern "C" {

int clk_ip_gw_options(clk_ctx *ctx, const clk_batch *b, const clk_ip_out_cfg *cfg, uint8_t *out_status,
                      uint8_t *out_problem, uint16_t *out_sum)
{
    if (b && b->n && !out_status)
        return fail(ctx, CLK_EINVAL, "clk_ip_gw_options: null output");
    return launch_ip_out<clk::OUT_GWOPT>(ctx, b, cfg, nullptr, out_status, out_problem, out_sum,
                                         "clk_ip_gw_options");
}

int clk_fix_ip_src(clk_ctx *ctx, const clk_batch *b, const clk_ip_out_cfg *cfg, const uint8_t *anno,
                   uint16_t *out_sum)
{
    return launch_ip_out<clk::OUT_FIXSRC>(ctx, b, cfg, anno, nullptr, nullptr, out_sum, "clk_fix_ip_src");
}

int clk_ip_output_combo(clk_ctx *ctx, const clk_batch *b, const clk_ip_out_cfg *cfg, const uint8_t *flags,
                        uint8_t *out_port, uint8_t *out_problem, uint16_t *out_sum)
{
    if (b && b->n && !out_port)
        return fail(ctx, CLK_EINVAL, "clk_ip_output_combo: null output");
    return launch_ip_out<clk::OUT_COMBO>(ctx, b, cfg, flags, out_port, out_problem, out_sum,
                                         "clk_ip_output_combo");
}

int clk_ip_fragment(clk_ctx *ctx, const clk_batch *b, const clk_frag_cfg *cfg, uint8_t *out_port,
                    uint32_t *out_first_len, uint64_t *out_frag_first, const clk_frag_out *out, uint64_t *totals)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_ip_fragment"))) return r;
    if (!cfg || !out || !totals)
        return fail(ctx, CLK_EINVAL, "clk_ip_fragment: null cfg, out or totals");
    if (cfg->mtu < 8)
        return fail(ctx, CLK_EINVAL, "clk_ip_fragment: MTU must be at least 8");   // ipfragmenter.cc:51-52
    if ((out->max_frags && (!out->frag_off || !out->frag_len || !out->frag_src)) ||
        (out->arena_bytes && !out->arena))
        return fail(ctx, CLK_EINVAL, "clk_ip_fragment: null fragment buffers");
    if (b->n >= (1ull << 32))
        return fail(ctx, CLK_EINVAL, "clk_ip_fragment: batch too large");
    hipError_t e;
    if (b->n == 0) {
        e = hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), ctx->cur);
        return e == hipSuccess ? CLK_SUCCESS : hip_fail(ctx, e, "hipMemsetAsync");
    }
    if (!out_port || !out_first_len)
        return fail(ctx, CLK_EINVAL, "clk_ip_fragment: null output");
    const uint32_t ntiles = (uint32_t)((b->n + clk::FRAG_TILE - 1) / clk::FRAG_TILE);
    // single pass (plan + look-back scan + write) when the fragments are written
    const bool fused = out->arena && CLK_FRAG_FUSED;
    // scratch, two-pass: [nextra u32 x n][bytes u32 x n][tile sums u64 x 2 x ntiles]
    //          single pass: [ticket, err u32 | 256 B][tagged words u64 x 2 x ntiles]
    //          then [frag_first u64 x n] if the caller gives none
    const size_t pl = (b->n * 4 + 255) & ~size_t(255);
    const size_t tb = (((size_t)ntiles * 16 + 255) & ~size_t(255));
    const size_t ts_end = fused ? 256 + tb : 2 * pl + tb;
    // FLAT: the fragments of plain-header packets written by frag_flat_kernel,
    // from one 16 B record per fragment, [FragFlat x max_frags] at fx_at
    const bool flat = fused && CLK_FRAG_FLAT && b->n >= ctx->frag_flat_min && out->max_frags &&
                      out->max_frags <= (1ull << 32);
    const size_t fx_at = (ts_end + (out_frag_first ? 0 : b->n * 8) + 255) & ~size_t(255);
    if ((r = ensure_scratch(ctx, flat ? fx_at + out->max_frags * sizeof(clk::FragFlat)
                                      : ts_end + (out_frag_first ? 0 : b->n * 8)))) return r;
    uint8_t *sc = (uint8_t *)ctx->scratch;
    uint32_t *pl_n = (uint32_t *)sc, *pl_b = (uint32_t *)(sc + pl);
    uint64_t *tile_sums = (uint64_t *)(sc + 2 * pl);
    uint64_t *ffirst = out_frag_first ? out_frag_first : (uint64_t *)(sc + ts_end);
    clk::FragArgs f;
    f.mtu = cfg->mtu;
    f.honor_df = cfg->honor_df ? 1 : 0;
    f.new_id = cfg->new_id;
    f.arena = out->arena;
    f.arena_bytes = out->arena ? out->arena_bytes : 0;
    f.frag_off = out->frag_off;
    f.frag_len = out->frag_len;
    f.frag_src = out->frag_src;
    f.max_frags = out->frag_off ? out->max_frags : 0;
    f.fx = flat ? (clk::FragFlat *)(sc + fx_at) : nullptr;
    if (fused) {
        clk::FragLookback lb;
        lb.ticket = (uint32_t *)sc;
        lb.err = ctx->dev_flags;
        ctx->check_flags = true;
        lb.word = (uint64_t *)(sc + 256);
        lb.totals = totals;
        lb.out_port = out_port;
        lb.out_first_len = out_first_len;
        lb.ntiles = ntiles;
        e = hipMemsetAsync(sc, 0, 256 + (size_t)ntiles * 16, ctx->cur);
        if (e != hipSuccess)
            return hip_fail(ctx, e, "hipMemsetAsync");
        if (!flat) {
            hipLaunchKernelGGL((clk::frag_write_kernel<true, false>), dim3(ntiles), dim3(BLOCK), 0, ctx->cur,
                               args_of(b), f, (const uint8_t *)nullptr, (const uint32_t *)nullptr,
                               (const uint32_t *)nullptr, (const uint64_t *)nullptr, ffirst, lb);
            return check_launch(ctx, "clk_ip_fragment");
        }
        // blocks of the flat pass for `frags` records: 4 waves of FLAT_F each
        auto flat_blocks = [](uint64_t frags) {
            const uint64_t nb = ((frags + clk::FLAT_F - 1) / clk::FLAT_F + 3) / 4;
            return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nb, 1u << 30));   // the kernel strides past it
        };
        const uint32_t nch = (uint32_t)std::min<uint64_t>(ctx->frag_chunks, ntiles / 2);
        if (nch <= 1) {
            hipLaunchKernelGGL((clk::frag_write_kernel<true, true>), dim3(ntiles), dim3(BLOCK), 0, ctx->cur,
                               args_of(b), f, (const uint8_t *)nullptr, (const uint32_t *)nullptr,
                               (const uint32_t *)nullptr, (const uint64_t *)nullptr, ffirst, lb);
            hipLaunchKernelGGL(clk::frag_flat_kernel, dim3(flat_blocks(out->max_frags)), dim3(BLOCK), 0, ctx->cur,
                               args_of(b), f, (const uint64_t *)nullptr, (const uint64_t *)totals);
            return check_launch(ctx, "clk_ip_fragment");
        }
        // in tile ranges: range c's plan on this stream (its tiles take the
        // next tickets and look back into the ranges before it), then its
        // flat pass on the side stream, over the fragments between the
        // inclusive prefixes of the tiles before and at its end, while range
        // c + 1's plan runs here
        if ((r = ensure_side(ctx))) return r;
        const uint32_t per = (ntiles + nch - 1) / nch;
        for (uint32_t t0 = 0; t0 < ntiles; t0 += per) {
            const uint32_t t1 = std::min(ntiles, t0 + per);
            hipLaunchKernelGGL((clk::frag_write_kernel<true, true>), dim3(t1 - t0), dim3(BLOCK), 0, ctx->cur,
                               args_of(b), f, (const uint8_t *)nullptr, (const uint32_t *)nullptr,
                               (const uint32_t *)nullptr, (const uint64_t *)nullptr, ffirst, lb);
            (void)hipEventRecord(ctx->ev_pass, ctx->cur);
            (void)hipStreamWaitEvent(ctx->side, ctx->ev_pass, 0);
            const uint64_t est = (out->max_frags * (t1 - t0) + ntiles - 1) / ntiles;
            hipLaunchKernelGGL(clk::frag_flat_kernel, dim3(flat_blocks(est)), dim3(BLOCK), 0, ctx->side, args_of(b), f,
                               t0 ? (const uint64_t *)(lb.word + 2 * (t0 - 1)) : (const uint64_t *)nullptr,
                               t1 < ntiles ? (const uint64_t *)(lb.word + 2 * (t1 - 1)) : (const uint64_t *)totals);
        }
        (void)hipEventRecord(ctx->ev_side, ctx->side);
        (void)hipStreamWaitEvent(ctx->cur, ctx->ev_side, 0);
        return check_launch(ctx, "clk_ip_fragment");
    }
    hipLaunchKernelGGL(clk::frag_plan_kernel, dim3(ntiles), dim3(BLOCK), 0, ctx->cur, args_of(b), f, out_port,
                       out_first_len, pl_n, pl_b, tile_sums);
    hipLaunchKernelGGL(clk::frag_scan_kernel, dim3(1), dim3(1024), 0, ctx->cur, tile_sums, ntiles, totals);
    if (!out->arena)                         // sizing call: nothing is written
        return check_launch(ctx, "clk_ip_fragment");
    hipLaunchKernelGGL(clk::frag_write_kernel<false>, dim3(ntiles), dim3(BLOCK), 0, ctx->cur, args_of(b), f,
                       (const uint8_t *)out_port, (const uint32_t *)pl_n, (const uint32_t *)pl_b,
                       (const uint64_t *)tile_sums, ffirst, clk::FragLookback{});
    return check_launch(ctx, "clk_ip_fragment");
}

}   // extern "C"

namespace {
struct HostRegion {
    uintptr_t host;
    size_t bytes;
    void *dev;
};
std::mutex g_regions_mu;
std::vector<HostRegion> g_regions;
std::atomic<uint64_t> &g_regions_gen = clk::host_regions_gen;
}   // namespace
namespace clk {
alignas(64) std::atomic<uint64_t> host_regions_gen{1};   // its own line: read per packet by every thread
}

extern "C" {

int clk_host_register(clk_ctx *ctx, void *host, size_t bytes, void **dev_base)
{
    int r = enter(ctx);
    if (r) return r;
    if (!host || !bytes || !dev_base)
        return fail(ctx, CLK_EINVAL, "clk_host_register: bad arguments");
    hipError_t e = hipHostRegister(host, bytes, hipHostRegisterMapped);
    if (e != hipSuccess)
        return hip_fail(ctx, e, "hipHostRegister");
    void *dev = nullptr;
    e = hipHostGetDevicePointer(&dev, host, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(host);
        return hip_fail(ctx, e, "hipHostGetDevicePointer");
    }
    std::lock_guard<std::mutex> g(g_regions_mu);
    g_regions.push_back(HostRegion{(uintptr_t)host, bytes, dev});
    g_regions_gen++;
    *dev_base = dev;
    return CLK_SUCCESS;
}

int clk_host_unregister(clk_ctx *ctx, void *host)
{
    int r = enter(ctx);
    if (r) return r;
    {
        std::lock_guard<std::mutex> g(g_regions_mu);
        for (size_t i = 0; i < g_regions.size(); i++)
            if (g_regions[i].host == (uintptr_t)host) {
                g_regions.erase(g_regions.begin() + (long)i);
                g_regions_gen++;
                hipError_t e = hipHostUnregister(host);
                return e == hipSuccess ? CLK_SUCCESS : hip_fail(ctx, e, "hipHostUnregister");
            }
    }
    return fail(ctx, CLK_EINVAL, "clk_host_unregister: not registered");
}

uint64_t clk_host_generation_internal(void) { return g_regions_gen.load(std::memory_order_acquire); }

int clk_host_lookup(const void *p, size_t len, void **host_start, size_t *bytes, void **dev_base)
{
    std::lock_guard<std::mutex> g(g_regions_mu);
    const uintptr_t a = (uintptr_t)p;
    for (const HostRegion &h : g_regions)
        if (a >= h.host && a + len <= h.host + h.bytes) {
            if (host_start) *host_start = (void *)h.host;
            if (bytes) *bytes = h.bytes;
            if (dev_base) *dev_base = h.dev;
            return CLK_SUCCESS;
        }
    return CLK_EINVAL;
}

int clk_count_codes(clk_ctx *ctx, const uint8_t *codes, uint64_t n, uint64_t *counts, uint32_t ncounts)
{
    int r = enter(ctx);
    if (r) return r;
    if (n == 0) return CLK_SUCCESS;
    if (!codes || !counts || ncounts == 0 || ncounts > 256)
        return fail(ctx, CLK_EINVAL, "clk_count_codes: bad arguments");
    unsigned grid = grid_for(ctx, n);
    if (grid > 1024) grid = 1024;
    hipLaunchKernelGGL(clk::count_codes_kernel, dim3(grid), dim3(BLOCK), 0, ctx->cur, codes, n,
                       (unsigned long long *)counts, ncounts);
    return check_launch(ctx, "clk_count_codes");
}

int clk_gen_packets(clk_ctx *ctx, const clk_batch *b, int proto, uint64_t seed, uint64_t first_idx)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_gen_packets"))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    hipLaunchKernelGGL(clk::gen_kernel, dim3(grid_for(ctx, b->n * 64)), dim3(BLOCK), 0, ctx->cur,
                       args_of(b), proto, seed, first_idx);
    return check_launch(ctx, "clk_gen_packets");
}

int clk_gen_corrupt_span(clk_ctx *ctx, const clk_batch *b, uint64_t seed, uint64_t first_idx, uint32_t rate_log2,
                         uint32_t lo, uint32_t hi)
{
    int r = enter(ctx);
    if (r) return r;
    if ((r = check_batch(ctx, b, "clk_gen_corrupt"))) return r;
    if (b->n == 0) return CLK_SUCCESS;
    hipLaunchKernelGGL(clk::corrupt_kernel, dim3(grid_for(ctx, b->n)), dim3(BLOCK), 0, ctx->cur,
                       args_of(b), seed, first_idx, rate_log2, lo, hi);
    return check_launch(ctx, "clk_gen_corrupt");
}

int clk_gen_corrupt(clk_ctx *ctx, const clk_batch *b, uint64_t seed, uint32_t rate_log2)
{
    return clk_gen_corrupt_span(ctx, b, seed, 0, rate_log2, ~0u, 0);
}

int clk_read_stream(clk_ctx *ctx, const void *base, uint64_t bytes, uint64_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if (!base || !out_sum || ((uint64_t)base & 15))
        return fail(ctx, CLK_EINVAL, "clk_read_stream: bad arguments");
    const uint64_t n16 = bytes / 16;
    if (n16 == 0) return CLK_SUCCESS;
    // tools/probes/read_probe.hip's best shapes (CLK_TUNE_READ_SHAPE)
    const clk::u32x4 *p = (const clk::u32x4 *)base;
    unsigned long long *o = (unsigned long long *)out_sum;
    auto grid = [&](uint64_t cap, uint64_t per) { return (unsigned)std::min<uint64_t>(cap, std::max<uint64_t>(1, n16 / per)); };
    switch (ctx->read_shape) {
    case 1:
        hipLaunchKernelGGL(clk::read_stream_kernel<4>, dim3(grid(8192, 4 * BLOCK)), dim3(BLOCK), 0, ctx->cur, p, n16, o);
        break;
    case 2:
        hipLaunchKernelGGL(clk::read_stream_kernel<16>, dim3(grid(2048, 16 * BLOCK)), dim3(BLOCK), 0, ctx->cur, p, n16, o);
        break;
    case 3:
        hipLaunchKernelGGL(clk::read_wave_kernel<8>, dim3(grid(4096, 8 * BLOCK)), dim3(BLOCK), 0, ctx->cur, p, n16, o);
        break;
    case 4:     // rows of 1536 B, one step of 16 rows per workgroup (the C3 Check kernels' pattern)
        hipLaunchKernelGGL(clk::read_rows_kernel<6>, dim3(grid(1u << 30, 16 * 96)), dim3(BLOCK), 0, ctx->cur, p, n16, o);
        break;
    case 5:     // ... on a grid capped at 8K workgroups
        hipLaunchKernelGGL(clk::read_rows_kernel<6>, dim3(grid(8192, 16 * 96)), dim3(BLOCK), 0, ctx->cur, p, n16, o);
        break;
    default:
        hipLaunchKernelGGL(clk::read_stream_kernel<8>, dim3(grid(8192, 8 * BLOCK)), dim3(BLOCK), 0, ctx->cur, p, n16, o);
    }
    return check_launch(ctx, "clk_read_stream");
}

int clk_copy_stream(clk_ctx *ctx, void *dst, const void *src, uint64_t bytes, int shape, uint64_t *out_sum)
{
    int r = enter(ctx);
    if (r) return r;
    if (!src || ((uint64_t)src & 15) || (shape != 4 && (!dst || ((uint64_t)dst & 15))) || (shape == 4 && !out_sum) ||
        shape < 0 || shape > 7)
        return fail(ctx, CLK_EINVAL, "clk_copy_stream: bad arguments");
    const uint64_t n16 = bytes / 16;
    if (n16 == 0) return CLK_SUCCESS;
    const clk::u32x4 *s = (const clk::u32x4 *)src;
    clk::u32x4 *d = (clk::u32x4 *)dst;
    auto grid = [&](uint64_t cap, uint64_t per) { return (unsigned)std::min<uint64_t>(cap, std::max<uint64_t>(1, n16 / per)); };
    switch (shape) {
    case 0:
        hipLaunchKernelGGL((clk::copy_stream_kernel<4, true>), dim3(grid(8192, 4 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    case 1:
        hipLaunchKernelGGL((clk::copy_stream_kernel<8, true>), dim3(grid(8192, 8 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    case 2:
        hipLaunchKernelGGL((clk::copy_stream_kernel<4, false>), dim3(grid(8192, 4 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    case 3:
        hipLaunchKernelGGL((clk::copy_stream_kernel<8, false>), dim3(grid(16384, 8 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    case 5:
        hipLaunchKernelGGL((clk::copy_stream_kernel<16, false>), dim3(grid(4096, 16 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    case 6:
        hipLaunchKernelGGL(clk::copy_wave_kernel<8>, dim3(grid(4096, 8 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    case 7:     // one step per thread: the grid covers the buffer
        hipLaunchKernelGGL((clk::copy_stream_kernel<4, false>), dim3(grid(1u << 30, 4 * BLOCK)), dim3(BLOCK), 0, ctx->cur, s, d, n16);
        break;
    default:    // the C4 Set pattern: read all, one 64 B block in six written back
        hipLaunchKernelGGL(clk::read_write_blocks_kernel<8>, dim3(grid(8192, 8 * BLOCK)), dim3(BLOCK), 0, ctx->cur,
                           (clk::u32x4 *)s, n16, 6u, (unsigned long long *)out_sum);
    }
    return check_launch(ctx, "clk_copy_stream");
}

} // extern "C"
