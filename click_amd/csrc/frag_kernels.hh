// frag_kernels.hh -- IPFragmenter (elements/ip/ipfragmenter.cc:53-171) on
// gfx950, for whole batches.
//
// When the fragments are written (arena given) one launch does it all
// (frag_write_kernel<true>: plan + decoupled look-back scan + write; the
// plan prologue also rewrites plain 20-byte first-fragment headers in
// place while their line is cached); a
// sizing call (no arena), or CLK_FRAG_FUSED=0, runs three launches, no
// host round trip:
//   frag_plan_kernel   lane per packet: the element's decision (port 0 / 1 /
//                      2), the first fragment's length, how many fragments
//                      it appends and their arena bytes (16 B-aligned
//                      slots); one (fragments, bytes) sum per 1024-packet tile.
//   frag_scan_kernel   one block: exclusive scan of the tile sums, totals.
//   frag_write_kernel  per tile: block scan of the per-packet counts; then
//                      one 16-lane group per fragmenting packet (four per
//                      wave) rewrites the first fragment's header in place
//                      (ip_len, MF, DF/ip_id, ip_sum) and writes the other
//                      fragments -- header (base header + copied options,
//                      per-fragment ip_off / ip_len / ip_sum) and payload,
//                      four unaligned 16 B loads per lane in flight, all
//                      issued before the packet's stores; the next
//                      packet's header is prefetched meanwhile.
// FLAT (default when fragments are written): frag_write_kernel<true, true>
// plans, scans and rewrites the first fragments' headers as above, but for
// the packets without options it writes only the descriptors and a 16 B
// record per appended fragment; frag_flat_kernel then writes those
// fragments, headers included, as one flat copy over the arena (every line
// written by one wave, 16 B-aligned stores).  Packets with options keep the
// 16-lane group path.
// Appended fragments are packed in packet order, as the reference pushes
// them, so the arena layout equals the oracle's (oracle_ip_fragment_batch).
#pragma once
#include "cksum_kernels.hh"

namespace clk {

#ifndef CLK_FRAG_TILE
#define CLK_FRAG_TILE 1024
#endif
constexpr uint32_t FRAG_TILE = CLK_FRAG_TILE;   // packets per block (256 threads x FRAG_PER)
constexpr int FRAG_PER = FRAG_TILE / 256;
static_assert(FRAG_TILE % 256 == 0 && FRAG_PER >= 1 && FRAG_PER <= 8, "tile of 256..2048 packets");

struct FragArgs {
    uint32_t mtu;
    int honor_df;
    const uint16_t *new_id;     // per packet, nullable (ip_id kept)
    uint8_t *arena;             // appended fragments
    uint64_t arena_bytes;
    uint64_t *frag_off;
    uint32_t *frag_len;
    uint32_t *frag_src;
    uint64_t max_frags;
    struct FragFlat *fx;        // FLAT: per appended fragment, the payload pass's record
};

// FLAT: what frag_flat_kernel needs of one appended fragment (16 B).  The
// write kernel fills one for every fragment index below min(total,
// max_frags): dlen 0 marks a fragment the write kernel wrote itself (copied
// options) or that has no room; its arena offset keeps the records ordered.
struct FragFlat {
    uint64_t bp_dlen;           // arena offset (bits 0..47) | payload bytes << 48
    uint32_t pkt;               // packet index
    uint16_t fo;                // the fragment's ip_off, host order (ipfragmenter.cc:145-147)
    uint16_t src;               // its payload's offset in the packet
};
constexpr uint64_t FLAT_BP = (1ull << 48) - 1;

struct FragPlan {
    uint32_t port, first_len, hlen, out_hlen, step, nextra, bytes;
    int first_dlen, in_dlen;
};

// Length of the copied options (ipfragmenter.cc:53-86 with ip2 == 0).
__device__ __forceinline__ uint32_t frag_optcopy_len(const uint8_t *ip, uint32_t hlen)
{
    uint32_t i = 20, out = 0;
    while (i < hlen) {
        const uint32_t t = ld_u8(ip + i);
        if (t == 1) {                                   // NOP: not copied
            i++;
            continue;
        }
        if (t == 0 || i + 1 == hlen)
            break;
        const uint32_t l = ld_u8(ip + i + 1);
        if (l < 2 || i + l > hlen)
            break;
        if (t & 0x80)
            out += l;
        i += l;
    }
    return (out + 3) & ~3u;
}

__device__ __forceinline__ uint32_t slot16(uint32_t b) { return (b + 15) & ~15u; }

// Whether frag_plan reads the header (it does only for packets longer than the MTU).
__device__ __forceinline__ bool frag_reads_header(uint32_t caplen, uint32_t mtu)
{
    return (int)caplen > (int)mtu && caplen >= 20;
}

// The element's decision for one packet (ipfragmenter.cc:88-171), from the
// header's bytes 0-3 (w0) and 4-7 (w4), loaded by the caller when
// frag_reads_header().
__device__ __forceinline__ FragPlan frag_plan_words(const uint8_t *ip, uint32_t caplen, uint32_t mtu, int honor_df,
                                                    uint32_t w0, uint32_t w4)
{
    FragPlan p;
    p.port = 0;
    p.first_len = caplen;
    p.hlen = p.out_hlen = p.step = p.nextra = p.bytes = 0;
    p.first_dlen = p.in_dlen = 0;
    if ((int)caplen <= (int)mtu)                       // ipfragmenter.cc:167-168
        return p;
    if (caplen < 20) {                                 // domain guard (oracle: the same)
        p.port = 1;
        return p;
    }
    p.hlen = (w0 & 0xF) << 2;                          // 92
    p.first_dlen = (int)((mtu - p.hlen) & ~7u);        // 93 (unsigned MTU, int result)
    p.in_dlen = (int)bswap16(w0 >> 16) - (int)p.hlen;  // 94
    if ((((w4 >> 16) & 0x40) && honor_df) || p.first_dlen < 8) {   // 96-102
        p.port = 1;
        return p;
    }
    p.port = 2;
    p.first_len = p.hlen + (uint32_t)p.first_dlen;     // 117, 121-122
    p.out_hlen = 20 + frag_optcopy_len(ip, p.hlen);    // 127
    p.step = (mtu - p.out_hlen) & ~7u;                 // 131 (>= first_dlen >= 8)
    const int rem = p.in_dlen - p.first_dlen;
    if (rem > 0) {
        p.nextra = ((uint32_t)rem + p.step - 1) / p.step;
        const uint32_t last = (uint32_t)rem - (p.nextra - 1) * p.step;
        p.bytes = (p.nextra - 1) * slot16(p.out_hlen + p.step) + slot16(p.out_hlen + last);
    }
    return p;
}

// K1: plan.  Thread t of a block takes packets tile + t + 256k (k < 4).
__global__ void __launch_bounds__(256) frag_plan_kernel(BatchArgs b, FragArgs f, uint8_t *out_port,
                                                        uint32_t *out_first_len, uint32_t *pl_n, uint32_t *pl_b,
                                                        uint64_t *tile_sums)
{
    __shared__ uint64_t red[2][4];
    const uint64_t tile = (uint64_t)blockIdx.x * FRAG_TILE;
    uint64_t sn = 0, sb = 0;
    // all four packets' header words in flight before any is planned
    uint32_t cl[FRAG_PER], w0[FRAG_PER], w4[FRAG_PER];
#pragma unroll
    for (int k = 0; k < FRAG_PER; k++) {
        const uint64_t i = tile + threadIdx.x + 256u * k;
        cl[k] = i < b.n ? pkt_len(b, i) : 0u;
        const bool rd = i < b.n && frag_reads_header(cl[k], f.mtu);
        const uint8_t *ip = b.base + (i < b.n ? pkt_off(b, i) : 0);
        w0[k] = rd ? ld_u32_unaligned(ip) : 0u;
        w4[k] = rd ? ld_u32_unaligned(ip + 4) : 0u;
    }
#pragma unroll
    for (int k = 0; k < FRAG_PER; k++) {
        const uint64_t i = tile + threadIdx.x + 256u * k;
        if (i < b.n) {
            const FragPlan p = frag_plan_words(b.base + pkt_off(b, i), cl[k], f.mtu, f.honor_df, w0[k], w4[k]);
            out_port[i] = (uint8_t)p.port;
            out_first_len[i] = p.first_len;
            pl_n[i] = p.nextra;
            pl_b[i] = p.bytes;
            sn += p.nextra;
            sb += p.bytes;
        }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        sn += __shfl_xor(sn, m, 64);
        sb += __shfl_xor(sb, m, 64);
    }
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wv] = sn;
        red[1][wv] = sb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        tile_sums[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        tile_sums[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
}

// K2: one block of 1024 threads, exclusive scan of the tile sums in place;
// totals = {fragments, arena bytes}.
__global__ void __launch_bounds__(1024) frag_scan_kernel(uint64_t *tile_sums, uint32_t ntiles, uint64_t *totals)
{
    __shared__ uint64_t part[2][1024];
    const uint32_t per = (ntiles + blockDim.x - 1) / blockDim.x;
    const uint32_t lo = threadIdx.x * per < ntiles ? threadIdx.x * per : ntiles;
    const uint32_t hi = lo + per < ntiles ? lo + per : ntiles;
    uint64_t sn = 0, sb = 0;
    for (uint32_t k = lo; k < hi; k++) {
        sn += tile_sums[2 * k];
        sb += tile_sums[2 * k + 1];
    }
    part[0][threadIdx.x] = sn;
    part[1][threadIdx.x] = sb;
    __syncthreads();
    if (threadIdx.x < 2) {                       // serial over 1024 partials, one thread per column
        uint64_t run = 0;
        for (uint32_t t = 0; t < blockDim.x; t++) {
            const uint64_t v = part[threadIdx.x][t];
            part[threadIdx.x][t] = run;
            run += v;
        }
        totals[threadIdx.x] = run;
    }
    __syncthreads();
    uint64_t rn = part[0][threadIdx.x], rb = part[1][threadIdx.x];
    for (uint32_t k = lo; k < hi; k++) {
        const uint64_t vn = tile_sums[2 * k], vb = tile_sums[2 * k + 1];
        tile_sums[2 * k] = rn;
        tile_sums[2 * k + 1] = rb;
        rn += vn;
        rb += vb;
    }
}

// 16 bytes from an arbitrary source address p; bytes at or past `hi` read
// as 0 (and are not loaded unless they share a dword with a byte below hi).
__device__ __forceinline__ u32x4 load16_guarded(uint64_t p, uint64_t hi)
{
    const uint64_t q = p & ~3ull;
    const uint32_t sh = (uint32_t)(p & 3);
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        d[k] = q + 4 * k < hi ? gload4(q + 4 * k) : 0u;
    u32x4 r;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t w = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
        const int64_t valid = (int64_t)hi - (int64_t)(p + 4 * j);
        r[j] = w & lowmask(valid > 4 ? 4 : (int)valid);
    }
    return r;
}

#ifndef CLK_FRAG_PRO
#define CLK_FRAG_PRO 1         // fused: plain headers rewritten in place by the tile prologue
#endif
#ifndef CLK_FRAG_FUSED
#define CLK_FRAG_FUSED 1       // one launch (plan + look-back scan + write) when fragments are written
#endif
#ifndef CLK_FRAG_FLAT
#define CLK_FRAG_FLAT 1        // fused: plain-header packets' fragments written by frag_flat_kernel
#endif
#ifndef CLK_FRAG_HDR_X4
#define CLK_FRAG_HDR_X4 1      // fused plan: a packet's 20 header bytes in two loads, not five
#endif
#ifndef CLK_FRAG_HDR_FIRST
#define CLK_FRAG_HDR_FIRST 0
#endif
#ifndef CLK_FRAG_UA
#define CLK_FRAG_UA 1
#endif
#ifndef CLK_FRAG_HDR16
#define CLK_FRAG_HDR16 1    // prologue: the rewritten first-fragment header as one 16 B store
#endif
#ifndef CLK_FRAG_HDR_NT
#define CLK_FRAG_HDR_NT 0   // ... nontemporal (tuning knob)
#endif
#ifndef CLK_FRAG_XCD
#define CLK_FRAG_XCD 0      // unfused write kernel: XCD-contiguous tiles (tuning knob)
#endif
#ifndef CLK_FRAG_NT_STORE
#define CLK_FRAG_NT_STORE 0
#endif
#ifndef CLK_FRAG_NT_LOAD
#define CLK_FRAG_NT_LOAD 0
#endif
// load16_guarded at ip + o with the bound ip + hi (offsets < 64 KiB).
__device__ __forceinline__ u32x4 load16_rel(const uint8_t *ip, uint32_t o, uint32_t hi)
{
#if CLK_FRAG_UA
    typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
    if (o + 16 <= hi)                    // one global_load_dwordx4 (the HSA queues run in unaligned mode)
        return *(const __attribute__((address_space(1))) u32x4_a1 *)(ip + o);
#endif
    const uint32_t q = o & ~3u, sh = o & 3;
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        d[k] = q + 4 * k < hi ? (CLK_FRAG_NT_LOAD ? __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t *)(ip + q + 4 * k))
                                                  : gload4((uint64_t)ip + q + 4 * k)) : 0u;
    u32x4 r;
#pragma unroll
    for (int j = 0; j < 4; j++)
        r[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh) & lowmask((int)(hi - (o + 4 * j)));
    return r;
}

__device__ __forceinline__ void st_u32(uint8_t *p, uint32_t v)
{
    *(__attribute__((address_space(1))) uint32_t *)p = v;
}

// Header word sum over the lanes [0, nw) of a 16-lane group (each lane one
// dword), folded and complemented: click_in_cksum of the header with
// ip_sum = 0 (the caller zeroes the upper half of the group's lane 2).
__device__ __forceinline__ uint32_t group_header_cksum(uint32_t dw, uint32_t gl, uint32_t nw)
{
    uint32_t s = gl < nw ? (dw & 0xFFFF) + (dw >> 16) : 0u;
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1)              // the header is within the group's first 16 lanes
        s += __shfl_xor(s, m, 64);
    return in_cksum_fold(s);
}

#ifndef CLK_FRAG_G
#define CLK_FRAG_G 16
#endif
#ifndef CLK_FRAG_U
#define CLK_FRAG_U 4
#endif
constexpr uint32_t FRAG_G = CLK_FRAG_G;  // lanes per fragmenting packet in frag_write_kernel (16, 32, 64)
constexpr int FRAG_U = CLK_FRAG_U;       // 16 B payload loads in flight per lane
#ifndef CLK_FRAG_WPE
#define CLK_FRAG_WPE 4
#endif

// Header dword gl (< 15) of a packet, 0 past caplen: the prefetch of the
// next fragmenting packet's header (port 2 implies caplen > mtu >= hlen + 8).
__device__ __forceinline__ uint32_t frag_hdr_dword(const uint8_t *ip, uint32_t caplen, uint32_t gl)
{
    return gl < 15 && 4 * gl + 4 <= caplen ? ld_u32_unaligned(ip + 4 * gl) : 0u;
}

// K3: write.  Block = one tile; 16 groups of 16 lanes, group g takes the
// tile's fragmenting packets among g, g+16, ...  Per packet the only
// dependent global round trip is the payload's: the next packet's header is
// prefetched while this one is written, the plan is rebuilt from the header
// registers (options from LDS), and the payload of all appended fragments
// is one chunk space loaded before any store of the packet is issued (gfx9
// counts stores in vmcnt too).
// Single-pass mode (FUSED): the block plans its own tile (frag_plan_words,
// writing port / first_len) and gets its tile's exclusive prefix by a
// decoupled look-back over the tiles before it.  Each tile publishes two
// words, (fragments, bytes), each tagged in its top bits with 1 =
// aggregate of the tile or 2 = inclusive prefix; relaxed agent-scope
// atomics keep a word whole and coherent across XCDs without cache
// invalidation.  Wave 0 reads 64 predecessors at once and stops at the
// nearest inclusive one.  Tiles are numbered by an atomic ticket in start
// order, so every tile waited on has started and publishes its aggregate
// without waiting: the wait always ends.  The spin is bounded anyway (a bug
// cannot hang the GPU; a timeout sets err).
constexpr uint8_t FRAG_PORT_NOROOM = 3;     // CLK_FRAG_NOROOM (include/click_amd_cksum.h)
constexpr uint8_t FRAG_PORT_FAULT = 0xFF;   // CLK_FRAG_FAULT

// Put back the four header fields the first-fragment rewrite changes
// (ip_len, ip_id, ip_off, ip_sum) from the original dwords h[0..2].
__device__ __forceinline__ void frag_restore_header(uint8_t *ip, const uint32_t *h)
{
    st_u16(ip + 2, h[0] >> 16);
    st_u16(ip + 4, h[1] & 0xFFFF);
    st_u16(ip + 6, h[1] >> 16);
    st_u16(ip + 10, h[2] >> 16);
}

struct FragLookback {
    uint32_t *ticket;           // 1 word, zeroed before the launch
    uint32_t *err;              // set when a look-back spin times out (the context's fault word, read by clk_ctx_sync)
    uint64_t *word;             // per tile: tagged (fragments, bytes), zeroed before the launch
    uint64_t *totals;           // {fragments, arena bytes} of the batch
    uint8_t *out_port;
    uint32_t *out_first_len;
    uint32_t ntiles;
};

constexpr uint64_t LB_VAL = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t lb_load(uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool FUSED, bool FLAT = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CLK_FRAG_WPE))) frag_write_kernel(BatchArgs b, FragArgs f, const uint8_t *port,
                                                         const uint32_t *pl_n, const uint32_t *pl_b,
                                                         const uint64_t *tile_sums, uint64_t *out_frag_first,
                                                         FragLookback lb)
{
    constexpr uint32_t NG = 256 / FRAG_G;
    __shared__ uint32_t pn[FRAG_TILE], pb[FRAG_TILE];     // exclusive prefixes within the tile
    __shared__ uint8_t lport[FRAG_TILE];
    __shared__ uint32_t wsum[2][4];
    __shared__ uint32_t hdr[NG][16];                       // per group: the packet's header dwords
    __shared__ uint32_t optw[NG][11];                      // per group: copied options (<= 40 B + pad)
    __shared__ uint64_t lb_base[2];
    __shared__ uint32_t lb_tile, lb_fault;
    // fused: the original 20-byte headers of the tile's plain (ip_hl 5)
    // fragmenting packets, whose first-fragment header the prologue already
    // rewrote in place (word 0 = 0 marks "not done here")
    __shared__ uint32_t lhdr[FUSED && CLK_FRAG_PRO ? FRAG_TILE : 1][5];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t gl = lane & (FRAG_G - 1), grp = threadIdx.x / FRAG_G, g0 = lane & ~(FRAG_G - 1);
    // unfused: the tiles' prefixes are known, so any order will do
    uint32_t tix = run_block<!FUSED && CLK_FRAG_XCD>();
    if (FUSED) {
        if (threadIdx.x == 0) {
            lb_tile = atomicAdd(lb.ticket, 1u);
            lb_fault = 0;
        }
        __syncthreads();
        tix = lb_tile;
    }
    const uint64_t tile = (uint64_t)tix * FRAG_TILE;
    // block exclusive scan of (nextra, bytes): thread t owns packets 4t..4t+3 of the tile
    uint32_t vn[FRAG_PER], vb[FRAG_PER], tn = 0, tb = 0;
    if (FUSED) {                           // the plan (frag_plan_kernel), header words loaded first
        constexpr int HW = CLK_FRAG_PRO ? 5 : 2;   // header dwords loaded per packet
        uint32_t cl[FRAG_PER], hw[FRAG_PER][HW];
#pragma unroll
        for (int k = 0; k < FRAG_PER; k++) {
            const uint64_t i = tile + FRAG_PER * threadIdx.x + k;
            cl[k] = i < b.n ? pkt_len(b, i) : 0u;
            const bool rd = i < b.n && frag_reads_header(cl[k], f.mtu);   // caplen >= 20
            const uint8_t *ip = b.base + (i < b.n ? pkt_off(b, i) : 0);
            if (HW == 5 && CLK_FRAG_HDR_X4) {          // bytes 0-15 in one load (unaligned mode), then 16-19
                typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
                const u32x4 q = rd ? *(const __attribute__((address_space(1))) u32x4_a1 *)ip : u32x4{0, 0, 0, 0};
#pragma unroll
                for (int d = 0; d < 4; d++)
                    hw[k][d] = q[d];
                hw[k][HW - 1] = rd ? ld_u32_unaligned(ip + 16) : 0u;
            } else {
#pragma unroll
                for (int d = 0; d < HW; d++)
                    hw[k][d] = rd ? ld_u32_unaligned(ip + 4 * d) : 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < FRAG_PER; k++) {
            const uint64_t i = tile + FRAG_PER * threadIdx.x + k;
            const uint32_t pk = FRAG_PER * threadIdx.x + k;
            vn[k] = vb[k] = 0;
            lport[pk] = 0;
            if (CLK_FRAG_PRO)
                lhdr[pk][0] = 0;
            if (i < b.n) {
                uint8_t *ip = b.base + pkt_off(b, i);
                const FragPlan p = frag_plan_words(ip, cl[k], f.mtu, f.honor_df, hw[k][0], hw[k][1]);
                lb.out_port[i] = (uint8_t)p.port;
                lb.out_first_len[i] = p.first_len;
                lport[pk] = (uint8_t)p.port;
                vn[k] = p.nextra;
                vb[k] = p.bytes;
                if (CLK_FRAG_PRO && p.port == 2 && p.hlen == 20) {
                    // the first fragment's header (112-120) while its line is in the
                    // cache: ip_len, MF set / DF cleared (ip_id when DF and new_id),
                    // ip_sum over the rewritten 20 bytes
                    uint32_t h[5];
#pragma unroll
                    for (int d = 0; d < 5; d++) {
                        h[d] = hw[k][d];
                        lhdr[pk][d] = hw[k][d];
                    }
                    const bool df = (h[1] >> 16) & 0x40;
                    h[0] = (h[0] & 0xFFFF) | (bswap16(p.first_len) << 16);
                    if (df && f.new_id)
                        h[1] = (h[1] & 0xFFFF0000u) | f.new_id[i];
                    h[1] = (h[1] & ~(0x40u << 16)) | (0x20u << 16);
                    h[2] &= 0xFFFF;
                    uint32_t sum = 0;
#pragma unroll
                    for (int d = 0; d < 5; d++)
                        sum += (h[d] & 0xFFFF) + (h[d] >> 16);
                    const uint32_t ck = in_cksum_fold(sum);
                    if (CLK_FRAG_HDR16 && ((uint64_t)ip & 3) == 0) {
                        // one 16 B store of bytes [0, 16) (ip_src rewritten
                        // unchanged): one partial-block write instead of four
                        const u32x4 w = {h[0], h[1], h[2] | (ck << 16), h[3]};
                        typedef __attribute__((address_space(1))) u32x4_a4 g4;
                        if (CLK_FRAG_HDR_NT)
                            __builtin_nontemporal_store(w, (g4 *)ip);
                        else
                            *(g4 *)ip = w;
                    } else {
                        st_u16(ip + 2, h[0] >> 16);
                        st_u16(ip + 4, h[1] & 0xFFFF);
                        st_u16(ip + 6, h[1] >> 16);
                        st_u16(ip + 10, ck);
                    }
                }
            }
            tn += vn[k];
            tb += vb[k];
        }
    } else {
#pragma unroll
        for (int k = 0; k < FRAG_PER; k++) {
            const uint64_t i = tile + FRAG_PER * threadIdx.x + k;
            vn[k] = i < b.n ? pl_n[i] : 0u;
            vb[k] = i < b.n ? pl_b[i] : 0u;
            lport[FRAG_PER * threadIdx.x + k] = i < b.n ? port[i] : 0u;
            tn += vn[k];
            tb += vb[k];
        }
    }
    uint32_t in_ = tn, ib = tb;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a = __shfl_up(in_, d, 64), c = __shfl_up(ib, d, 64);
        if ((int)lane >= d) {
            in_ += a;
            ib += c;
        }
    }
    if (lane == 63) {
        wsum[0][wv] = in_;
        wsum[1][wv] = ib;
    }
    __syncthreads();
    uint32_t bn = 0, bb = 0;
    for (uint32_t w = 0; w < wv; w++) {
        bn += wsum[0][w];
        bb += wsum[1][w];
    }
    uint32_t rn = bn + in_ - tn, rb = bb + ib - tb;
#pragma unroll
    for (int k = 0; k < FRAG_PER; k++) {
        pn[FRAG_PER * threadIdx.x + k] = rn;
        pb[FRAG_PER * threadIdx.x + k] = rb;
        rn += vn[k];
        rb += vb[k];
    }
    if (FUSED && wv == 0) {                // decoupled look-back over the tiles before this one
        const uint64_t an = (uint64_t)wsum[0][0] + wsum[0][1] + wsum[0][2] + wsum[0][3];
        const uint64_t ab = (uint64_t)wsum[1][0] + wsum[1][1] + wsum[1][2] + wsum[1][3];
        if (lane == 0) {
            const uint64_t tag = (tix == 0 ? 2ull : 1ull) << 62;
            lb_store(&lb.word[2 * tix + 1], tag | ab);
            lb_store(&lb.word[2 * tix], tag | an);
        }
        uint64_t en = 0, eb = 0;
        int64_t top = (int64_t)tix - 1;
        uint32_t spins = 0;
        while (top >= 0) {
            const int64_t j = top - (int64_t)lane;
            uint64_t vn = 0, vb = 0;
            uint32_t st = 2;                           // before tile 0: an inclusive 0
            if (j >= 0) {
                vn = lb_load(&lb.word[2 * j]);
                vb = lb_load(&lb.word[2 * j + 1]);
                st = (uint32_t)(vn >> 62);
                if ((uint32_t)(vb >> 62) != st)        // the pair is being rewritten: read again
                    st = 0;
                vn &= LB_VAL;
                vb &= LB_VAL;
            }
            const uint64_t m2 = __ballot(st == 2), m0 = __ballot(st == 0);
            const uint32_t first2 = m2 ? (uint32_t)__builtin_ctzll(m2) : 64u;
            const uint64_t below = first2 >= 64 ? ~0ull : ((1ull << first2) - 1);
            if (m0 & below) {                          // a nearer tile has not published yet
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22)) {            // never reached when the tiles start in ticket order
                    if (lane == 0) {
                        atomicOr(lb.err, 1u);
                        lb_fault = 1;
                    }
                    break;
                }
                continue;
            }
            uint32_t n_lo = lane <= first2 ? (uint32_t)vn : 0u, n_hi = lane <= first2 ? (uint32_t)(vn >> 32) : 0u;
            uint32_t b_lo = lane <= first2 ? (uint32_t)vb : 0u, b_hi = lane <= first2 ? (uint32_t)(vb >> 32) : 0u;
            uint64_t sn = 0, sb = 0;
            // exact 64-bit sum of the 64 lanes' values: sum halves separately (each < 2^38 over 64 lanes)
            uint64_t a0 = n_lo, a1 = n_hi, c0 = b_lo, c1 = b_hi;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) {
                a0 += __shfl_xor(a0, m, 64);
                a1 += __shfl_xor(a1, m, 64);
                c0 += __shfl_xor(c0, m, 64);
                c1 += __shfl_xor(c1, m, 64);
            }
            sn = a0 + (a1 << 32);
            sb = c0 + (c1 << 32);
            en += sn;
            eb += sb;
            if (first2 < 64)
                break;
            top -= 64;
        }
        if (lane == 0) {
            if (tix != 0) {
                lb_store(&lb.word[2 * tix + 1], (2ull << 62) | (eb + ab));
                lb_store(&lb.word[2 * tix], (2ull << 62) | (en + an));
            }
            if (tix == lb.ntiles - 1) {
                lb.totals[0] = en + an;
                lb.totals[1] = eb + ab;
            }
            lb_base[0] = en;
            lb_base[1] = eb;
        }
    }
    __syncthreads();
    if (FUSED && lb_fault) {
        // this tile's prefix is unknown: put back the headers the prologue
        // rewrote, mark every packet of the tile CLK_FRAG_FAULT, write nothing
        for (uint32_t j = threadIdx.x; j < FRAG_TILE && tile + j < b.n; j += blockDim.x) {
            if (FUSED && CLK_FRAG_PRO && lhdr[j][0] != 0u)
                frag_restore_header(b.base + pkt_off(b, tile + j), lhdr[j]);
            lb.out_port[tile + j] = FRAG_PORT_FAULT;
        }
        return;
    }
    const uint64_t fbase = FUSED ? lb_base[0] : tile_sums[2 * tix], bbase = FUSED ? lb_base[1] : tile_sums[2 * tix + 1];
    for (uint32_t j = threadIdx.x; j < FRAG_TILE && tile + j < b.n; j += blockDim.x)
        out_frag_first[tile + j] = fbase + pn[j];
    const uint32_t lim = b.n - tile < FRAG_TILE ? (uint32_t)(b.n - tile) : FRAG_TILE;
    if (FLAT) {
        // the plain-header packets (first-fragment header rewritten by the
        // prologue, original words in lhdr), a thread per packet: their
        // descriptors and frag_flat_kernel's records; the 16-lane groups
        // below take only the packets with options.  Packet t + 256k, so a
        // wave's stores cover consecutive records
#pragma unroll
        for (int k = 0; k < FRAG_PER; k++) {
            const uint32_t pk = threadIdx.x + 256u * k;
            if (pk >= lim || lhdr[pk][0] == 0u)
                continue;
            const uint64_t i = tile + pk;
            uint8_t *ip = b.base + pkt_off(b, i);
            const uint32_t h0 = lhdr[pk][0], h1 = lhdr[pk][1];
            const FragPlan p = frag_plan_words(ip, pkt_len(b, i), f.mtu, f.honor_df, h0, h1);   // hlen 20: no option read
            const uint64_t fidx = fbase + pn[pk], bpos = bbase + pb[pk];
            const uint32_t slot_f = slot16(20 + p.step);
            lport[pk] = 0;                                 // not for the groups
            if (!(fidx + p.nextra <= f.max_frags && bpos + p.bytes <= f.arena_bytes)) {
                frag_restore_header(ip, lhdr[pk]);         // port CLK_FRAG_NOROOM, bytes kept
                lb.out_port[i] = FRAG_PORT_NOROOM;
                for (uint32_t q = 0; q < p.nextra && fidx + q < f.max_frags; q++)
                    f.fx[fidx + q] = FragFlat{(bpos + (uint64_t)q * slot_f) & FLAT_BP, 0u, 0, 0};
                continue;
            }
            // ntohs(ip_off) of the first fragment: MF set, DF cleared (112-118)
            const uint32_t off_first = bswap16((((h1 >> 16) & ~0x40u) | 0x20u) & 0xFFFF);
            const bool had_mf = (h1 >> 16) & 0x20;
            const uint32_t pay0 = 20 + (uint32_t)p.first_dlen;
            const int rem = p.in_dlen - p.first_dlen;
            const uint32_t last = (uint32_t)rem - (p.nextra - 1) * p.step;
            for (uint32_t q = 0; q < p.nextra; q++) {
                const int off = p.first_dlen + (int)(q * p.step);
                const uint32_t dlen = q + 1 < p.nextra ? p.step : last;
                const uint64_t bp = bpos + (uint64_t)q * slot_f;
                uint32_t fo = (off_first + ((uint32_t)off >> 3)) & 0xFFFF;                 // 145
                if ((int)dlen + off >= p.in_dlen && !had_mf)                              // 146-147
                    fo &= ~0x2000u;
                f.frag_off[fidx + q] = bp;                 // (from the flat pass: 1.5 % slower overall, r06x)
                f.frag_len[fidx + q] = 20 + dlen;
                f.frag_src[fidx + q] = (uint32_t)i;
                f.fx[fidx + q] = FragFlat{bp | (uint64_t)dlen << 48, (uint32_t)i, (uint16_t)fo,
                                          (uint16_t)(pay0 + q * p.step)};
            }
        }
        __syncthreads();                                   // lport
    }
    auto next_j = [&](uint32_t j) {
        while (j < lim && lport[j] != 2)
            j += NG;
        return j;
    };
    // header dword gl of tile packet jj: from LDS when the prologue rewrote
    // its header (the original words), else from memory
    auto hdr_word = [&](uint32_t jj, const uint8_t *ipp, uint32_t cap) -> uint32_t {
        if (FUSED && CLK_FRAG_PRO && lhdr[jj][0] != 0u)
            return gl < 5 ? lhdr[jj][gl] : 0u;
        return frag_hdr_dword(ipp, cap, gl);
    };
    uint32_t j = next_j(grp);
    const uint8_t *nip = nullptr;
    uint32_t ncap = 0, ndw = 0;
    if (j < lim) {
        nip = b.base + pkt_off(b, tile + j);
        ncap = pkt_len(b, tile + j);
        ndw = hdr_word(j, nip, ncap);
    }
    while (j < lim) {
        const uint64_t i = tile + j;
        uint8_t *ip = (uint8_t *)nip;
        const uint32_t caplen = ncap;
        uint32_t dw = ndw;
        const uint32_t jn = next_j(j + NG);
        if (jn < lim) {                                    // prefetch the group's next packet
            nip = b.base + pkt_off(b, tile + jn);
            ncap = pkt_len(b, tile + jn);
            ndw = hdr_word(jn, nip, ncap);
        }
        // the plan (frag_plan for a port-2 packet), from the header registers
        const uint32_t w0 = __shfl(dw, g0, 64), w1 = __shfl(dw, g0 + 1, 64);
        const uint32_t hlen = (w0 & 0xF) << 2, nw = hlen >> 2;                 // 92
        const int first_dlen = (int)((f.mtu - hlen) & ~7u);                     // 93
        const int in_dlen = (int)bswap16(w0 >> 16) - (int)hlen;                // 94
        if (gl < 16)
            hdr[grp][gl] = gl < nw ? dw : 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // copied options (53-86): every lane walks the LDS bytes, lane 0 copies
        uint32_t olen = 0;
        {
            const uint8_t *hb = (const uint8_t *)hdr[grp];
            uint8_t *ob = (uint8_t *)optw[grp];
            uint32_t k = 20;
            while (k < hlen) {
                const uint32_t t = hb[k];
                if (t == 1) {
                    k++;
                    continue;
                }
                if (t == 0 || k + 1 == hlen)
                    break;
                const uint32_t l = hb[k + 1];
                if (l < 2 || k + l > hlen)
                    break;
                if (t & 0x80) {
                    if (gl == 0)
                        for (uint32_t c = 0; c < l; c++)
                            ob[olen + c] = hb[k + c];
                    olen += l;
                }
                k += l;
            }
            if (gl == 0)
                for (uint32_t c = olen; c & 3; c++)
                    ob[c] = 0;
            olen = (olen + 3) & ~3u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t out_hlen = 20 + olen, qw = out_hlen >> 2;               // 127
        const uint32_t step = (f.mtu - out_hlen) & ~7u;                         // 131
        const int rem = in_dlen - first_dlen;
        const uint32_t nextra = rem > 0 ? ((uint32_t)rem + step - 1) / step : 0u;
        const uint32_t last = rem > 0 ? (uint32_t)rem - (nextra - 1) * step : 0u;
        const uint32_t slot_f = slot16(out_hlen + step);
        // the first fragment's header (112-120), in the lanes' registers
        const bool df = (w1 >> 16) & 0x40, had_mf = (w1 >> 16) & 0x20;
        if (gl == 0)
            dw = (dw & 0xFFFF) | (bswap16(hlen + (uint32_t)first_dlen) << 16);
        if (gl == 1) {
            if (df && f.new_id)
                dw = (dw & 0xFFFF0000u) | f.new_id[i];
            dw = (dw & ~(0x40u << 16)) | (0x20u << 16);
        }
        if (gl == 2)
            dw &= 0xFFFF;
        const uint32_t sum = group_header_cksum(dw, gl, nw);
        if (gl == 2)
            dw |= sum << 16;
        // the fragment header template: base 20 bytes of the rewritten
        // header + copied options (140-144)
        uint32_t tpl = gl < 5 ? dw : (gl < qw ? optw[grp][gl - 5] : 0u);
        if (gl == 0)
            tpl = (tpl & ~0xFu) | (qw & 0xF);                                   // ip_hl (144)
        const uint32_t off_first = bswap16(__shfl(dw, g0 + 1, 64) >> 16);      // ntohs(ip->ip_off) after 112-118
        const uint64_t fidx = fbase + pn[j];
        const uint64_t bpos = bbase + pb[j];
        // all of the packet's fragments fit the caller's buffers, or none is
        // written and the packet keeps its bytes (port CLK_FRAG_NOROOM)
        if (!(fidx + nextra <= f.max_frags &&
              bpos + (nextra ? (uint64_t)(nextra - 1) * slot16(out_hlen + step) + slot16(out_hlen + last) : 0) <=
                  f.arena_bytes)) {
            if (gl == 0) {
                if (FUSED && CLK_FRAG_PRO && lhdr[j][0] != 0u)
                    frag_restore_header(ip, lhdr[j]);
                (FUSED ? lb.out_port : (uint8_t *)port)[i] = FRAG_PORT_NOROOM;
            }
            if (FLAT)                                      // nothing for the payload pass
                for (uint32_t k = gl; k < nextra && fidx + k < f.max_frags; k += FRAG_G)
                    f.fx[fidx + k] = FragFlat{(bpos + (uint64_t)k * slot_f) & FLAT_BP, 0u, 0, 0};
            j = jn;
            continue;
        }
        // payload offsets are relative to ip (32-bit): fragment k's payload
        // starts at pay0 + k * step and ends at min(that + dlen_k, caplen)
        const uint32_t pay0 = hlen + (uint32_t)first_dlen;
        // payload chunk space: fragment k < nextra-1 has nch_f chunks, the last nch_l
        const uint32_t nch_f = (step + 15) / 16, nch_l = (last + 15) / 16;
        const uint32_t total = nextra ? (nextra - 1) * nch_f + nch_l : 0u;
        auto write_headers = [&]() {
            // the first fragment's header fields, in place (112-120), unless
            // the prologue wrote them
            if (!(FUSED && CLK_FRAG_PRO && lhdr[j][0] != 0u)) {
                if (gl == 0)
                    st_u16(ip + 2, dw >> 16);
                if (gl == 1) {
                    st_u16(ip + 4, dw & 0xFFFF);
                    st_u16(ip + 6, dw >> 16);
                }
                if (gl == 2)
                    st_u16(ip + 10, dw >> 16);
            }
            // the appended fragments' headers (140-150) and descriptors
            for (uint32_t k = 0; k < nextra; k++) {
                const int off = first_dlen + (int)(k * step);
                const uint32_t dlen = k + 1 < nextra ? step : last;
                const uint32_t qlen = out_hlen + dlen;
                const uint64_t bp = bpos + (uint64_t)k * slot_f;
                const bool fits = fidx + k < f.max_frags && bp + slot16(qlen) <= f.arena_bytes;
                uint32_t h = tpl;
                if (gl == 0)
                    h = (h & 0xFFFF) | (bswap16(qlen) << 16);                // 148
                if (gl == 1) {
                    uint32_t fo = (off_first + ((uint32_t)off >> 3)) & 0xFFFF;  // 145
                    if ((int)dlen + off >= in_dlen && !had_mf)              // 146-147
                        fo &= ~0x2000u;
                    h = (h & 0xFFFF) | (bswap16(fo) << 16);
                }
                if (gl == 2)
                    h &= 0xFFFF;                                            // 149
                const uint32_t s = group_header_cksum(h, gl, qw);
                if (gl == 2)
                    h |= s << 16;                                           // 150
                if (fits) {
                    if (FLAT && gl == (k & (FRAG_G - 1)))
                        f.fx[fidx + k] = FragFlat{bp & FLAT_BP, 0u, 0, 0};   // written here
                    if (gl < qw)
                        st_u32(f.arena + bp + 4 * gl, h);
                    if (gl == (k & (FRAG_G - 1))) {
                        f.frag_off[fidx + k] = bp;
                        f.frag_len[fidx + k] = qlen;
                        f.frag_src[fidx + k] = (uint32_t)i;
                    }
                }
            }
        };
#if CLK_FRAG_HDR_FIRST
        write_headers();
#endif
        uint32_t ck = 0, cc = gl;                          // this lane's next (fragment, chunk)
        for (uint32_t c0 = 0; c0 == 0 || c0 < total; c0 += FRAG_G * FRAG_U) {
            u32x4 v[FRAG_U];
            uint32_t vkc[FRAG_U];                          // k << 16 | chunk, ~0u: none
#pragma unroll
            for (int u = 0; u < FRAG_U; u++) {
                while (ck + 1 < nextra && cc >= nch_f) {
                    cc -= nch_f;
                    ck++;
                }
                const bool ok = ck < nextra && cc < (ck + 1 < nextra ? nch_f : nch_l);
                const uint32_t fs = pay0 + ck * step;
                const uint32_t fe = fs + (ck + 1 < nextra ? step : last);
                v[u] = ok ? load16_rel(ip, fs + 16 * cc, fe < caplen ? fe : caplen) : u32x4{0, 0, 0, 0};
                vkc[u] = ok ? (ck << 16) | cc : 0xFFFFFFFFu;
                cc += FRAG_G;
            }
#if !CLK_FRAG_HDR_FIRST
            if (c0 == 0)
                write_headers();
#endif
#pragma unroll
            for (int u = 0; u < FRAG_U; u++) {
                if (vkc[u] == 0xFFFFFFFFu)
                    continue;
                const uint32_t k = vkc[u] >> 16, c = vkc[u] & 0xFFFF;
                const uint32_t dlen = k + 1 < nextra ? step : last;
                const uint32_t slot = slot16(out_hlen + dlen);
                const uint64_t bp = bpos + (uint64_t)k * slot_f;
                if (fidx + k >= f.max_frags || bp + slot > f.arena_bytes)
                    continue;
                uint8_t *q = f.arena + bp;
                const uint32_t at = out_hlen + 16 * c;    // 4-aligned; the slot ends at `slot`
                if (at + 16 <= slot) {
#if CLK_FRAG_NT_STORE
                    __builtin_nontemporal_store(v[u], (__attribute__((address_space(1))) u32x4_a4 *)(q + at));
#else
                    *(__attribute__((address_space(1))) u32x4_a4 *)(q + at) = v[u];
#endif
                } else {
#pragma unroll
                    for (int d = 0; d < 4; d++)
                        if (at + 4 * d < slot)
                            st_u32(q + at + 4 * d, v[u][d]);
                }
            }
        }
        j = jn;
    }
}

// FLAT payload pass: the appended fragments of the plain-header packets,
// headers included, as a flat copy of the arena.  One wave = FLAT_F
// consecutive fragment records, whose slots are consecutive in the arena;
// lane k < FLAT_F loads record k, the slot starts go to scalar registers,
// and the wave's lanes take the 16 B chunks of the range in order (one
// store instruction = 1 KB of contiguous arena, every store 16 B-aligned),
// each chunk's record found by FLAT_F - 1 scalar compares and its fields
// fetched from that record's lane.  No LDS, no barrier: a wave waits only
// on its own records and loads.  Chunk 0 of a slot is header bytes 0-15
// (the packet's rewritten first-fragment header with the fragment's
// ip_len, ip_off, ip_sum: ipfragmenter.cc:140-150), chunk 1 the header's
// last dword and the payload's first 12 bytes; bytes past the payload up to
// the slot's end are 0, as frag_write_kernel writes them.
#ifndef CLK_FRAG_FLAT_F
#define CLK_FRAG_FLAT_F 8
#endif
#ifndef CLK_FRAG_FLAT_U
#define CLK_FRAG_FLAT_U 4
#endif
#ifndef CLK_FRAG_FLAT_NT
#define CLK_FRAG_FLAT_NT 1      // nontemporal arena stores (r06ag: the pass 6.71 vs 6.82 ms)
#endif
constexpr uint32_t FLAT_F = CLK_FRAG_FLAT_F;     // fragment records per wave (<= 64)
constexpr int FLAT_U = CLK_FRAG_FLAT_U;           // chunks per lane in flight
static_assert(FLAT_F >= 1 && FLAT_F <= 64, "records per wave");

// Records [f0, f0 + FLAT_F) of [.., nf), by one wave.
__device__ __forceinline__ void frag_flat_wave(const BatchArgs &b, const FragArgs &f, uint64_t f0, uint64_t nf)
{
    uint8_t *const arena = f.arena;
    const uint64_t arena_bytes = f.arena_bytes;
    const FragFlat *const fx = f.fx;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t cnt = nf - f0 < FLAT_F ? (uint32_t)(nf - f0) : FLAT_F;
    uint64_t bp = 0, ipa = 0;
    uint32_t dlen = 0, src = 0, hi = 0, fo = 0;
    if (lane < cnt) {
        const FragFlat e = fx[f0 + lane];
        bp = e.bp_dlen & FLAT_BP;
        dlen = (uint32_t)(e.bp_dlen >> 48);
        src = e.src;
        fo = e.fo;
        if (dlen && e.pkt < b.n) {
            const uint32_t caplen = pkt_len(b, e.pkt);
            const uint32_t fe = src + dlen;
            ipa = (uint64_t)(b.base + pkt_off(b, e.pkt));
            hi = fe < caplen ? fe : caplen;
        }
    }
    const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bp >> 32), 0) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bp, 0);
    const uint32_t slot = slot16(20 + dlen);
    // a record this call did not write (a tile whose look-back failed)
    // cannot send a store out of the arena
    const bool ok = ipa != 0 && bp >= base && bp + slot <= arena_bytes;
    const uint32_t stc = lane < cnt ? (uint32_t)((bp - base) >> 4) : 0xFFFFFFFFu;
    const uint32_t endc = lane < cnt ? stc + (ok ? slot >> 4 : 0u) : 0u;
    const uint32_t nchunks = (uint32_t)__builtin_amdgcn_readlane((int)endc, (int)cnt - 1);   // records in arena order
    uint32_t sk[FLAT_F];
#pragma unroll
    for (uint32_t k = 1; k < FLAT_F; k++)
        sk[k] = (uint32_t)__builtin_amdgcn_readlane((int)stc, (int)k);
    typedef __attribute__((address_space(1))) u32x4_a4 g4;
    // wave-uniform trip count: every lane takes part in the shuffles
    for (uint32_t p0 = 0; p0 < nchunks; p0 += 64 * FLAT_U) {
        const uint32_t c0 = p0 + lane;
        u32x4 v[FLAT_U];
        uint32_t x[FLAT_U], ss[FLAT_U], qq[FLAT_U];   // header dword 4; byte in the slot (~0u: none); ip_len | ip_off
#pragma unroll
        for (int u = 0; u < FLAT_U; u++) {
            const uint32_t c = c0 + 64u * u;
            uint32_t j = 0;
#pragma unroll
            for (uint32_t k = 1; k < FLAT_F; k++)
                j += sk[k] <= c;
            const uint64_t ip = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(ipa >> 32), (int)j, 64) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)ipa, (int)j, 64);
            const uint32_t st_j = (uint32_t)__shfl((int)stc, (int)j, 64);
            const uint32_t end_j = (uint32_t)__shfl((int)endc, (int)j, 64);
            const uint32_t src_j = (uint32_t)__shfl((int)src, (int)j, 64);
            const uint32_t hi_j = (uint32_t)__shfl((int)hi, (int)j, 64);
            qq[u] = (uint32_t)__shfl((int)(fo << 16 | (20 + dlen)), (int)j, 64);
            const bool live = c < nchunks && c < end_j;
            const uint32_t sb = 16 * (c - st_j);
            ss[u] = live ? sb : 0xFFFFFFFFu;
            x[u] = live && sb <= 16 ? ld_u32_unaligned((const uint8_t *)ip + 16) : 0u;
            v[u] = !live ? u32x4{0, 0, 0, 0}
                         : sb == 0 ? load16_rel((const uint8_t *)ip, 0, 20)
                                   : load16_rel((const uint8_t *)ip, src_j + sb - 20, hi_j);
        }
#pragma unroll
        for (int u = 0; u < FLAT_U; u++) {
            if (ss[u] == 0xFFFFFFFFu)
                continue;
            u32x4 w = v[u];
            if (ss[u] == 0) {
                const uint32_t q = qq[u];
                w[0] = (w[0] & 0xFFFF) | (bswap16(q & 0xFFFF) << 16);           // ip_len (148)
                w[1] = (w[1] & 0xFFFF) | (bswap16(q >> 16) << 16);             // ip_off (145-147)
                w[2] &= 0xFFFF;                                                 // ip_sum (149-150)
                uint32_t sum = (x[u] & 0xFFFF) + (x[u] >> 16);
#pragma unroll
                for (int d = 0; d < 4; d++)
                    sum += (w[d] & 0xFFFF) + (w[d] >> 16);
                w[2] |= in_cksum_fold(sum) << 16;
            } else if (ss[u] == 16) {
                w[0] = x[u];
            }
            if (CLK_FRAG_FLAT_NT)
                __builtin_nontemporal_store(w, (g4 *)(arena + base + 16ull * (c0 + 64u * u)));
            else
                *(g4 *)(arena + base + 16ull * (c0 + 64u * u)) = w;
        }
    }
}

// Records [lo, min(hi, max_frags)), lo and hi read from device words (a
// tile's look-back word or totals; their tag bits masked): a wave per
// FLAT_F records, the grid striding when the range is larger than it.
__global__ void __launch_bounds__(256) frag_flat_kernel(BatchArgs b, FragArgs f, const uint64_t *lo_p,
                                                        const uint64_t *hi_p)
{
    const uint64_t lo = lo_p ? (lo_p[0] & LB_VAL) : 0;
    const uint64_t hv = hi_p[0] & LB_VAL;
    const uint64_t nf = hv < f.max_frags ? hv : f.max_frags;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;; w += nwaves) {
        const uint64_t f0 = lo + w * FLAT_F;
        if (f0 >= nf)
            return;                                   // wave-uniform
        frag_flat_wave(b, f, f0, nf);
    }
}

} // namespace clk
