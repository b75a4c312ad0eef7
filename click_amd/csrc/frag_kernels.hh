// frag_kernels.hh -- IPFragmenter (elements/ip/ipfragmenter.cc:53-171) on
// gfx950, for whole batches.
//
// Three launches, no host round trip:
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
//                      four 16 B chunks per lane in flight from an
//                      unaligned source.
// Appended fragments are packed in packet order, as the reference pushes
// them, so the arena layout equals the oracle's (oracle_ip_fragment_batch).
#pragma once
#include "cksum_kernels.hh"

namespace clk {

constexpr uint32_t FRAG_TILE = 1024;    // packets per block (256 threads x 4)

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
};

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

__device__ __forceinline__ FragPlan frag_plan(const uint8_t *ip, uint32_t caplen, uint32_t mtu, int honor_df)
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
    const uint32_t w0 = ld_u32_unaligned(ip), w4 = ld_u32_unaligned(ip + 4);
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
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t i = tile + threadIdx.x + 256u * k;
        if (i < b.n) {
            const FragPlan p = frag_plan(b.base + pkt_off(b, i), pkt_len(b, i), f.mtu, f.honor_df);
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
    for (int m = 8; m >= 1; m >>= 1)
        s += __shfl_xor(s, m, 64);
    return in_cksum_fold(s);
}

constexpr uint32_t FRAG_G = 16;          // lanes per fragmenting packet in frag_write_kernel
constexpr int FRAG_U = 4;                // 16 B payload loads in flight per lane

// K3: write.  Block = one tile; 16 groups of 16 lanes, group g takes the
// tile's packets g, g+16, ...  (the same trip count for every group).
__global__ void __launch_bounds__(256) frag_write_kernel(BatchArgs b, FragArgs f, const uint8_t *port,
                                                         const uint32_t *pl_n, const uint32_t *pl_b,
                                                         const uint64_t *tile_sums, uint64_t *out_frag_first)
{
    __shared__ uint32_t pn[FRAG_TILE], pb[FRAG_TILE];     // exclusive prefixes within the tile
    __shared__ uint32_t wsum[2][4];
    __shared__ uint32_t hdr[16][16];                       // per group: the rewritten header dwords
    __shared__ uint32_t optw[16][11];                      // per group: copied options (<= 40 B + pad)
    const uint64_t tile = (uint64_t)blockIdx.x * FRAG_TILE;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t gl = lane & (FRAG_G - 1), grp = threadIdx.x / FRAG_G, g0 = lane & ~(FRAG_G - 1);
    // block exclusive scan of (nextra, bytes): thread t owns packets 4t..4t+3 of the tile
    uint32_t vn[4], vb[4], tn = 0, tb = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t i = tile + 4 * threadIdx.x + k;
        vn[k] = i < b.n ? pl_n[i] : 0u;
        vb[k] = i < b.n ? pl_b[i] : 0u;
        tn += vn[k];
        tb += vb[k];
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
    for (int k = 0; k < 4; k++) {
        pn[4 * threadIdx.x + k] = rn;
        pb[4 * threadIdx.x + k] = rb;
        rn += vn[k];
        rb += vb[k];
    }
    __syncthreads();
    const uint64_t fbase = tile_sums[2 * blockIdx.x], bbase = tile_sums[2 * blockIdx.x + 1];
    for (uint32_t j = threadIdx.x; j < FRAG_TILE && tile + j < b.n; j += blockDim.x)
        out_frag_first[tile + j] = fbase + pn[j];
    // one 16-lane group per fragmenting packet
    for (uint32_t j = grp; j < FRAG_TILE; j += 256 / FRAG_G) {
        const uint64_t i = tile + j;
        if (i >= b.n)
            break;
        if (port[i] != 2)
            continue;
        uint8_t *ip = b.base + pkt_off(b, i);
        const uint32_t caplen = pkt_len(b, i);
        const FragPlan p = frag_plan(ip, caplen, f.mtu, f.honor_df);   // group-uniform; port 2
        const uint32_t nw = p.hlen >> 2;
        uint32_t dw = gl < nw ? ld_u32_unaligned(ip + 4 * gl) : 0u;
        // the first fragment's header (112-120)
        const uint32_t w1 = __shfl(dw, g0 + 1, 64);
        const bool df = (w1 >> 16) & 0x40, had_mf = (w1 >> 16) & 0x20;
        if (gl == 0)
            dw = (dw & 0xFFFF) | (bswap16(p.hlen + (uint32_t)p.first_dlen) << 16);
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
        hdr[grp][gl] = dw;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (gl == 0) {
            const uint32_t h0 = hdr[grp][0], h1 = hdr[grp][1], h2 = hdr[grp][2];
            st_u16(ip + 2, h0 >> 16);
            st_u16(ip + 4, h1 & 0xFFFF);
            st_u16(ip + 6, h1 >> 16);
            st_u16(ip + 10, h2 >> 16);
            // copied options (53-86) into optw[], EOL-padded
            const uint8_t *hb = (const uint8_t *)hdr[grp];
            uint8_t *ob = (uint8_t *)optw[grp];
            uint32_t k = 20, o = 0;
            while (k < p.hlen) {
                const uint32_t t = hb[k];
                if (t == 1) {
                    k++;
                    continue;
                }
                if (t == 0 || k + 1 == p.hlen)
                    break;
                const uint32_t l = hb[k + 1];
                if (l < 2 || k + l > p.hlen)
                    break;
                if (t & 0x80)
                    for (uint32_t c = 0; c < l; c++)
                        ob[o++] = hb[k + c];
                k += l;
            }
            while (o & 3)
                ob[o++] = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the fragment header template: base 20 bytes of the rewritten
        // header + copied options (140-144)
        const uint32_t qw = p.out_hlen >> 2;
        uint32_t tpl = 0;
        if (gl < 5)
            tpl = hdr[grp][gl];
        else if (gl < qw)
            tpl = optw[grp][gl - 5];
        if (gl == 0)
            tpl = (tpl & ~0xFu) | (qw & 0xF);                // ip_hl (144)
        const uint32_t off_first = bswap16(hdr[grp][1] >> 16);  // ntohs(ip->ip_off) after 112-118
        uint64_t fidx = fbase + pn[j];
        uint64_t bpos = bbase + pb[j];
        const uint64_t src_end = (uint64_t)ip + caplen;
        for (uint32_t k = 0; k < p.nextra; k++) {
            const int off = p.first_dlen + (int)(k * p.step);
            uint32_t dlen = p.step;
            if ((int)dlen + off > p.in_dlen)                       // 132-133
                dlen = (uint32_t)(p.in_dlen - off);
            const uint32_t qlen = p.out_hlen + dlen, slot = slot16(qlen);
            const bool fits = fidx < f.max_frags && bpos + slot <= f.arena_bytes;
            if (fits) {
                uint8_t *q = f.arena + bpos;
                uint32_t h = tpl;
                if (gl == 0)
                    h = (h & 0xFFFF) | (bswap16(qlen) << 16);     // 148
                if (gl == 1) {
                    uint32_t fo = (off_first + ((uint32_t)off >> 3)) & 0xFFFF;   // 145
                    if ((int)dlen + off >= p.in_dlen && !had_mf)  // 146-147
                        fo &= ~0x2000u;
                    h = (h & 0xFFFF) | (bswap16(fo) << 16);
                }
                if (gl == 2)
                    h &= 0xFFFF;                                  // 149
                const uint32_t s = group_header_cksum(h, gl, qw);
                if (gl == 2)
                    h |= s << 16;                                 // 150
                if (gl < qw)
                    st_u32(q + 4 * gl, h);
                // payload (142): FRAG_U 16 B chunks per lane in flight
                const uint64_t src0 = (uint64_t)ip + p.hlen + (uint32_t)off;
                const uint64_t hi = src0 + dlen < src_end ? src0 + dlen : src_end;
                const uint32_t nch = (dlen + 15) / 16;
                for (uint32_t c0 = 0; c0 < nch; c0 += FRAG_G * FRAG_U) {
                    u32x4 v[FRAG_U];
#pragma unroll
                    for (int u = 0; u < FRAG_U; u++) {
                        const uint32_t c = c0 + u * FRAG_G + gl;
                        v[u] = c < nch ? load16_guarded(src0 + 16ull * c, hi) : u32x4{0, 0, 0, 0};
                    }
#pragma unroll
                    for (int u = 0; u < FRAG_U; u++) {
                        const uint32_t c = c0 + u * FRAG_G + gl;
                        if (c >= nch)
                            continue;
                        const uint32_t at = p.out_hlen + 16 * c;  // 4-aligned; the slot ends at `slot`
                        if (at + 16 <= slot) {
                            *(__attribute__((address_space(1))) u32x4_a4 *)(q + at) = v[u];
                        } else {
#pragma unroll
                            for (int d = 0; d < 4; d++)
                                if (at + 4 * d < slot)
                                    st_u32(q + at + 4 * d, v[u][d]);
                        }
                    }
                }
                if (gl == 0) {
                    f.frag_off[fidx] = bpos;
                    f.frag_len[fidx] = qlen;
                    f.frag_src[fidx] = (uint32_t)i;
                }
            }
            fidx++;
            bpos += slot;
        }
    }
}

} // namespace clk
