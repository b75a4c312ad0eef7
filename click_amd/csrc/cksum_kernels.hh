// cksum_kernels.hh -- hand-written gfx950 kernels for Click's checksum path.
//
// Two geometries (DESIGN.md "Kernels"):
//   * lane-per-packet  (ip_header_kernel): IP header check/set, 20-60 bytes
//     per packet; each lane reads its header with a dwordx4 + dwordx2 from
//     the dword-aligned address below it and realigns with v_alignbyte.
//   * group-per-packet (l4_kernel, range_kernel): G lanes (G | 64) share one
//     packet; lane l of the group loads 16-byte chunks l, l+G, ... of the
//     packet with K loads in flight per pass, masks the bytes outside the
//     summed range, keeps even/odd-address byte sums (cksum_device.hh), and
//     the group reduces them with xor shuffles.  Loads of a wave instruction
//     cover 16*G contiguous bytes of each of its 64/G packets.
// Every kernel is a grid-stride loop over packets whose exit condition every
// lane reaches; no inter-workgroup communication.
#pragma once
#include "cksum_device.hh"

#ifndef CLK_NT_LOADS
#define CLK_NT_LOADS -1    // nontemporal chunk loads: -1 auto (fixed-geometry Check kernels), 0 never, 1 always
#endif
#ifndef CLK_NT_STORES
#define CLK_NT_STORES 0    // tuning knob: nontemporal checksum-field stores
#endif
#ifndef CLK_SWPE
#define CLK_SWPE 4         // packet-stream Set kernels: request this many waves per SIMD (the dense path's LDS allows 4 at CLK_SKV 4)
#endif
#ifndef CLK_STREAM_NT_CHECK
#define CLK_STREAM_NT_CHECK 0   // packet-stream Check: nontemporal chunk loads (tuning knob)
#endif
#ifndef CLK_SWPE_CHECK
#define CLK_SWPE_CHECK 5   // ... the Check kernels, with 4 chunks per lane per pass (CLK_SKV_CHECK; LDS allows 5)
#endif
#ifndef CLK_DENSE
#define CLK_DENSE 1        // packet-stream Check: dense runs load coalesced + nontemporal, through LDS
#endif
#ifndef CLK_DENSE_SET
#define CLK_DENSE_SET 1    // ... the Set kernels too (with XCD-contiguous runs and 4 chunks per lane: C4 Set 5.08 vs 5.33 ms)
#endif
#ifndef CLK_L4_RUNS
#define CLK_L4_RUNS 1      // l4_kernel: a workgroup owns runs of packets and stores their outputs whole
#endif
#ifndef CLK_XCD_BLOCKS
#define CLK_XCD_BLOCKS 0   // tuning: every run loop walks XCD-contiguous runs (reads: C3 / C4 / C5 Check 2-8 % slower)
#endif
#ifndef CLK_XCD_SET
#define CLK_XCD_SET 1      // the fused packet-stream Set does (C4 Set 5.38 vs 6.01 ms: DESIGN.md §6)
#endif
#ifndef CLK_L4_RUNS_SET_G
#define CLK_L4_RUNS_SET_G 16   // Set kernels use runs from this G up (C5 -6 %; C3 -5 % with nontemporal scatter stores: DESIGN.md §6)
#endif

// Load-site hooks: the identity in the library.  tools/addr_check builds a
// copy of these sources in which each hook checks its address against a
// registered window; nothing of that check is compiled here.
#define CLK_CHK(a, n, site) (a)
#define CLK_CHK_IF(cond, site, a) do { } while (0)

namespace clk {

// The workgroup's place in the run order.  XCD-contiguous (XCD): workgroup b
// (dispatched to XCD b % 8) takes position (b % 8) * q + min(b % 8, r) + b / 8
// (q = grid / 8, r = grid % 8), a bijection under which each XCD walks one
// contiguous share of the runs.  The two-byte field stores of neighbouring
// packets in different runs (IMIX packets share 64 B blocks) then meet in one
// L2 and leave it merged, instead of reaching the memory controller as
// partial-block writes from two XCDs.  Read-only kernels keep the dealt
// order: with eight separate read fronts they run 2-8 % slower.
template <bool XCD>
__device__ __forceinline__ uint32_t run_block()
{
    if (!XCD)
        return blockIdx.x;
    const uint32_t g = gridDim.x, x = blockIdx.x & 7, q = g >> 3, r = g & 7;
    return x * q + (x < r ? x : r) + (blockIdx.x >> 3);
}

// NT: nontemporal loads (once-read stream; measured faster for the
// fixed-geometry Check kernels, slower for the Set and packet-stream ones,
// DESIGN.md §6).
template <bool NT_AUTO>
struct UseNT {
    static constexpr bool value = CLK_NT_LOADS < 0 ? NT_AUTO : CLK_NT_LOADS != 0;
};

struct BatchArgs {
    uint8_t *base;
    const uint64_t *off;
    uint64_t stride;
    const uint32_t *len;
    uint32_t fixed_len;
    uint64_t n;
};

__device__ __forceinline__ uint64_t pkt_off(const BatchArgs &b, uint64_t i)
{
    return b.off ? b.off[i] : i * b.stride;
}
__device__ __forceinline__ uint32_t pkt_len(const BatchArgs &b, uint64_t i)
{
    return b.len ? b.len[i] : b.fixed_len;
}

enum Proto { ICMP = 1, UDP = 17, TCP = 6 };

// The packet-stream kernel's packet-length bound (cksum_api.hip use_stream).
constexpr uint32_t STREAM_MAX_LEN = 1u << 24;

// codes (include/click_amd_cksum.h)
constexpr uint32_t OK = 0;
constexpr uint32_t IP_MINISCULE = 1, IP_BAD_VERSION = 2, IP_BAD_HLEN = 3, IP_BAD_IP_LEN = 4,
                   IP_BAD_CHECKSUM = 5, IP_BAD_SADDR = 6;
constexpr uint32_t L4_NOT_PROTO = 1, L4_BAD_LENGTH = 2, L4_BAD_CHECKSUM = 3;
constexpr uint32_t SET_OUTPUT1 = 1, SET_KILL = 2;
constexpr uint32_t TTL_EXPIRED = 1, TTL_UNCHANGED = 2;

// ---------------------------------------------------------------------------
// IP header: CheckIPHeader (checkipheader.cc:161-226) and SetIPChecksum
// (setipchecksum.cc:74-95), one lane per packet.
// ---------------------------------------------------------------------------
enum IpMode { IP_CHECK = 0, IP_CHECK_NOCKSUM = 1, IP_SET = 2 };

// Field stores of the one-lane-per-packet rewriting kernels (SetIPChecksum,
// DecIPTTL).  CLK_FIELD_NT: nontemporal, so the partial-block write reaches
// HBM inside the kernel instead of lingering dirty in the caches until the
// next kernel's reads evict it.
#ifndef CLK_FIELD_NT
#define CLK_FIELD_NT 1     // C2 SetIPChecksum 0.4065 vs 0.4116 ms, DecIPTTL 0.4083 vs 0.4122
#endif
__device__ __forceinline__ void field_st_u16(uint8_t *p, uint32_t v)
{
    if (CLK_FIELD_NT && ((uint64_t)p & 1) == 0)
        __builtin_nontemporal_store((uint16_t)v, (__attribute__((address_space(1))) uint16_t *)p);
    else
        st_u16(p, v);
}
__device__ __forceinline__ void field_st_u32(uint8_t *p, uint32_t v)    // 4-byte aligned p
{
    if (CLK_FIELD_NT)
        __builtin_nontemporal_store(v, (__attribute__((address_space(1))) uint32_t *)p);
    else
        *(__attribute__((address_space(1))) uint32_t *)p = v;
}

#ifndef CLK_IPH_PAIR
#define CLK_IPH_PAIR 1   // C2 CheckIPHeader 0.168 vs 0.182 ms with one lane per packet
#endif
template <int MODE>
__global__ void __launch_bounds__(256) ip_header_kernel(BatchArgs b, uint32_t offset,
                                                        const uint32_t *badsrc, uint32_t nbadsrc,
                                                        const uint32_t *gooddst, uint32_t ngooddst,
                                                        uint8_t *out_code, uint16_t *out_sum)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    // PAIR (Check): two lanes per packet, one 12 B load each, so one
    // request per packet carries its header (CLK_IPH_PAIR)
    constexpr bool PAIR = MODE != IP_SET && CLK_IPH_PAIR;
    constexpr uint32_t PL = PAIR ? 2 : 1;
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    typedef __attribute__((address_space(1))) u32x3 __attribute__((aligned(4))) g3;
    // the packet of work item j: its header address and length after OFFSET
    auto locate = [&](uint64_t j, uint8_t *&ip, uint32_t &plen) {
        const uint64_t i = PAIR ? j >> 1 : j;
        ip = b.base + pkt_off(b, i);
        plen = pkt_len(b, i);
        if (MODE != IP_SET) {           // data() + OFFSET, length() - OFFSET (checkipheader.cc:163-164)
            ip += offset;
            plen -= offset;
        }
    };
    // PAIR: lane 0 of the pair loads dwords 0-2 of the dword below ip, lane 1
    // dwords 3-5 (ip not 4-aligned) or 2-4
    auto pair_load = [&](uint64_t j, const uint8_t *ip) -> u32x3 {
        const uint64_t a = (uint64_t)ip;
        const uint32_t sh = (uint32_t)(a & 3);
        const uint8_t *q = (const uint8_t *)(a & ~3ull);
        return __builtin_nontemporal_load((const g3 *)(q + (((uint32_t)j & 1) ? (sh ? 12 : 8) : 0)));
    };
    auto one = [&](uint64_t j, uint8_t *ip, uint32_t plen, u32x3 m) {
        const uint64_t i = PAIR ? j >> 1 : j;
        uint32_t code = OK, stored = 0;
        if ((int)plen < 20) {           // checkipheader.cc:168-170 / setipchecksum.cc:82
            code = MODE == IP_SET ? SET_KILL : IP_MINISCULE;
        } else {
            // bytes [ip, ip+20): dwordx4 + dwordx2 from the dword below ip
            const uint64_t a = (uint64_t)ip;
            const uint32_t sh = (uint32_t)(a & 3);
            const uint8_t *q = (const uint8_t *)(a & ~3ull);
            u32x4 d0;
            uint32_t d4, d5;
            if (PAIR) {
                const uint32_t odd = (uint32_t)j & 1;
                const uint32_t o0 = __shfl_xor(m.x, 1, 64), o1 = __shfl_xor(m.y, 1, 64), o2 = __shfl_xor(m.z, 1, 64);
                const u32x3 lo = odd ? u32x3{o0, o1, o2} : m, hi = odd ? m : u32x3{o0, o1, o2};
                d0 = u32x4{lo.x, lo.y, lo.z, sh ? hi.x : hi.y};
                d4 = sh ? hi.y : hi.z;
                d5 = sh ? hi.z : 0u;
            } else if (UseNT<MODE != IP_SET>::value) {
                typedef __attribute__((address_space(1))) u32x4_a4 g4;
                typedef __attribute__((address_space(1))) uint32_t g1;
                d0 = __builtin_nontemporal_load((const g4 *)q);
                d4 = __builtin_nontemporal_load((const g1 *)(q + 16));
                d5 = sh ? __builtin_nontemporal_load((const g1 *)(q + 20)) : 0u;
            } else {
                d0 = gload16_a4((uint64_t)q);
                d4 = gload4((uint64_t)(q + 16));
                d5 = sh ? gload4((uint64_t)(q + 20)) : 0u;
            }
            uint32_t h[5];
            h[0] = __builtin_amdgcn_alignbyte(d0[1], d0[0], sh);
            h[1] = __builtin_amdgcn_alignbyte(d0[2], d0[1], sh);
            h[2] = __builtin_amdgcn_alignbyte(d0[3], d0[2], sh);
            h[3] = __builtin_amdgcn_alignbyte(d4, d0[3], sh);
            h[4] = __builtin_amdgcn_alignbyte(d5, d4, sh);
            const uint32_t b0 = h[0] & 0xFF;
            const uint32_t hlen = (b0 & 0xF) << 2;
            uint32_t sum = 0;
#pragma unroll
            for (int k = 0; k < 5; k++)
                sum = dot_words(h[k], sum);
            if (MODE == IP_SET) {
                if (hlen < 20 || hlen > plen) {
                    code = SET_KILL;
                } else {
                    for (uint32_t o = 20; o < hlen; o += 4) {
                        const uint32_t w = ld_u32_unaligned(ip + o);
                        sum += (w & 0xFFFF) + (w >> 16);
                    }
                    sum -= h[2] >> 16;                 // ip_sum = 0 (setipchecksum.cc:85)
                    stored = in_cksum_fold(sum);       // setipchecksum.cc:86
                    field_st_u16(ip + 10, stored);
                }
            } else {
                const uint32_t len = bswap16(h[0] >> 16);
                if ((b0 >> 4) != 4)
                    code = IP_BAD_VERSION;
                else if (hlen < 20)
                    code = IP_BAD_HLEN;
                else if (len > plen || len < hlen)
                    code = IP_BAD_IP_LEN;
                else {
                    if (MODE == IP_CHECK) {
                        for (uint32_t o = 20; o < hlen; o += 4) {
                            const uint32_t w = ld_u32_unaligned(ip + o);
                            sum += (w & 0xFFFF) + (w >> 16);
                        }
                        if (in_cksum_fold(sum) != 0)
                            code = IP_BAD_CHECKSUM;
                    }
                    if (code == OK && nbadsrc) {       // checkipheader.cc:204-206
                        bool bad = false, good = false;
                        for (uint32_t k = 0; k < nbadsrc; k++)
                            bad |= badsrc[k] == h[3];
                        if (bad) {
                            for (uint32_t k = 0; k < ngooddst; k++)
                                good |= gooddst[k] == h[4];
                            if (!good)
                                code = IP_BAD_SADDR;
                        }
                    }
                }
            }
        }
        if (!PAIR || (j & 1) == 0)
            out_code[i] = (uint8_t)code;
        if (MODE == IP_SET && out_sum)
            out_sum[i] = (uint16_t)stored;
    };
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < PL * b.n; j += nthreads) {
        uint8_t *ip;
        uint32_t plen;
        locate(j, ip, plen);
        one(j, ip, plen, PAIR && (int)plen >= 20 ? pair_load(j, ip) : u32x3{0, 0, 0});
    }
}

// ---------------------------------------------------------------------------
// Group-per-packet range sum: G lanes, K chunk loads per lane per pass.
// Returns the A/B byte sums of [s, s+len) (len <= 0: empty), reduced over the
// group.  `first` holds the chunks of pass 0, already loaded by the caller
// so that they were in flight while the caller parsed the header.
// ---------------------------------------------------------------------------

template <int G, int K, bool NT = false>
__device__ __forceinline__ void load_pass(const uint8_t *c0, uint32_t nch, uint32_t pass, uint32_t gl,
                                          u32x4 (&v)[K])
{
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = pass * (G * K) + (uint32_t)k * G + gl;
        if (NT)
            v[k] = idx < nch ? __builtin_nontemporal_load((const u32x4 *)(c0 + 16ull * idx)) : u32x4{0, 0, 0, 0};
        else
            v[k] = idx < nch ? gload16((uint64_t)(c0 + 16ull * idx)) : u32x4{0, 0, 0, 0};
    }
}

template <int G, int K, bool NT = false>
__device__ __forceinline__ uint32_t group_range_sum(const uint8_t *c0, uint32_t nch, uint32_t gl,
                                                    const u32x4 (&first)[K], uint64_t s, int len)
{
    RangeAcc acc{0, 0};
    const bool odd = (s & 1) != 0;
    const int rel0 = (int)((uint64_t)c0 - s);       // chunk 0 relative to s (<= 0)
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = (uint32_t)k * G + gl;
        chunk_accumulate(first[k], rel0 + 16 * (int)idx, len, odd, acc);
    }
    const uint32_t npass = (nch + G * K - 1) / (G * K);
    for (uint32_t p = 1; p < npass; p++) {
        u32x4 v[K];
        load_pass<G, K, NT>(c0, nch, p, gl, v);
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint32_t idx = p * (G * K) + (uint32_t)k * G + gl;
            chunk_accumulate(v[k], rel0 + 16 * (int)idx, len, odd, acc);
        }
    }
#pragma unroll
    for (int m = 1; m < G; m <<= 1) {
        acc.s0 += __shfl_xor(acc.s0, m, 64);
        if (odd)
            acc.s1 += __shfl_xor(acc.s1, m, 64);
    }
    return word_sum(acc, odd);
}

// clk_in_cksum: click_in_cksum(base+off_i, len_i) (lib/in_cksum.c:20-51).
// RUNS (packets 0..n-1): a workgroup owns max(64, 256/G) consecutive
// packets and writes their sums whole after one barrier, as l4_kernel does;
// nontemporal loads (once-read stream).  Else the grid-stride loop, which
// for the multi-pass geometry hint paths.
template <int G, int K, bool RUNS>
__global__ void __launch_bounds__(256) range_kernel(BatchArgs b, uint16_t *out_sum)
{
    const uint32_t lane = threadIdx.x & 63, gl = lane & (G - 1);
    constexpr bool NT = UseNT<true>::value;
    auto one = [&](uint64_t i) -> uint32_t {
        const uint8_t *p = b.base + pkt_off(b, i);
        const int len = (int)pkt_len(b, i);
        const uint64_t s = (uint64_t)p;
        const uint8_t *c0 = (const uint8_t *)(s & ~15ull);
        const uint32_t nch = len > 0 ? (uint32_t)(((s + (uint64_t)len + 15) & ~15ull) - (uint64_t)c0) / 16 : 0;
        u32x4 v[K];
        load_pass<G, K, NT>(c0, nch, 0, gl, v);
        return in_cksum_fold(group_range_sum<G, K, NT>(c0, nch, gl, v, s, len));
    };
    if (RUNS) {
        constexpr uint32_t PPB = 256 / G, RB = PPB < 64 ? 64 : PPB;
        __shared__ uint16_t r_sum[RB];
        const uint64_t nruns = (b.n + RB - 1) / RB;
        for (uint64_t run = run_block<CLK_XCD_BLOCKS != 0>(); run < nruns; run += gridDim.x) {       // uniform per workgroup
            const uint64_t i0 = run * RB;
#pragma unroll 1
            for (uint32_t p = 0; p < RB / PPB; p++) {
                const uint32_t q = p * PPB + threadIdx.x / G;
                if (i0 + q < b.n) {
                    const uint32_t r = one(i0 + q);
                    if (gl == 0)
                        r_sum[q] = (uint16_t)r;
                }
            }
            __syncthreads();
            if (threadIdx.x < RB && i0 + threadIdx.x < b.n)
                out_sum[i0 + threadIdx.x] = r_sum[threadIdx.x];
            __syncthreads();
        }
        return;
    }
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / G;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; i < b.n; i += groups) {
        const uint32_t r = one(i);
        if (gl == 0)
            out_sum[i] = (uint16_t)r;
    }
}

// ---------------------------------------------------------------------------
// UDP / TCP check and set (checkudpheader.cc:84-107, setudpchecksum.cc:37-69,
// checktcpheader.cc:85-107, settcpchecksum.cc:44-75), split in three steps
// shared by the fixed-geometry kernel (l4_kernel) and the packet-stream
// kernel (l4_stream_kernel, which parses from its LDS stash: l4_parse_words):
//   l4_parse  -- header checks; the summed range [nh+hl, nh+hl+rlen)
//   (range sum by the caller)
//   l4_finish -- Set field correction, fold, pseudo-header, verdict / store
// The header parse reads the first 28 (UDP) / 40 (TCP) bytes as aligned
// dwords and is speculative on ip_hl = 5; other header lengths re-read.
// ---------------------------------------------------------------------------
// What the finish needs once the header is parsed.  The pseudo-header is
// reduced to one partial sum at parse time (ph), and a Set's corrections
// (its zeroed field, FIXOFF's rewritten byte) to one u32 added to the range
// sum (adj), so few registers stay live across the payload sum.
struct L4State {
    uint32_t code;
    int rlen;            // summed range length (int, as click_in_cksum's)
    uint32_t plen_ph;    // packet_len for the pseudo-header
    uint32_t hl;
    uint32_t ph;         // src + dst (+ SSRR/LSRR) halves + htons(len) + htons(proto)
    uint32_t adj;        // Set: added to the range sum (mod 2^32)
    uint32_t new_b12;
    uint32_t caplen;
    bool fix, summing;
};

template <int PROTO>
struct L4Hdr {
    static constexpr int DW = PROTO == TCP ? 11 : 8;   // aligned dwords covering bytes [0, 40) / [0, 28)
};

// Parse from the header dwords d[k] = the aligned dword at (nh & ~3) + 4k
// (0 at and beyond nh + caplen).
template <int PROTO, bool SET>
__device__ __forceinline__ void l4_parse_words(uint8_t *nh, uint32_t caplen, int fixoff,
                                               const uint32_t (&d)[L4Hdr<PROTO>::DW], L4State &st)
{
    constexpr int HDR_DW = L4Hdr<PROTO>::DW;
    constexpr uint32_t FIELD = PROTO == UDP ? 6 : 16;
    const uint32_t sh = (uint32_t)((uint64_t)nh & 3);
    uint32_t h[HDR_DW - 1];                 // h[k] = bytes [4k, 4k+4) of the header, LE
#pragma unroll
    for (int k = 0; k < HDR_DW - 1; k++)
        h[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);

    const uint32_t b0 = h[0] & 0xFF;
    const uint32_t hl = (b0 & 0xF) << 2;
    const uint32_t ip_len = bswap16(h[0] >> 16);
    const uint32_t proto = (h[2] >> 8) & 0xFF;
    const bool isfrag = (bswap16(h[1] >> 16) & 0x3FFF) != 0;   // IP_ISFRAG, ip.h:121
    auto tbyte = [&](uint32_t r) -> uint32_t {    // byte hl + r (speculated hl = 20)
        if (hl == 20) {
            const uint32_t o = 20 + r;
            return (h[o >> 2] >> (8 * (o & 3))) & 0xFF;
        }
        const uint32_t v = ld_u8(nh + hl + r);
        vm_retire();
        return v;
    };
    st.code = OK;
    st.rlen = 0;
    st.plen_ph = 0;
    st.caplen = caplen;
    st.hl = hl;
    st.new_b12 = 0;
    st.adj = st.ph = 0;
    uint32_t fix_delta = 0;
    st.fix = false;
    if (caplen < 20) {
        st.code = PROTO == UDP ? (SET ? SET_OUTPUT1 : L4_BAD_LENGTH) : (SET ? SET_KILL : L4_BAD_LENGTH);
    } else if (PROTO == UDP && !SET) {
        if (proto != 17)
            st.code = L4_NOT_PROTO;
        else if (caplen < hl + 8)
            st.code = L4_BAD_LENGTH;
        else {
            const uint32_t ulen = (tbyte(4) << 8) | tbyte(5);
            if (ulen < 8 || caplen < ulen + hl)
                st.code = L4_BAD_LENGTH;
            else if ((tbyte(6) | tbyte(7)) != 0) {      // uh_sum == 0: not checked (checkudpheader.cc:100)
                st.rlen = (int)ulen;
                st.plen_ph = ulen;
            }
        }
    } else if (PROTO == UDP && SET) {
        const int tlen = (int)caplen - (int)hl;
        if (isfrag || tlen < 8)
            st.code = SET_OUTPUT1;
        else {
            const uint32_t ulen = (tbyte(4) << 8) | tbyte(5);
            if (tlen < (int)ulen)
                st.code = SET_OUTPUT1;
            else {
                st.rlen = (int)ulen;
                st.plen_ph = ulen;
            }
        }
    } else if (PROTO == ICMP) {          // checkicmpheader.cc:83-141 (check only)
        if (proto != 1)
            st.code = L4_NOT_PROTO;
        else if (caplen < hl || caplen - hl < 8)   // guard (icmp_len would wrap) / 93-94
            st.code = L4_BAD_LENGTH;
        else {
            const uint32_t ilen = caplen - hl, type = tbyte(0);
            bool bad = false;                    // 96-134
            if (type == 3 || type == 4 || type == 5 || type == 11 || type == 12)
                bad = ilen < 8 + 28;
            else if (type == 13 || type == 14)
                bad = ilen != 20;
            else if (type == 15 || type == 16)
                bad = ilen != 8;
            if (bad)
                st.code = L4_BAD_LENGTH;
            else {
                st.rlen = (int)ilen;
                st.plen_ph = ilen;
            }
        }
    } else if (PROTO == TCP && !SET) {
        if (proto != 6)
            st.code = L4_NOT_PROTO;
        else if (caplen < hl + 13)
            st.code = L4_BAD_LENGTH;
        else {
            const uint32_t len = ip_len - hl;
            const uint32_t thl = (tbyte(12) >> 4) << 2;
            if (thl < 20 || len < thl || caplen < len + hl)
                st.code = L4_BAD_LENGTH;
            else {
                st.rlen = (int)len;
                st.plen_ph = len;
            }
        }
    } else {   // TCP set
        if (hl > caplen)
            st.code = SET_KILL;
        else {
            const uint32_t plen = ip_len - hl, tlen = caplen - hl;
            if (plen < 20 || plen > tlen)
                st.code = SET_KILL;
            else {
                st.rlen = (int)plen;
                st.plen_ph = plen;
                if (fixoff) {                   // settcpchecksum.cc:57-63
                    const uint32_t ob = tbyte(12);
                    const uint32_t off = (ob >> 4) << 2;
                    if (off < 20) {
                        st.new_b12 = (ob & 0x0F) | (5u << 4);
                        st.fix = true;
                    } else if (off > plen && !isfrag) {
                        st.new_b12 = (ob & 0x0F) | (((plen >> 2) & 0xF) << 4);
                        st.fix = true;
                    }
                    if (st.fix)
                        fix_delta = st.new_b12 - ob;
                }
            }
        }
    }
    st.summing = (st.code == OK) && (st.rlen != 0 || st.plen_ph != 0 || SET);
    if (SET && st.summing) {
        // the field is zeroed before summing (setudpchecksum.cc:64,
        // settcpchecksum.cc:65): remove its bytes that lie in range; FIXOFF's
        // rewritten th_off byte is summed as rewritten (57-63)
        const uint32_t fb0 = (int)FIELD < st.rlen ? tbyte(FIELD) : 0;
        const uint32_t fb1 = (int)FIELD + 1 < st.rlen ? tbyte(FIELD + 1) : 0;
        st.adj = (st.fix && 12 < st.rlen ? fix_delta : 0u) - (fb0 + (fb1 << 8));
    }
    if (PROTO != ICMP && st.summing) {
        uint32_t s2 = h[3], d2 = h[4];
        if (SET && hl < 20) {
            // ip_hl < 5: the transport header overlaps the IP header.  The
            // reference zeroes the field (and FIXOFF rewrites th_off)
            // BEFORE the pseudo-header reads ip_src/ip_dst, and the option
            // walk is empty (in_cksum.c:86-88), so patch those bytes in.
            auto patch = [&](uint32_t pos, uint32_t val) {
                if (pos >= 12 && pos < 16)
                    s2 = (s2 & ~(0xFFu << (8 * (pos - 12)))) | (val << (8 * (pos - 12)));
                else if (pos >= 16 && pos < 20)
                    d2 = (d2 & ~(0xFFu << (8 * (pos - 16)))) | (val << (8 * (pos - 16)));
            };
            if (st.fix)
                patch(hl + 12, st.new_b12);
            patch(hl + FIELD, 0);
            patch(hl + FIELD + 1, 0);
        } else if ((b0 & 0xF) != 5) {
            d2 = route_dst(nh, hl, d2);              // ip.h:156-159 -> in_cksum.c:83-108
        }
        st.ph = pseudohdr_partial(s2, d2, proto, st.plen_ph);
    }
}

template <int PROTO, bool SET>
__device__ __forceinline__ void l4_parse(uint8_t *nh, uint32_t caplen, int fixoff, L4State &st)
{
    constexpr int HDR_DW = L4Hdr<PROTO>::DW;
    const uint64_t a = (uint64_t)nh;
    const uint8_t *q = (const uint8_t *)(a & ~3ull);
    const uint64_t end = a + caplen;
    uint32_t d[HDR_DW];
#pragma unroll
    for (int k = 0; k < HDR_DW; k++)
        d[k] = (uint64_t)(q + 4 * k) < end ? gload4((uint64_t)(q + 4 * k)) : 0u;
    l4_parse_words<PROTO, SET>(nh, caplen, fixoff, d, st);
}

// The header dwords from the group's pass-0 registers instead of loads of
// their own (CLK_HDR_FROM_CHUNKS, G >= 4): lanes 0..3 of the group hold
// chunks 0..3 = [c0, c0 + 64) in v[0], which cover every aligned header
// dword (at most 3 + 11 dwords past c0).  Same values as l4_parse: dwords at
// or past nh + caplen read as 0.
// Used by the two-phase Set compute pass (C3 Set 5.30 -> 5.14 ms); the
// Check kernels keep their own header loads (C3 Check 3.83 vs 3.86 ms).
#ifndef CLK_HDR_FROM_CHUNKS
#define CLK_HDR_FROM_CHUNKS 1
#endif
template <int PROTO, bool SET, int G, int K>
__device__ __forceinline__ void l4_parse_from_chunks(uint8_t *nh, uint32_t caplen, int fixoff, uint64_t c0,
                                                     uint32_t lane, const u32x4 (&v)[K], L4State &st)
{
    constexpr int HDR_DW = L4Hdr<PROTO>::DW;
    const int gbase = (int)(lane & ~(uint32_t)(G - 1));
    uint32_t D[16];
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int w = 0; w < 4; w++)
            D[4 * q + w] = __shfl(v[0][w], gbase + q, 64);
    const uint64_t a = (uint64_t)nh, qa = a & ~3ull, end = a + caplen;
    const uint32_t q0 = (uint32_t)(qa - c0) >> 2;           // 0..3
    uint32_t d[HDR_DW];
#pragma unroll
    for (int k = 0; k < HDR_DW; k++) {
        const uint32_t x = q0 == 0 ? D[k] : q0 == 1 ? D[k + 1] : q0 == 2 ? D[k + 2] : D[k + 3];
        d[k] = qa + 4 * k < end ? x : 0u;
    }
    l4_parse_words<PROTO, SET>(nh, caplen, fixoff, d, st);
}

// Finish one packet from its range sum.  `writer` lanes store.
// Replace byte `val` at absolute address `at` if it lies in the 16 bytes of
// v at absolute address `va`.
__device__ __forceinline__ void patch_byte(u32x4 &v, uint64_t va, uint64_t at, uint32_t val)
{
    const uint64_t rel = at - va;
    if (rel < 16) {
        const uint32_t d = (uint32_t)rel >> 2, sh = 8 * ((uint32_t)rel & 3);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (k == d)
                v[k] = (v[k] & ~(0xFFu << sh)) | ((val & 0xFF) << sh);
    }
}

// Fused Set store of the field bytes alone (and FIXOFF's th_off byte) by the
// writer lane, when the field's 64 B block cannot be stored whole.  (HBM
// rewrites a partially written 64 B block by read-modify-write: alone, one
// 2 B store per 1536 B slot runs at 21.6 G stores/s and a full 64 B block at
// 39 G/s, tools/probes/write_probe.hip.)
template <int PROTO>
__device__ __forceinline__ void set_field_store(uint8_t *nh, const L4State &st, uint32_t r, bool writer)
{
    constexpr uint32_t FIELD = PROTO == UDP ? 6 : 16;
    if (writer) {
        if (st.fix)
            nh[st.hl + 12] = (uint8_t)st.new_b12;
        st_u16(nh + st.hl + FIELD, r);
    }
}

// Set stores from registers (CLK_SET_REGBLK).  When the 64 B-aligned block
// holding the checksum field lies inside the packet, the lanes that loaded
// its four 16 B chunks in pass 0 still hold them: they patch the field (and
// the FIXOFF byte) and store the whole block, so HBM sees a full-block write
// and no read-modify-write, with no re-read.  Returns false when the block
// is not available (the caller stores the field bytes alone).
//   v[k] holds chunk k*G + gl of [c0, ...) (group_range_sum's layout); the
//   block's chunks are q0..q0+3 with q0 <= 4, so only v[k] with k*G < 8 can
//   hold one and the rest need not stay live across later passes.
#ifndef CLK_SET_REGBLK
#define CLK_SET_REGBLK 1
#endif
__device__ __forceinline__ void store_block16(uint64_t ca, u32x4 w)
{
    if (CLK_NT_STORES)
        __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4 *)ca);
    else
        *(__attribute__((address_space(1))) u32x4 *)ca = w;
}

template <int PROTO, int G, int K>
__device__ __forceinline__ bool set_block_store_regs(uint8_t *nh, const L4State &st, uint32_t r, uint32_t gl,
                                                     uint64_t c0, const u32x4 (&v)[K])
{
    constexpr uint32_t FIELD = PROTO == UDP ? 6 : 16;
    const uint64_t a = (uint64_t)nh, fa = a + st.hl + FIELD, xa = a + st.hl + 12;
    const uint64_t blk = fa & ~63ull;
    // fa + 1 in the block too (an odd field at byte 63 straddles two blocks)
    if (!(blk >= a && blk + 64 <= a + st.caplen && fa + 1 < blk + 64))
        return false;
    const uint32_t q0 = (uint32_t)(blk - c0) >> 4;          // 0..4
    if (q0 + 4 > (uint32_t)(G * K))
        return false;
    const bool fix_in = st.fix && xa >= blk && xa < blk + 64;
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (k * G >= 8)
            break;
        const uint32_t c = (uint32_t)(k * G) + gl;
        if (c >= q0 && c < q0 + 4) {
            u32x4 w = v[k];
            const uint64_t ca = c0 + 16ull * c;
            patch_byte(w, ca, fa, r);
            patch_byte(w, ca, fa + 1, r >> 8);
            if (fix_in)
                patch_byte(w, ca, xa, st.new_b12);
            store_block16(ca, w);
        }
    }
    if (gl == 0 && st.fix && !fix_in)
        nh[st.hl + 12] = (uint8_t)st.new_b12;
    return true;
}

// l4_finish with the fused Set store given as store(r).
// The same from the packet-stream kernel's LDS stash: chunks 0..HC-1 of
// [c0, ...) of this lane's packet.
template <int PROTO, int HC>
__device__ __forceinline__ bool set_block_store_stash(uint8_t *nh, const L4State &st, uint32_t r, uint64_t c0,
                                                      const u32x4 (&hs)[HC])
{
    constexpr uint32_t FIELD = PROTO == UDP ? 6 : 16;
    const uint64_t a = (uint64_t)nh, fa = a + st.hl + FIELD, xa = a + st.hl + 12;
    const uint64_t blk = fa & ~63ull;
    if (!(blk >= a && blk + 64 <= a + st.caplen && fa + 1 < blk + 64))
        return false;
    const uint32_t q0 = (uint32_t)(blk - c0) >> 4;
    if (q0 + 4 > (uint32_t)HC)
        return false;
    const bool fix_in = st.fix && xa >= blk && xa < blk + 64;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        u32x4 w = hs[q0 + q];
        const uint64_t ca = blk + 16ull * q;
        patch_byte(w, ca, fa, r);
        patch_byte(w, ca, fa + 1, r >> 8);
        if (fix_in)
            patch_byte(w, ca, xa, st.new_b12);
        store_block16(ca, w);
    }
    if (st.fix && !fix_in)
        nh[st.hl + 12] = (uint8_t)st.new_b12;
    return true;
}

// The same, patching the stash in LDS instead of storing: returns the
// block's address | its first stash chunk (0: not available), and the
// packet-stream kernel stores the patched blocks coalesced
// (CLK_STASH_COALESCE).
#ifndef CLK_STASH_COALESCE
#define CLK_STASH_COALESCE 1   // C4 Set 6.10 ms with nontemporal stores, 6.72 plain, 6.65 per-lane blocks
#endif
#ifndef CLK_STASH_NT
#define CLK_STASH_NT 1         // full 64 B nontemporal writes: no read-modify-write, nothing left dirty
#endif
template <int PROTO, int HC>
__device__ __forceinline__ uint64_t set_block_patch_stash(uint8_t *nh, const L4State &st, uint32_t r, uint64_t c0,
                                                          u32x4 (&hs)[HC])
{
    constexpr uint32_t FIELD = PROTO == UDP ? 6 : 16;
    const uint64_t a = (uint64_t)nh, fa = a + st.hl + FIELD, xa = a + st.hl + 12;
    const uint64_t blk = fa & ~63ull;
    if (!(blk >= a && blk + 64 <= a + st.caplen && fa + 1 < blk + 64))
        return 0;
    const uint32_t q0 = (uint32_t)(blk - c0) >> 4;
    if (q0 + 4 > (uint32_t)HC)
        return 0;
    const bool fix_in = st.fix && xa >= blk && xa < blk + 64;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const uint64_t ca = blk + 16ull * q;
        if (fa - ca < 16 || fa + 1 - ca < 16 || (fix_in && xa - ca < 16)) {
            u32x4 w = hs[q0 + q];
            patch_byte(w, ca, fa, r);
            patch_byte(w, ca, fa + 1, r >> 8);
            if (fix_in)
                patch_byte(w, ca, xa, st.new_b12);
            hs[q0 + q] = w;
        }
    }
    if (st.fix && !fix_in)
        nh[st.hl + 12] = (uint8_t)st.new_b12;
    return blk | q0;
}

// A packet's outputs: status code, two-phase work word, Set checksum.
struct L4Out {
    uint32_t code, work, sum;
};

template <int PROTO, bool SET, bool DEFER, typename Store>
__device__ __forceinline__ L4Out l4_result(uint8_t *nh, uint32_t sum, L4State &st, bool writer, Store &&store)
{
    L4Out o{0, 0, 0};
    if (st.code == OK && st.summing) {
        if (SET)
            sum += st.adj;
        const uint32_t csum = in_cksum_fold(sum);
        // click_in_cksum(icmph, icmp_len) != 0 (checkicmpheader.cc:136-138), else the pseudo-header
        const uint32_t r = PROTO == ICMP ? csum : pseudohdr_ph(csum, st.ph);
        if (SET) {
            o.sum = r;
            if (DEFER) {         // the field is written by field_scatter_kernel
                if (writer && st.fix)
                    nh[st.hl + 12] = (uint8_t)st.new_b12;
                o.work = 0x80000000u | (st.hl << 16) | r;
            } else {
                store(r);
            }
        } else if (r != 0) {
            st.code = L4_BAD_CHECKSUM;
        }
    }
    o.code = st.code;
    if (SET && DEFER && st.code != OK)
        o.work = st.code;    // bit 31 clear: no field; field_scatter_kernel writes the code
    return o;
}

template <int PROTO, bool SET, bool DEFER, typename Store>
__device__ __forceinline__ void l4_finish_with(uint8_t *nh, uint64_t i, uint32_t sum, L4State &st, bool writer,
                                               uint8_t *out_code, uint16_t *out_sum, uint32_t *work, Store &&store)
{
    const L4Out o = l4_result<PROTO, SET, DEFER>(nh, sum, st, writer, store);
    if (writer) {
        if (SET && DEFER) {          // status and sum follow from the work word (field_scatter_kernel)
            work[i] = o.work;
        } else {
            out_code[i] = (uint8_t)o.code;
            if (SET && out_sum)
                out_sum[i] = (uint16_t)o.sum;
        }
    }
}

template <int PROTO, bool SET, bool DEFER>
__device__ __forceinline__ void l4_finish(uint8_t *nh, uint64_t i, uint32_t sum, L4State &st, bool writer,
                                          uint8_t *out_code, uint16_t *out_sum, uint32_t *work)
{
    l4_finish_with<PROTO, SET, DEFER>(nh, i, sum, st, writer, out_code, out_sum, work,
                                      [&](uint32_t r) { set_field_store<PROTO>(nh, st, r, writer); });
}

// Fixed geometry: G lanes per packet.  Every lane of a group issues the
// packet's pass-0 chunk loads for [nh, nh+caplen) AND the header dwords
// (same addresses across the group: one request per wave instruction), so
// one memory round trip serves the parse and the sum.
#ifndef CLK_L4_WPE_SET
#define CLK_L4_WPE_SET 4     // UDP Set l4_kernels: 4 waves/SIMD, as the Check run loop (C3 Set 4.60 vs 4.65 ms at 5)
#endif
#ifndef CLK_SET_OCC_PAD
#define CLK_SET_OCC_PAD 28672   // two-phase compute pass (runs): LDS caps it at 5 waves/SIMD (C3 3.75 vs 3.83 ms at 6)
#endif
#ifndef CLK_SET_OCC_PAD64
#define CLK_SET_OCC_PAD64 28672 // ... for 64-lane groups (C5)
#endif
#ifndef CLK_L4_WPE_CHECK
#define CLK_L4_WPE_CHECK 4   // 4 waves/SIMD: the run loop spills at 5 (C3 Check 4.14 vs 3.81 ms)
#endif
// One packet by its G-lane group: parse, sum, and (fused Set) the field store.
template <int PROTO, bool SET, int G, int K, bool DEFER, bool HDRC>
__device__ __forceinline__ L4Out l4_group(const BatchArgs &b, int fixoff, uint64_t i, uint32_t lane, uint32_t gl)
{
    uint8_t *nh = b.base + pkt_off(b, i);
    const uint32_t caplen = pkt_len(b, i);
    const uint64_t a = (uint64_t)nh;
    const uint8_t *c0 = (const uint8_t *)(a & ~15ull);
    const uint32_t nch = (uint32_t)((((a + caplen + 15) & ~15ull) - (uint64_t)c0) / 16);
    u32x4 v[K];
    // nontemporal for Check and for the read-only compute pass of a
    // two-phase Set
    constexpr bool NT = UseNT<!SET || DEFER>::value;
    load_pass<G, K, NT>(c0, nch, 0, gl, v);  // issued before the header loads
    L4State st;
    if (SET && DEFER && HDRC && G >= 4)    // two-phase compute pass, grid-stride loop
        l4_parse_from_chunks<PROTO, SET, G, K>(nh, caplen, fixoff, (uint64_t)c0, lane, v, st);
    else
        l4_parse<PROTO, SET>(nh, caplen, fixoff, st);
    // a lane whose packet needs no sum masks everything (len 0)
    const uint32_t sum = group_range_sum<G, K, NT>(c0, nch, gl, v, a + st.hl, st.summing ? st.rlen : 0);
    if (SET && !DEFER && CLK_SET_REGBLK)
        return l4_result<PROTO, SET, DEFER>(nh, sum, st, gl == 0, [&](uint32_t r) {
            if (!set_block_store_regs<PROTO, G, K>(nh, st, r, gl, (uint64_t)c0, v))
                set_field_store<PROTO>(nh, st, r, gl == 0);
        });
    return l4_result<PROTO, SET, DEFER>(nh, sum, st, gl == 0,
                                        [&](uint32_t r) { set_field_store<PROTO>(nh, st, r, gl == 0); });
}

// RUNS: packets 0..n-1 in runs per workgroup (below); else the grid-stride
// loop over groups (the two-phase Set's compute pass for G < CLK_L4_RUNS_SET_G).
template <int PROTO, bool SET, int G, int K, bool DEFER, bool RUNS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SET && PROTO == UDP ? CLK_L4_WPE_SET : SET ? 1 : CLK_L4_WPE_CHECK)))
l4_kernel(BatchArgs b, int fixoff, uint8_t *out_code,
                                                 uint16_t *out_sum, uint32_t *work)
{
    const uint32_t lane = threadIdx.x & 63, gl = lane & (G - 1);
    if (RUNS) {
        // A workgroup owns runs of RB consecutive packets (at least 64), 256 / G
        // per pass, as the grid-stride loop visits them.  The groups' writer
        // lanes put the results in LDS, and after a workgroup barrier one
        // store instruction per output and wave writes the run's outputs:
        // every output block (64 B of codes, 256 B of work words, 128 B of
        // sums) is written whole by one workgroup, so no partial block
        // reaches the memory controller's read-modify-write and no block is
        // shared by the L2s of two XCDs (DESIGN.md §6,
        // tools/probes/stash_probe.hip).  The two-phase Set parses its
        // header from loads of its own here (measured faster in runs).
        constexpr uint32_t PPB = 256 / G, RB = PPB < 64 ? 64 : PPB;
#if CLK_SET_OCC_PAD
        // tuning: LDS padding caps the two-phase compute pass's occupancy
        __shared__ uint8_t occ_pad[SET && DEFER ? (G == 64 ? CLK_SET_OCC_PAD64 : CLK_SET_OCC_PAD) : 1];
        if (b.n == ~0ull)
            occ_pad[threadIdx.x] = 1;
#endif
        __shared__ uint8_t r_code[SET && DEFER ? 1 : RB];
        __shared__ uint32_t r_work[SET && DEFER ? RB : 1];
        __shared__ uint16_t r_sum[SET && !DEFER ? RB : 1];
        const uint64_t nruns = (b.n + RB - 1) / RB;
        for (uint64_t run = run_block<CLK_XCD_BLOCKS != 0>(); run < nruns; run += gridDim.x) {       // uniform per workgroup
            const uint64_t i0 = run * RB;
#pragma unroll 1
            for (uint32_t p = 0; p < RB / PPB; p++) {
                const uint32_t q = p * PPB + threadIdx.x / G;
                if (i0 + q < b.n) {
                    const L4Out o = l4_group<PROTO, SET, G, K, DEFER, false>(b, fixoff, i0 + q, lane, gl);
                    if (gl == 0) {
                        if (SET && DEFER) {
                            r_work[q] = o.work;
                        } else {
                            r_code[q] = (uint8_t)o.code;
                            if (SET && out_sum)
                                r_sum[q] = (uint16_t)o.sum;
                        }
                    }
                }
            }
            __syncthreads();
            const uint64_t i = i0 + threadIdx.x;
            if (threadIdx.x < RB && i < b.n) {
                if (SET && DEFER) {
                    work[i] = r_work[threadIdx.x];
                } else {
                    out_code[i] = r_code[threadIdx.x];
                    if (SET && out_sum)
                        out_sum[i] = r_sum[threadIdx.x];
                }
            }
            __syncthreads();
        }
        return;
    }
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / G;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; i < b.n; i += groups) {
        const L4Out o = l4_group<PROTO, SET, G, K, DEFER, CLK_HDR_FROM_CHUNKS != 0>(b, fixoff, i, lane, gl);
        if (gl == 0) {
            if (SET && DEFER) {
                work[i] = o.work;
            } else {
                out_code[i] = (uint8_t)o.code;
                if (SET && out_sum)
                    out_sum[i] = (uint16_t)o.sum;
            }
        }
    }
}

// Sum of a byte range read straight from global memory by one lane (the
// stream kernel's fallback for ranges its stash cannot correct).
__device__ __noinline__ uint32_t lane_range_sum(uint64_t s, int len)
{
    if (len <= 0)
        return 0;
    RangeAcc acc{0, 0};
    const bool odd = (s & 1) != 0;
    const uint64_t c = s & ~15ull;
    const uint32_t nch = (uint32_t)((((s + (uint64_t)len + 15) & ~15ull) - c) >> 4);
    for (uint32_t k = 0; k < nch; k++)
        chunk_accumulate(gload16(CLK_CHK(c + 16ull * k, 16, CHK_RANGE)), (int)(c + 16ull * k - s), len, odd, acc);
    return word_sum(acc, odd);
}

// Word sum (relative to a range start of parity `odd`) of the bytes of one
// 16-byte chunk at absolute address ca that lie OUTSIDE [s, s + len).
__device__ __forceinline__ uint32_t chunk_outside(const u32x4 V, uint64_t ca, uint64_t s, int len, uint32_t sel,
                                                  uint32_t acc)
{
    const int rel = (int)(int64_t)(ca - s);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t in = lowmask(len - rel - 4 * q) & ~lowmask(-rel - 4 * q);
        const uint32_t dm = V[q] & ~in;
        acc = dot_words(__builtin_amdgcn_perm(dm, dm, sel), acc);
    }
    return acc;
}

// Variable lengths, packet-stream form (default for IMIX).  A wave takes 64
// consecutive packets and streams, unmasked, the 16-byte chunks covering
// each packet's captured bytes [nh, nh + caplen) -- known from the batch
// descriptors alone, so the header is not fetched ahead of the stream:
//   Phase A: lane per packet: chunk span from off/len, wave scan into LDS.
//   Phase B: lane l owns KV consecutive chunks of the wave's concatenated
//            chunk list per pass (binary search for its first packet, step
//            at boundaries); whole-chunk word sums (v_dot2; byte-swapped
//            when the wave holds an odd-address packet) go to the packet's
//            LDS accumulator at packet changes.  The lane holding a
//            packet's chunk 0..HC-1 or its last chunk stashes it in LDS.
//   Phase C: lane per packet: parse the header from the stash (l4_parse_words),
//            subtract the stashed chunks' bytes outside the summed range
//            [nh+hl, nh+hl+rlen), finish.  A range whose unstashed middle
//            chunks are not all inside it (options past the stash, trailing
//            bytes) is re-summed from global memory by its lane.
// The sum mod 2^32 is order-free (cksum_device.hh), so whole-chunk sums
// minus the excluded bytes equal the reference's word sum exactly.
template <int PROTO, bool SET, bool DEFER, int KV>
__global__ void __launch_bounds__(256)
#if CLK_SWPE
__attribute__((amdgpu_waves_per_eu(!SET ? CLK_SWPE_CHECK : SET && !DEFER && CLK_SET_REGBLK && CLK_SWPE > 6 ? 6 : PROTO == TCP && CLK_SWPE > 7 ? 7 : CLK_SWPE)))
#endif
l4_stream_kernel(BatchArgs b, int fixoff, uint8_t *out_code,
                                                        uint16_t *out_sum, uint32_t *work)
{
    constexpr int HDR_DW = L4Hdr<PROTO>::DW;
    // stashed head chunks: every header dword when (nh&~3) - c0 + 4*HDR_DW <= 16*HC
    // (always for HC = 4 / 3; for 16 B-aligned packets with 3 / 2), else
    // the parse loads the missing dwords itself
    // A fused Set stashes 4 (the field's 64 B block, stored whole from the
    // stash); the two-phase compute pass stores nothing and needs no more.
    constexpr int HC0 = PROTO == TCP ? 3 : 2;
    constexpr int HC = SET && !DEFER && CLK_SET_REGBLK && HC0 < 4 ? 4 : HC0;
    constexpr bool COAL = SET && !DEFER && CLK_SET_REGBLK && CLK_STASH_COALESCE;
    __shared__ u32x4 head[4][64][HC];
    // dense runs: the pass's chunks, coalesced order in, lane-consecutive out;
    // the generic path keeps its packet records in the first 64 entries
    constexpr bool DENSE = CLK_DENSE && (!SET || CLK_DENSE_SET);
    __shared__ u32x4 stg[4][DENSE ? 64 * KV : 64];
    __shared__ uint32_t cst[4][68];   // chunk starts; cst[64] = total (dense: span)
    __shared__ uint32_t acc[4][64];
    __shared__ uint32_t pnf[4][DENSE ? 64 : 1];   // dense: nch | odd << 31
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32x4 *const pk = stg[wv];       // {c0 lo, c0 hi, chunk start, nch | odd << 31}
    const uint64_t nruns = (b.n + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * (blockDim.x / 64);
    uint64_t run = (uint64_t)run_block<CLK_XCD_BLOCKS || (SET && !DEFER && CLK_XCD_SET)>() * (blockDim.x / 64) + wv;
    if (run >= nruns)
        return;                      // wave-uniform; no workgroup barrier below
    // Phase A of one run: this lane's packet and the wave's chunk list.
    struct RunA {
        uint64_t a;                  // the packet's first byte (b.base for no packet)
        uint32_t caplen, nch;
        uint32_t start;              // first chunk in the wave's list (dense: in the span)
        uint32_t total;              // wave-uniform: chunks in the list (dense: the span)
        uint64_t sbase;              // dense: the span's first chunk address
        bool anyodd, dense;
        bool huge;                   // a packet longer than 16 MiB: per-lane sums from memory
    };
    // the raw descriptors, loaded unconditionally (index clamped) and not
    // yet used, so that a prefetch leaves them in flight
    auto load_desc = [&](uint64_t r, uint64_t &off, uint32_t &len) {
        const uint64_t i = r * 64 + lane;
        const uint64_t ii = i < b.n ? i : 0;
        off = pkt_off(b, ii);
        len = pkt_len(b, ii);
    };
    auto phase_a = [&](uint64_t off, uint32_t len, uint64_t r) {
        RunA R;
        const bool live = r * 64 + lane < b.n;
        const uint64_t a = live ? (uint64_t)b.base + off : (uint64_t)b.base;
        const uint32_t caplen = live ? len : 0u;
        const uint64_t c0 = a & ~15ull;
        const uint32_t nch = caplen ? (uint32_t)((((a + caplen + 15) & ~15ull) - c0) >> 4) : 0u;
        uint32_t incl = nch;                                   // wave-inclusive scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d, 64);
            if ((int)lane >= d)
                incl += t;
        }
        const uint32_t total = __shfl(incl, 63, 64);
        R.a = a;
        R.caplen = caplen;
        R.nch = nch;
        R.anyodd = __ballot(live && (a & 1)) != 0;
        R.dense = false;
        R.sbase = 0;
        R.start = incl - nch;
        R.total = total;
        // The chunk list packs a packet's chunk index into 26 bits and the
        // run's count into 32: both hold for packets up to 16 MiB (the host
        // sends only batches with max_len <= 16 MiB here, use_stream()).  A
        // run with a longer packet -- a descriptor past its batch's max_len
        // -- streams nothing: phase C sums each packet from memory, so no
        // index can wrap whatever the lengths are.
        R.huge = __ballot(caplen > STREAM_MAX_LEN) != 0;
        if (R.huge) {
            R.start = 0;
            R.total = 0;
        }
        // Dense run: the packets' chunk ranges are increasing and disjoint
        // and their span [c0 of packet 0, end of the last) holds few gap
        // chunks -- as a packed arena does.  A chunk's address is then
        // sbase + 16 c with no lookup, so the wave loads the span coalesced
        // (lane l: chunks k*64 + l of the pass, one 1 KiB line-run per
        // instruction) and nontemporal -- 6.9-7.1 TB/s where the
        // lane-consecutive shape reads 6.2-6.3 (default policy) or 4.6
        // (nontemporal: a line's pieces come from three instructions;
        // tools/probes/shape_probe.hip) -- and hands the chunks to their
        // lane-consecutive owners through LDS.  Gap chunks are loaded, not
        // summed (at most total/8 + 64 of them).
        if (DENSE) {
            const uint64_t cend = c0 + 16ull * nch;
            const uint32_t pe_lo = __shfl_up((uint32_t)cend, 1, 64), pe_hi = __shfl_up((uint32_t)(cend >> 32), 1, 64);
            const uint64_t pend = (uint64_t)pe_lo | ((uint64_t)pe_hi << 32);
            const bool bad = live && lane > 0 && c0 < pend;
            const uint64_t nlive = __popcll(__ballot(live));          // live lanes are a prefix
            const uint64_t sb = (uint64_t)__shfl((uint32_t)c0, 0, 64) | ((uint64_t)__shfl((uint32_t)(c0 >> 32), 0, 64) << 32);
            const uint32_t lastl = nlive ? (uint32_t)nlive - 1 : 0u;
            const uint64_t send = (uint64_t)__shfl((uint32_t)cend, (int)lastl, 64) |
                                  ((uint64_t)__shfl((uint32_t)(cend >> 32), (int)lastl, 64) << 32);
            const uint64_t sp = send >= sb ? (send - sb) >> 4 : ~0ull;
            if (!R.huge && __ballot(bad) == 0 && total > 0 && sp <= (uint64_t)total + (total >> 3) + 64) {
                R.dense = true;
                R.sbase = sb;
                R.total = (uint32_t)sp;
                R.start = live ? (uint32_t)((c0 - sb) >> 4) : (uint32_t)sp;
            }
        }
        return R;
    };
    uint64_t na;
    uint32_t ncap;
    load_desc(run, na, ncap);
    // issue: find the packets of this lane's KV chunks at cb and load them
    // per chunk the consumer needs its packet (jk) and inf = its index r in
    // the packet | last chunk << 30 | odd packet << 31 (2 VGPRs per chunk
    // rather than the packet's 4-word record: KV = 4 fits 8 waves)
    auto issue = [&](const RunA &R, uint32_t cb, u32x4 (&v)[KV], uint32_t (&jk)[KV], uint32_t (&inf)[KV]) {
        const uint32_t cl = cb + lane * KV, total = R.total;
        uint32_t j = 0;                                    // last packet whose chunk start <= cl
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (cst[wv][j + step] <= cl)
                j += step;
        uint32_t nxt = cst[wv][j + 1];
#pragma unroll
        for (int k = 0; k < KV; k++) {
            const uint32_t c = cl + k;
            if (c < total && c >= nxt) {
                do {
                    j++;
                    nxt = cst[wv][j + 1];
                } while (c >= nxt);
            }
            jk[k] = j;
        }
#pragma unroll
        for (int k = 0; k < KV; k++) {
            const uint32_t c = cl + k;
            const u32x4 P = pk[jk[k]];
            const uint32_t r = c - P[2];
            // r | (last chunk: 1 << 30 | end offset << 26) | odd start << 31
            inf[k] = r | (r == (P[3] & 0x07FFFFFFu) - 1 ? (1u << 30) | (((P[3] >> 27) & 15) << 26) : 0u) |
                     (P[3] & 0x80000000u);
            const uint64_t cf = (uint64_t)P[0] | ((uint64_t)P[1] << 32);
            CLK_CHK_IF(c < total && c < P[2], CHK_UNDERFLOW, cf);
            if (UseNT<CLK_STREAM_NT_CHECK && !SET>::value)
                v[k] = c < total ? __builtin_nontemporal_load(
                                       (const u32x4 *)CLK_CHK(cf + 16ull * (c - P[2]), 16, CHK_GENERIC))
                                 : u32x4{0, 0, 0, 0};
            else
                v[k] = c < total ? gload16(CLK_CHK(cf + 16ull * (c - P[2]), 16, CHK_GENERIC)) : u32x4{0, 0, 0, 0};
        }
    };
    // consume: whole-chunk sums into the packets' accumulators, stash
    auto consume = [&](const RunA &R, uint32_t cb, const u32x4 (&v)[KV], const uint32_t (&jk)[KV],
                       const uint32_t (&inf)[KV]) {
        const uint32_t cl = cb + lane * KV, total = R.total;
        uint32_t cj = jk[0], part = 0;
#pragma unroll
        for (int k = 0; k < KV; k++) {
            const uint32_t c = cl + k;
            if (c >= total)
                break;
            if (jk[k] != cj) {
                atomicAdd(&acc[wv][cj], part);
                part = 0;
                cj = jk[k];
            }
            u32x4 V = v[k];
            const uint32_t r = inf[k] & 0x03FFFFFFu;       // chunk index within the packet
            if (inf[k] & (1u << 30))                      // the last chunk: bytes past the packet out
                V = keep_below(V, (inf[k] >> 26) & 15);
            if (r < (uint32_t)HC)
                head[wv][jk[k]][r] = V;
            if (R.anyodd) {
                const uint32_t sel = (inf[k] >> 31) ? 0x02030001u : 0x03020100u;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    part = dot_words(__builtin_amdgcn_perm(V[q], V[q], sel), part);
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    part = dot_words(V[q], part);
            }
        }
        if (cl < total)
            atomicAdd(&acc[wv][cj], part);
    };
    // dense: lane l eats chunks cb + l*KV .. + KV-1 of the span from LDS
    auto dense_eat = [&](const RunA &R, uint32_t cb) {
        const uint32_t cl = cb + lane * KV, span = R.total;
        if (cl >= span)
            return;
        uint32_t j = 0;                                    // last packet whose first chunk <= cl
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (cst[wv][j + step] <= cl)
                j += step;
        uint32_t sj = cst[wv][j], nxt = cst[wv][j + 1], pn = pnf[wv][j];
        uint32_t cj = j, part = 0;
#pragma unroll
        for (int k = 0; k < KV; k++) {
            const uint32_t c = cl + k;
            if (c >= span)
                break;
            if (c >= nxt) {
                do {
                    j++;
                    nxt = cst[wv][j + 1];
                } while (c >= nxt);
                sj = cst[wv][j];
                pn = pnf[wv][j];
            }
            const uint32_t r = c - sj, pnch = pn & 0x07FFFFFFu;
            if (r >= pnch)                                 // a gap chunk
                continue;
            if (j != cj) {
                atomicAdd(&acc[wv][cj], part);
                part = 0;
                cj = j;
            }
            u32x4 V = stg[wv][lane * KV + k];
            if (r == pnch - 1)                             // the last chunk: bytes past the packet out
                V = keep_below(V, (pn >> 27) & 15);
            if (r < (uint32_t)HC)
                head[wv][j][r] = V;
            if (R.anyodd) {
                const uint32_t sel = (pn >> 31) ? 0x02030001u : 0x03020100u;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    part = dot_words(__builtin_amdgcn_perm(V[q], V[q], sel), part);
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    part = dot_words(V[q], part);
            }
        }
        if (part)
            atomicAdd(&acc[wv][cj], part);
    };
    // dense loads: coalesced, nontemporal, addresses clamped into the span
    // rather than the loads predicated (a predicated load forces its wait
    // before the next use of the register)
    constexpr uint32_t PASS = 64 * KV;
    u32x4 dv[DENSE ? KV : 1];
    auto dense_load_to = [&](const RunA &R, uint32_t cb, auto &d) {
#pragma unroll
        for (int k = 0; k < KV; k++) {
            const uint32_t c = min(cb + (uint32_t)k * 64 + lane, R.total - 1);
            d[k] = __builtin_nontemporal_load(
                (const __attribute__((address_space(1))) u32x4 *)CLK_CHK(R.sbase + 16ull * c, 16, CHK_DENSE));
        }
    };
    auto dense_load = [&](const RunA &R, uint32_t cb) { dense_load_to(R, cb, dv); };
    // one pass parked in LDS and eaten while the next ones load
    auto dense_step = [&](const RunA &R, uint32_t cb, auto &d, uint32_t ahead) {
#pragma unroll
        for (int k = 0; k < KV; k++)
            stg[wv][k * 64 + lane] = d[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (cb + ahead < R.total)
            dense_load_to(R, cb + ahead, d);
        dense_eat(R, cb);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (;;) {
        // (the descriptors are used from here on, not earlier: the compiler
        // would hoist their use, and its wait, above the previous run)
        asm volatile("" : "+v"(na), "+v"(ncap));
        const RunA cur = phase_a(na, ncap, run);
        {   // publish the run's phase A
            const uint64_t c0 = cur.a & ~15ull;
            // nch | end offset in the last chunk << 27 | odd start << 31
            const uint32_t pnv = cur.nch | ((uint32_t)((cur.a + cur.caplen) & 15) << 27) | ((uint32_t)(cur.a & 1) << 31);
            cst[wv][lane] = cur.start;
            if (lane == 63)
                cst[wv][64] = cur.total;
            if (DENSE && cur.dense)
                pnf[wv][lane] = pnv;
            else
                pk[lane] = u32x4{(uint32_t)c0, (uint32_t)(c0 >> 32), cur.start, pnv};
            acc[wv][lane] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // the next run's descriptors load while this run streams (a wave
        // takes several runs only under a grid cap; issuing the next run's
        // first dense pass ahead of phase C was tried, tools/gpu_runs/r03/gpu_r03f.sh and
        // r03g, and is not kept)
        const uint64_t nrun = run + wstride;
        if (DENSE && cur.dense) {
            dense_load(cur, 0);
            load_desc(nrun, na, ncap);
            for (uint32_t cb = 0; cb < cur.total; cb += PASS)           // wave-uniform
                dense_step(cur, cb, dv, PASS);
        } else {
            load_desc(nrun, na, ncap);
            for (uint32_t cb = 0; cb < cur.total; cb += 64 * KV) {     // wave-uniform
                u32x4 v[KV];
                uint32_t jk[KV], inf[KV];
                issue(cur, cb, v, jk, inf);
                consume(cur, cb, v, jk, inf);
            }
            vm_retire();             // chunks past the list were loaded and not used
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // Phase C
        const uint64_t i = run * 64 + lane;
        const uint64_t a = cur.a, c0 = a & ~15ull;
        const uint32_t caplen = cur.caplen, nch = cur.nch;
        uint8_t *nh = (uint8_t *)a;
        uint64_t blk_q0 = 0;         // COAL: the patched block's address | its first stash chunk
        if (i < b.n) {
            const uint32_t *hw = (const uint32_t *)&head[wv][lane][0];
            const uint32_t q0 = (uint32_t)((a & ~3ull) - c0) >> 2;   // first header dword in the stash
            const uint64_t end = a + caplen;
            uint32_t d[HDR_DW];
#pragma unroll
            for (int k = 0; k < HDR_DW; k++) {
                if ((a & ~3ull) + 4 * k >= end) {
                    d[k] = 0u;
                } else if (!cur.huge && q0 + k < 4u * HC) {
                    d[k] = hw[q0 + k];
                } else {                 // past the stash (unaligned or option-bearing header)
                    d[k] = gload4(CLK_CHK((a & ~3ull) + 4 * k, 4, CHK_HDR));
                    vm_retire();
                }
            }
            L4State st;
            l4_parse_words<PROTO, SET>(nh, caplen, fixoff, d, st);
            uint32_t sum = 0;
            const int rlen = st.summing ? st.rlen : 0;
            if (rlen > 0) {
                const uint64_t s = a + st.hl, e = s + (uint64_t)rlen;
                const uint32_t sel = (a & 1) ? 0x02030001u : 0x03020100u;
                const bool stashed = !cur.huge && (nch <= (uint32_t)HC + 1 ||
                                                   (s <= c0 + 16 * HC && e >= c0 + 16ull * (nch - 1)));
                if (stashed) {
                    uint32_t out = 0;
                    const uint32_t nh_ = nch < (uint32_t)HC ? nch : (uint32_t)HC;
                    for (uint32_t k = 0; k < nh_; k++)
                        out = chunk_outside(head[wv][lane][k], c0 + 16ull * k, s, rlen, sel, out);
                    const uint64_t cl = c0 + 16ull * (nch - 1);
                    if (nch > (uint32_t)HC && (e < a + caplen || s > cl)) {
                        // the last chunk was summed up to the packet's end:
                        // its bytes outside [s, e) -- in [e, end) (link-layer
                        // padding, bytes past the transport length), or before
                        // s (a short packet with options) -- are re-read and
                        // taken out
                        u32x4 T = gload16(CLK_CHK(cl, 16, CHK_LAST));
                        vm_retire();
                        T = keep_below(T, (uint32_t)((a + caplen) & 15));
                        out = chunk_outside(T, cl, s, rlen, sel, out);
                    }
                    sum = acc[wv][lane] - out;
                } else {
                    sum = lane_range_sum(s, rlen);
                }
            }
            if (COAL)
                l4_finish_with<PROTO, SET, DEFER>(nh, i, sum, st, true, out_code, out_sum, work, [&](uint32_t r) {
                    blk_q0 = cur.huge ? 0 : set_block_patch_stash<PROTO, HC>(nh, st, r, c0, head[wv][lane]);
                    if (!blk_q0)
                        set_field_store<PROTO>(nh, st, r, true);
                });
            else if (SET && !DEFER && CLK_SET_REGBLK)
                l4_finish_with<PROTO, SET, DEFER>(nh, i, sum, st, true, out_code, out_sum, work, [&](uint32_t r) {
                    if (cur.huge || !set_block_store_stash<PROTO, HC>(nh, st, r, c0, head[wv][lane]))
                        set_field_store<PROTO>(nh, st, r, true);
                });
            else
                l4_finish<PROTO, SET, DEFER>(nh, i, sum, st, true, out_code, out_sum, work);
        }
        if (COAL) {
            // the patched blocks leave by 4 store instructions, each writing
            // 16 whole blocks: lanes 4p'..4p'+3 store quarters 0..3 of packet
            // 16 s + p' (a full 64 B write per 4 lanes)
            pk[lane] = u32x4{(uint32_t)blk_q0, (uint32_t)(blk_q0 >> 32), 0, 0};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (uint32_t s4 = 0; s4 < 4; s4++) {
                const uint32_t p = 16 * s4 + (lane >> 2), q = lane & 3;
                const u32x4 P = pk[p];
                const uint64_t bq = (uint64_t)P[0] | ((uint64_t)P[1] << 32);
                if (bq) {
                    const uint64_t ca = (bq & ~63ull) + 16ull * q;
                    const u32x4 w = head[wv][p][(bq & 63) + q];
                    if (CLK_STASH_NT)
                        __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4 *)ca);
                    else
                        *(__attribute__((address_space(1))) u32x4 *)ca = w;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        run = nrun;
        if (run >= nruns)
            break;
    }
}

// ---------------------------------------------------------------------------
// DecIPTTL (decipttl.cc:45-77) with ACTIVE true: one lane per packet reads
// ip_ttl..ip_sum and the first byte of ip_dst, and rewrites ip_ttl and
// ip_sum by the reference's RFC 1624 shortcut ~(~sum + 0xFEFF) (72-73).
// Codes: OK (decremented), TTL_EXPIRED (ttl <= 1: output 1), TTL_UNCHANGED.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) dec_ttl_kernel(BatchArgs b, int multicast, uint8_t *out_code,
                                                      uint16_t *out_sum)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += nthreads) {
        uint8_t *ip = b.base + pkt_off(b, i);
        uint32_t code = TTL_UNCHANGED, stored = 0;
        if (pkt_len(b, i) >= 20) {               // guard: no length check in the reference
            const uint32_t w = ld_u32_unaligned(ip + 8);        // ttl, proto, sum (LE)
            if (multicast || (ld_u8(ip + 16) & 0xF0) != 0xE0) { // 51-52, is_multicast
                const uint32_t ttl = w & 0xFF;
                if (ttl <= 1) {
                    code = TTL_EXPIRED;                          // 54-57
                } else {
                    const uint32_t s = (~(uint32_t)bswap16(w >> 16) & 0xFFFF) + 0xFEFF;
                    stored = ~(uint32_t)bswap16((s + (s >> 16)) & 0xFFFF) & 0xFFFF;
                    if (((uint64_t)ip & 3) == 0) {
                        field_st_u32(ip + 8, (ttl - 1) | (w & 0xFF00) | (stored << 16));
                    } else {
                        ip[8] = (uint8_t)(ttl - 1);
                        field_st_u16(ip + 10, stored);
                    }
                    code = OK;
                }
            }
        }
        out_code[i] = (uint8_t)code;
        if (out_sum)
            out_sum[i] = (uint16_t)stored;
    }
}

// ---------------------------------------------------------------------------
// RFC 1624 incremental update (include/clicknet/ip.h:177-185) and the zero
// fixup (ip.h:196-201, lib/in_cksum.c:113-121), one lane per packet.  Words
// are read and stored as the reference's uint16_t accesses do (host order).
// Codes: 0 updated, 1 a field lies past len_i (nothing written).
// ---------------------------------------------------------------------------
struct UpdateArgs {
    uint32_t sum_off, hw_off, zero_lo;
    int32_t zero_fix, replace;
};

__device__ __forceinline__ uint32_t ld_u16_any(const uint8_t *p)
{
    return ld_u8(p) | (ld_u8(p + 1) << 8);
}

// click_update_zero_in_cksum_hard: all bytes of [x, x + len) zero?
__device__ __noinline__ bool all_zero(const uint8_t *x, int len)
{
    for (; len > 0 && ((uint64_t)x & 3); --len, ++x)
        if (ld_u8(x))
            return false;
    for (; len >= 4; len -= 4, x += 4)
        if (gload4((uint64_t)x))
            return false;
    for (; len > 0; --len, ++x)
        if (ld_u8(x))
            return false;
    return true;
}

__global__ void __launch_bounds__(256) update_kernel(BatchArgs b, UpdateArgs u, const uint16_t *new_hw,
                                                     uint8_t *out_code, uint16_t *out_sum)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += nthreads) {
        uint8_t *p = b.base + pkt_off(b, i);
        const uint32_t len = pkt_len(b, i);
        uint32_t code = 0, csum = 0;
        if ((uint64_t)u.sum_off + 2 > len || (u.replace && (uint64_t)u.hw_off + 2 > len)) {
            code = 1;
        } else {
            csum = ld_u16_any(p + u.sum_off);
            if (u.replace) {
                const uint32_t old_hw = ld_u16_any(p + u.hw_off), nw = new_hw[i];
                st_u16(p + u.hw_off, nw);
                uint32_t sum = (~csum & 0xFFFFu) + (~old_hw & 0xFFFFu) + nw;    // ip.h:182
                sum = (sum & 0xFFFFu) + (sum >> 16);                            // 183
                csum = ~(sum + (sum >> 16)) & 0xFFFFu;                          // 184
                st_u16(p + u.sum_off, csum);
            }
            // ip.h:196-201: a zero checksum of all-zero data is ~0
            if (u.zero_fix && csum == 0 && all_zero(p + u.zero_lo, (int)len - (int)u.zero_lo)) {
                csum = 0xFFFFu;
                st_u16(p + u.sum_off, csum);
                code = 2;
            }
        }
        if (out_code)
            out_code[i] = (uint8_t)code;
        if (out_sum)
            out_sum[i] = (uint16_t)csum;
    }
}

// ---------------------------------------------------------------------------
// IP output path, one lane per packet: IPGWOptions (ipgwoptions.cc:53-172),
// FixIPSrc (fixipsrc.cc:52-72) and IPOutputCombo after its annotation-only
// steps (ipoutputcombo.cc:59-199).  Option-free headers (ip_hl = 5, the
// common case) take the straight path: one dword and one byte read, TTL
// and ip_sum rewritten as in DecIPTTL; options are walked byte by byte.
// ---------------------------------------------------------------------------
enum IpOutMode { OUT_GWOPT = 0, OUT_FIXSRC = 1, OUT_COMBO = 2 };

struct IpOutArgs {
    uint32_t my_ip, ts, n_my_addrs, mtu;
    const uint32_t *my_addrs;
    const uint8_t *flags;      // per packet: bit 0 FIX_IP_SRC_ANNO (nullptr: FixIPSrc all set, combo none)
};

__device__ __forceinline__ void st_u8(uint8_t *p, uint32_t v)
{
    *(__attribute__((address_space(1))) uint8_t *)p = (uint8_t)v;
}
__device__ __forceinline__ void st_u32_bytes(uint8_t *p, uint32_t v)
{
    for (int k = 0; k < 4; k++)
        st_u8(p + k, v >> (8 * k));
}

// The option walk (ipgwoptions.cc:59-153 / ipoutputcombo.cc:65-166) over a
// header with 20 < hlen <= caplen.  An option byte at or past caplen reads
// as 0 (oracle/cksum_oracle.c: the same domain guard).  Returns 1 on a
// parameter problem (offset in *problem).
__device__ __noinline__ uint32_t ip_gw_options(uint8_t *ip, int hlen, uint32_t caplen, uint32_t my_ip,
                                               const uint32_t *my_addrs, uint32_t nmy, uint32_t ts,
                                               uint32_t *problem, bool *touched, bool *changed)
{
    auto optb = [&](int i) -> int { return (uint32_t)i < caplen ? (int)ld_u8(ip + i) : 0; };
    for (int oi = 20; oi < hlen;) {
        const int type = (int)ld_u8(ip + oi);
        if (type == 1) {                          // IPOPT_NOP
            oi++;
            continue;
        } else if (type == 0)                     // IPOPT_EOL
            break;
        const int xlen = optb(oi + 1);
        if (xlen < 2 || oi + xlen > hlen) {
            *problem = oi + 1;
            return 1;
        } else if (type != 7 && type != 68) {     // not IPOPT_RR / IPOPT_TS
            oi += xlen;
            continue;
        }
        *touched = true;
        const int p = optb(oi + 2) - 1;
        if (type == 7) {                          // Record Route
            if (p >= 3 && p + 4 <= xlen) {
                st_u32_bytes(ip + oi + p, my_ip);
                st_u8(ip + oi + 2, (uint32_t)(p + 1 + 4));
                *changed = true;
            } else if (p != xlen) {
                *problem = oi + 2;
                return 1;
            }
        } else {                                  // Timestamp
            const int oflw = optb(oi + 3) >> 4, flg = optb(oi + 3) & 0xF;
            bool overflowed = false;
            if (p < 4) {
                *problem = oi + 2;
                return 1;
            } else if (flg == 0) {
                if (p + 4 <= xlen) {
                    st_u32_bytes(ip + oi + p, ts);
                    st_u8(ip + oi + 2, (uint32_t)(p + 1 + 4));
                    *changed = true;
                } else
                    overflowed = true;
            } else if (flg == 1) {
                if (p + 8 <= xlen) {
                    st_u32_bytes(ip + oi + p, my_ip);
                    st_u32_bytes(ip + oi + p + 4, ts);
                    st_u8(ip + oi + 2, (uint32_t)(p + 1 + 8));
                    *changed = true;
                } else
                    overflowed = true;
            } else if (flg == 3 && p + 8 <= xlen) {
                const uint32_t addr = ld_u32_unaligned(ip + oi + p);
                bool mine = !my_addrs && addr == my_ip;   // IPOutputCombo: IPADDR only (144)
                for (uint32_t k = 0; my_addrs && k < nmy; k++)
                    mine |= my_addrs[k] == addr;
                if (mine) {
                    st_u32_bytes(ip + oi + p + 4, ts);
                    st_u8(ip + oi + 2, (uint32_t)(p + 1 + 8));
                    *changed = true;
                }
            } else {
                *problem = oi + 3;
                return 1;
            }
            if (overflowed) {
                if (oflw < 15) {
                    st_u8(ip + oi + 3, (uint32_t)(((oflw + 1) << 4) | flg));
                    *changed = true;
                } else {
                    *problem = oi + 3;
                    return 1;
                }
            }
        }
        oi += xlen;
    }
    return 0;
}

// ip_sum = 0; ip_sum = click_in_cksum(ip, hlen): stores and returns it.
__device__ __forceinline__ uint32_t ip_resum(uint8_t *ip, uint32_t hlen)
{
    uint32_t sum = 0;
    for (uint32_t o = 0; o < hlen; o += 4) {
        const uint32_t w = ld_u32_unaligned(ip + o);
        sum += (w & 0xFFFF) + (w >> 16);
    }
    if (hlen >= 12)                                // the stored ip_sum is in range: zero it
        sum -= ld_u32_unaligned(ip + 8) >> 16;
    const uint32_t v = in_cksum_fold(sum);
    st_u16(ip + 10, v);
    return v;
}

template <int MODE>
__global__ void __launch_bounds__(256) ip_out_kernel(BatchArgs b, IpOutArgs c, uint8_t *out_code,
                                                     uint8_t *out_problem, uint16_t *out_sum)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += nthreads) {
        uint8_t *ip = b.base + pkt_off(b, i);
        const uint32_t caplen = pkt_len(b, i);
        uint32_t code = 0, problem = 0, cur = 0;
        if (caplen >= 20) {
            const uint32_t w8 = ld_u32_unaligned(ip + 8);       // ttl, proto, ip_sum
            cur = w8 >> 16;
            const uint32_t hlen = (ld_u8(ip) & 0xF) << 2;
            const uint32_t flag = c.flags ? c.flags[i] : (MODE == OUT_FIXSRC ? 1u : 0u);
            bool touched = false, changed = false;
            if (MODE != OUT_FIXSRC && hlen > 20 && hlen <= caplen &&    // hlen > caplen: domain guard
                ip_gw_options(ip, (int)hlen, caplen, c.my_ip, MODE == OUT_COMBO ? nullptr : c.my_addrs,
                              c.n_my_addrs, c.ts, &problem, &touched, &changed)) {
                code = MODE == OUT_GWOPT ? 1u : 2u;                     // output 1 / output 2
            } else {
                bool resum = MODE == OUT_GWOPT && touched;              // ipgwoptions.cc:155-159
                if (MODE != OUT_GWOPT && (flag & 1) && (MODE == OUT_COMBO || hlen <= caplen)) {
                    st_u32_bytes(ip + 12, c.my_ip);                     // fixipsrc.cc:60-64 / combo 169-173
                    changed = true;
                }
                if (MODE != OUT_GWOPT)
                    resum = changed && hlen <= caplen;                  // combo 176-179
                if (resum)
                    cur = ip_resum(ip, hlen);
                if (MODE == OUT_COMBO) {                        // DecIPTTL, ipoutputcombo.cc:182-191
                    const uint32_t ttl = w8 & 0xFF;             // no earlier step writes byte 8
                    if (ttl <= 1) {
                        code = 3;
                    } else {
                        const uint32_t s = (~(uint32_t)bswap16(cur) & 0xFFFF) + 0xFEFF;
                        cur = ~(uint32_t)bswap16((s + (s >> 16)) & 0xFFFF) & 0xFFFF;
                        st_u8(ip + 8, ttl - 1);
                        st_u16(ip + 10, cur);
                        if (caplen > c.mtu)                     // 194-197
                            code = 4;
                    }
                }
            }
        }
        out_code[i] = (uint8_t)code;
        if (out_problem)
            out_problem[i] = (uint8_t)problem;
        if (out_sum)
            out_sum[i] = (uint16_t)cur;
    }
}

// ---------------------------------------------------------------------------
// Deferred Set stores.  Writing the 2-byte checksum field into the packet
// while the same kernel streams packet bytes in costs far more than its
// bytes (DESIGN.md "Why Set is slower"); the two-phase Set computes in a
// read-only pass (field value + transport offset into work[]) and this pass
// scatters the fields: base + off_i + hl + FIELD <- value for work bit 31
// (hl in work bits 16..23).  Nontemporal stores, so the partial-block write
// reaches HBM inside this kernel instead of lingering dirty in the caches
// until the next kernel's reads evict it.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void scatter_st_u16(uint8_t *p, uint32_t v)
{
    if ((uint64_t)p & 1)
        st_u16(p, v);
    else
        __builtin_nontemporal_store((uint16_t)v, (__attribute__((address_space(1))) uint16_t *)p);
}

template <int FIELD>
__global__ void __launch_bounds__(256) field_scatter_kernel(BatchArgs b, const uint32_t *work, uint8_t *out_code,
                                                            uint16_t *out_sum)
{
    // the compute pass wrote only work[i] (bit 31: the field value, else the
    // status code); this pass writes the field and, one lane per packet, the
    // status codes and sums -- 64 consecutive packets per wave, so whole
    // output blocks
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += nthreads) {
        const uint32_t w = work[i];
        if (w & 0x80000000u)
            scatter_st_u16(b.base + pkt_off(b, i) + ((w >> 16) & 0xFF) + FIELD, w & 0xFFFF);
        out_code[i] = (w & 0x80000000u) ? 0 : (uint8_t)w;
        if (out_sum)
            out_sum[i] = (w & 0x80000000u) ? (uint16_t)w : 0;
    }
}

// ---------------------------------------------------------------------------
// Utilities: verdict histogram, synthetic traffic, corruption, read stream.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) count_codes_kernel(const uint8_t *codes, uint64_t n,
                                                          unsigned long long *counts, uint32_t nc)
{
    __shared__ unsigned int hist[256];
    hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthreads)
        atomicAdd(&hist[codes[i]], 1u);
    __syncthreads();
    if (threadIdx.x < nc && hist[threadIdx.x])
        atomicAdd(&counts[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
}

__device__ __forceinline__ uint64_t gen_word(uint64_t seed, uint64_t idx, uint64_t w)
{
    return splitmix64(seed ^ ((idx << 13) | (w & 0x1FFF)));
}

// Same bytes as oracle_gen_packet (oracle/cksum_oracle.c): 64 lanes per
// packet, lane l writes 8-byte words l, l+64, ... masked to [0, len).
__global__ void __launch_bounds__(256) gen_kernel(BatchArgs b, int proto, uint64_t seed, uint64_t first_idx)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / 64;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; i < b.n; i += groups) {
        uint8_t *p = b.base + pkt_off(b, i);
        const uint32_t len = pkt_len(b, i);
        const uint64_t idx = first_idx + i;
        const uint64_t ha = gen_word(seed, idx, 0x1FFF), hb = gen_word(seed, idx, 0x1FFE);
        const uint32_t src = 0x0A000000u | (uint32_t)(ha & 0xFFFFFF);
        const uint32_t dst = 0xC0A80000u | (uint32_t)((ha >> 24) & 0xFFFF);
        const uint32_t hlen = proto == 17 ? 28 : (proto == 6 ? 40 : 20);
        for (uint32_t w = lane; 8 * w < len; w += 64) {
            uint64_t x = gen_word(seed, idx, w);
            if (8 * w < hlen) {
                uint8_t hb8[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t o = 8 * w + k;
                    uint32_t v = (uint32_t)(x >> (8 * k)) & 0xFF;
                    if (o < hlen) {
                        v = 0;
                        switch (o) {
                        case 0: v = 0x45; break;
                        case 2: v = (len >> 8) & 0xFF; break;
                        case 3: v = len & 0xFF; break;
                        case 4: v = (uint32_t)(idx >> 8) & 0xFF; break;
                        case 5: v = (uint32_t)idx & 0xFF; break;
                        case 8: v = 64; break;
                        case 9: v = (uint32_t)proto; break;
                        case 12: v = src >> 24; break;
                        case 13: v = (src >> 16) & 0xFF; break;
                        case 14: v = (src >> 8) & 0xFF; break;
                        case 15: v = src & 0xFF; break;
                        case 16: v = dst >> 24; break;
                        case 17: v = (dst >> 16) & 0xFF; break;
                        case 18: v = (dst >> 8) & 0xFF; break;
                        case 19: v = dst & 0xFF; break;
                        default: {
                            const uint32_t sport = (uint32_t)(ha >> 40) & 0xFFFF;
                            if (proto == 17) {
                                const uint32_t dport = ((uint32_t)(ha >> 56) | 0x400) & 0xFFFF;
                                const uint32_t ulen = len >= 20 ? len - 20 : 0;
                                if (o == 20) v = sport >> 8;
                                else if (o == 21) v = sport & 0xFF;
                                else if (o == 22) v = dport >> 8;
                                else if (o == 23) v = dport & 0xFF;
                                else if (o == 24) v = (ulen >> 8) & 0xFF;
                                else if (o == 25) v = ulen & 0xFF;
                            } else if (proto == 6) {
                                const uint32_t win = (uint32_t)(ha >> 48) & 0xFFFF;
                                if (o == 20) v = sport >> 8;
                                else if (o == 21) v = sport & 0xFF;
                                else if (o == 22) v = 0;
                                else if (o == 23) v = 80;
                                else if (o >= 24 && o < 32) v = (uint32_t)(hb >> (8 * (o - 24))) & 0xFF;
                                else if (o == 32) v = 0x50;
                                else if (o == 33) v = 0x10;
                                else if (o == 34) v = win >> 8;
                                else if (o == 35) v = win & 0xFF;
                            }
                        }
                        }
                    }
                    hb8[k] = (uint8_t)v;
                }
                x = 0;
#pragma unroll
                for (int k = 0; k < 8; k++)
                    x |= (uint64_t)hb8[k] << (8 * k);
            }
            uint8_t *dstp = p + 8 * w;
            const uint32_t nb = len - 8 * w < 8 ? len - 8 * w : 8;
            if (nb == 8 && (((uint64_t)dstp & 7) == 0)) {
                *(uint64_t *)dstp = x;
            } else {
                for (uint32_t k = 0; k < nb; k++)
                    dstp[k] = (uint8_t)(x >> (8 * k));
            }
        }
    }
}

// Packet i (global index first_idx + i) is picked when the low rate_log2
// bits of h = splitmix64(seed ^ (first_idx + i) * C) are zero; one bit of
// byte lo + (h >> 20) % (hi' - lo) is flipped, hi' = min(hi, len) (hi = 0:
// len; lo = ~0u: 40 / 20 / 0 by length, the payload past the headers).
// Flipping twice restores the batch.  bench.py recomputes the picks.
__global__ void __launch_bounds__(256) corrupt_kernel(BatchArgs b, uint64_t seed, uint64_t first_idx,
                                                      uint32_t rate_log2, uint32_t lo_arg, uint32_t hi_arg)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t mask = rate_log2 >= 64 ? ~0ull : ((1ull << rate_log2) - 1);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += nthreads) {
        const uint64_t h = splitmix64(seed ^ ((first_idx + i) * 0xD1B54A32D192ED03ull));
        if ((h & mask) != 0)
            continue;
        const uint32_t len = pkt_len(b, i);
        const uint32_t lo = lo_arg != ~0u ? lo_arg : (len > 40 ? 40 : (len > 20 ? 20 : 0));
        const uint32_t hi = hi_arg && hi_arg < len ? hi_arg : len;
        if (hi <= lo)
            continue;
        const uint32_t pos = lo + (uint32_t)((h >> 20) % (uint64_t)(hi - lo));
        uint8_t *p = b.base + pkt_off(b, i) + pos;
        *p ^= (uint8_t)(1u << ((h >> 8) & 7));
    }
}

// The measured read ceiling (bench only): grid-stride, U nontemporal 16 B
// loads per lane in flight, launched on a capped grid -- the best of the
// twelve shapes of tools/probes/read_probe.hip (gs8_nt at 8K workgroups,
// 7.01-7.07 TB/s; the uncapped gs4 grid read 6.5).
template <int U>
__global__ void __launch_bounds__(256) read_stream_kernel(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * nthreads < n16; i += U * nthreads) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            a[u] = __builtin_nontemporal_load(p + i + u * nthreads);
#pragma unroll
        for (int u = 0; u < U; u++)
            acc += a[u][0] ^ a[u][1] ^ a[u][2] ^ a[u][3];
    }
    for (; i < n16; i += nthreads) {
        const u32x4 a0 = p[i];
        acc += a0[0] ^ a0[1] ^ a0[2] ^ a0[3];
    }
    for (int m = 32; m >= 1; m >>= 1)
        acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0 && acc)
        atomicAdd(out, (unsigned long long)acc);
}

// ... each wave reading U KiB contiguous per step (lane l: 16 B at l*16 +
// u*1 KiB), the steps dealt round-robin to the waves; the tail grid-strided
template <int U>
__global__ void __launch_bounds__(256) read_wave_kernel(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t nsteps = n16 / (64 * U);
    uint32_t acc = 0;
    for (uint64_t s = w0; s < nsteps; s += nwaves) {
        const u32x4 *q = p + s * 64 * U + lane;
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            a[u] = __builtin_nontemporal_load(q + 64 * u);
#pragma unroll
        for (int u = 0; u < U; u++)
            acc += a[u][0] ^ a[u][1] ^ a[u][2] ^ a[u][3];
    }
    for (uint64_t i = nsteps * 64 * U + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 a0 = p[i];
        acc += a0[0] ^ a0[1] ^ a0[2] ^ a0[3];
    }
    for (int m = 32; m >= 1; m >>= 1)
        acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0 && acc)
        atomicAdd(out, (unsigned long long)acc);
}

// ... or as the fixed-geometry Check kernels read a C3 batch: 16-lane groups,
// each reading one row of K x 256 B (K nontemporal 16 B loads per lane in
// flight, lane l at l*16 + u*256), a workgroup's 16 groups on 16 consecutive
// rows per step; the rows past the last whole step and the tail grid-strided
template <int K>
__global__ void __launch_bounds__(256) read_rows_kernel(const u32x4 *p, uint64_t n16, unsigned long long *out)
{
    const uint32_t gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint64_t row16 = 16 * K;                       // 16 B chunks per row
    const uint64_t nsteps = n16 / (16 * row16);
    uint32_t acc = 0;
    for (uint64_t s = blockIdx.x; s < nsteps; s += gridDim.x) {
        const u32x4 *q = p + (s * 16 + grp) * row16 + gl;
        u32x4 a[K];
#pragma unroll
        for (int u = 0; u < K; u++)
            a[u] = __builtin_nontemporal_load(q + 16 * u);
#pragma unroll
        for (int u = 0; u < K; u++)
            acc += a[u][0] ^ a[u][1] ^ a[u][2] ^ a[u][3];
    }
    for (uint64_t i = nsteps * 16 * row16 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 a0 = p[i];
        acc += a0[0] ^ a0[1] ^ a0[2] ^ a0[3];
    }
    for (int m = 32; m >= 1; m >>= 1)
        acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0 && acc)
        atomicAdd(out, (unsigned long long)acc);
}

// The measured copy ceiling (bench only): grid-stride, U nontemporal 16 B
// loads per lane in flight, then their U stores (NTS: nontemporal), on a
// capped grid -- equal read and write streams, the fragmenter's traffic.
template <int U, bool NTS>
__global__ void __launch_bounds__(256) copy_stream_kernel(const u32x4 *src, u32x4 *dst, uint64_t n16)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * nthreads < n16; i += U * nthreads) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            a[u] = __builtin_nontemporal_load(src + i + u * nthreads);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NTS)
                __builtin_nontemporal_store(a[u], dst + i + u * nthreads);
            else
                dst[i + u * nthreads] = a[u];
        }
    }
    for (; i < n16; i += nthreads)
        dst[i] = src[i];
}

// ... each wave copying U KiB contiguous per step (lane l: 16 B at l*16 +
// u*1 KiB), the steps dealt round-robin to the waves; the tail grid-strided
template <int U>
__global__ void __launch_bounds__(256) copy_wave_kernel(const u32x4 *src, u32x4 *dst, uint64_t n16)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t nsteps = n16 / (64 * U);
    for (uint64_t s = w0; s < nsteps; s += nwaves) {
        const uint64_t q = s * 64 * U + lane;
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            a[u] = __builtin_nontemporal_load(src + q + 64 * u);
#pragma unroll
        for (int u = 0; u < U; u++)
            dst[q + 64 * u] = a[u];
    }
    for (uint64_t i = nsteps * 64 * U + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// ... and the IMIX Set's traffic without its arithmetic: the stream read as
// read_stream_kernel<U> reads it, and one whole 64 B block in every `every`
// written back in place (nontemporal; C4 SetUDPChecksum writes the block
// holding each packet's field, one per 354 B on average)
template <int U>
__global__ void __launch_bounds__(256) read_write_blocks_kernel(u32x4 *p, uint64_t n16, uint32_t every,
                                                                unsigned long long *out)
{
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * nthreads < n16; i += U * nthreads) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            a[u] = __builtin_nontemporal_load(p + i + u * nthreads);
#pragma unroll
        for (int u = 0; u < U; u++) {
            acc += a[u][0] ^ a[u][1] ^ a[u][2] ^ a[u][3];
            if (((i + u * nthreads) >> 2) % every == 0)
                __builtin_nontemporal_store(a[u], p + i + u * nthreads);
        }
    }
    for (; i < n16; i += nthreads) {
        const u32x4 a0 = p[i];
        acc += a0[0] ^ a0[1] ^ a0[2] ^ a0[3];
    }
    for (int m = 32; m >= 1; m >>= 1)
        acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0 && acc)
        atomicAdd(out, (unsigned long long)acc);
}

} // namespace clk
