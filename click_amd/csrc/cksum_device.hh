// cksum_device.hh -- gfx950 device arithmetic for Click's Internet checksum.
//
// The reference sums native (little-endian) 16-bit words into a uint32_t that
// silently wraps (lib/in_cksum.c:25,33-36), so the result is the sum taken
// mod 2^32 and ANY reduction order reproduces it as long as partial sums are
// never end-around folded.  For a byte range [s, e) with A = sum of the bytes
// at even absolute addresses and B = sum of the bytes at odd absolute
// addresses (both mod 2^32), the reference's word sum is
//     S = A + 256*B   when s is even   (word k = b[s+2k] | b[s+2k+1] << 8)
//     S = B + 256*A   when s is odd,
// and an odd trailing byte lands in the low half as in_cksum.c:39-42 adds it.
// Lanes therefore load 16-byte-aligned chunks and accumulate S directly
// with v_dot2_u32_u16 (even s), or A and B with v_dot4_u32_u8 (odd s); only
// the bytes of the two boundary chunks are masked.  Any alignment is exact.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

// Loads and stores through the global address space: global_load/store
// (vmcnt only) instead of flat instructions, which also count in lgkmcnt,
// for addresses the compiler cannot prove global (e.g. read back from LDS).
// Measured equal speed on C3/C4; kept for the cleaner ISA.
__device__ __forceinline__ u32x4 gload16(uint64_t addr)
{
    return *(const __attribute__((address_space(1))) u32x4 *)addr;
}
__device__ __forceinline__ u32x4 gload16_a4(uint64_t addr)   // 4-byte aligned
{
    return *(const __attribute__((address_space(1))) u32x4_a4 *)addr;
}
__device__ __forceinline__ uint32_t gload4(uint64_t addr)
{
    return *(const __attribute__((address_space(1))) uint32_t *)addr;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v)
{
    return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}

// lib/in_cksum.c:45-49: two-step carry fold of the u32 sum, complement.
__device__ __forceinline__ uint32_t in_cksum_fold(uint32_t sum)
{
    sum = (sum & 0xffffu) + (sum >> 16);
    sum += sum >> 16;
    return (~sum) & 0xffffu;
}

// lib/in_cksum.c:53-80, portable branch 74-78 (htons truncates to 16 bits).
__device__ __forceinline__ uint32_t pseudohdr_raw(uint32_t csum, uint32_t src, uint32_t dst,
                                                  uint32_t proto, uint32_t packet_len)
{
    csum = ~csum & 0xFFFFu;
    csum += (src & 0xffffu) + (src >> 16);
    csum += (dst & 0xffffu) + (dst >> 16);
    csum += bswap16(packet_len & 0xFFFFu) + bswap16(proto & 0xFFFFu);
    csum = (csum & 0xffffu) + (csum >> 16);
    return ~(csum + (csum >> 16)) & 0xFFFFu;
}

// Bytes of a dword at absolute address a that lie in [s, e): mask of the
// bytes j with lo <= j < hi, lo = s - a, hi = e - a (clamped to [0, 4]).
__device__ __forceinline__ uint32_t lowmask(int k)
{
    k = k < 0 ? 0 : (k > 4 ? 4 : k);
    return k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * k)) - 1u);
}

// Chunk V with its bytes at positions eo..15 zeroed (eo 0: whole chunk).
__device__ __forceinline__ u32x4 keep_below(u32x4 V, uint32_t eo)
{
    if (eo) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            V[q] &= lowmask((int)eo - 4 * q);
    }
    return V;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// v_dot2_u32_u16: acc + lo16(d) + hi16(d), wrapping mod 2^32 (no clamp) --
// one instruction per dword of an even-start range (the word sum A + 256 B).
__device__ __forceinline__ uint32_t dot_words(uint32_t d, uint32_t acc)
{
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), u16x2{1, 1}, acc, false);
}
// v_dot4_u32_u8 with byte weights: acc + sum of the selected bytes.
__device__ __forceinline__ uint32_t dot_even_bytes(uint32_t d, uint32_t acc)
{
    return __builtin_amdgcn_udot4(d, 0x00010001u, acc, false);
}
__device__ __forceinline__ uint32_t dot_odd_bytes(uint32_t d, uint32_t acc)
{
    return __builtin_amdgcn_udot4(d, 0x01000100u, acc, false);
}

// Per-lane accumulators of a range sum.  Even start: s0 = the word sum.
// Odd start: s0 = A (even-address bytes), s1 = B (odd-address bytes).
struct RangeAcc {
    uint32_t s0, s1;
};

// Accumulate one 16-byte chunk whose first byte is at relative position rel
// (chunk address - range start, may be negative) against a range of length
// len.  Interior chunks take 4 (even) or 8 (odd start) dot instructions;
// only the two boundary chunks of a range pay for byte masks.
__device__ __forceinline__ void chunk_accumulate(const u32x4 v, int rel, int len, bool odd, RangeAcc &acc)
{
    if (rel >= 0 && rel + 16 <= len) {
        if (!odd) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                acc.s0 = dot_words(v[j], acc.s0);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                acc.s0 = dot_even_bytes(v[j], acc.s0);
                acc.s1 = dot_odd_bytes(v[j], acc.s1);
            }
        }
    } else if (rel < len && rel + 16 > 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int lo = -rel - 4 * j;
            const int hi = len - rel - 4 * j;
            const uint32_t d = v[j] & lowmask(hi) & ~lowmask(lo);
            if (!odd) {
                acc.s0 = dot_words(d, acc.s0);
            } else {
                acc.s0 = dot_even_bytes(d, acc.s0);
                acc.s1 = dot_odd_bytes(d, acc.s1);
            }
        }
    }
}

// Word sum of a range from its accumulators and start parity.
__device__ __forceinline__ uint32_t word_sum(const RangeAcc &acc, bool odd)
{
    return odd ? (acc.s1 + (acc.s0 << 8)) : acc.s0;
}

__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p)
{
    return *(const __attribute__((address_space(1))) uint8_t *)p;
}

// Retire this wave's outstanding vector-memory loads here, inside the branch
// that issued a rare load: the join after the branch then needs no wait.  A
// kernel that keeps loads in flight across such code (the packet stream's
// next-run pass) would otherwise wait for all of them at the join, since
// vmcnt retires in order.  (gfx9 encoding: vmcnt 0, expcnt and lgkmcnt free.)
__device__ __forceinline__ void vm_retire()
{
    __builtin_amdgcn_s_waitcnt(0x0F70);
}

__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t *p)
{
    const uint64_t a = (uint64_t)p;
    const uint64_t q = a & ~3ull;
    const uint32_t sh = (uint32_t)(a & 3);
    if (sh == 0)
        return gload4(q);
    return __builtin_amdgcn_alignbyte(gload4(q + 4), gload4(q), sh);
}

__device__ __forceinline__ void st_u16(uint8_t *p, uint32_t v)
{
    typedef __attribute__((address_space(1))) uint8_t g8;
    typedef __attribute__((address_space(1))) uint16_t g16;
    if (((uint64_t)p & 1) == 0) {
        *(g16 *)p = (uint16_t)v;
    } else {
        ((g8 *)p)[0] = (uint8_t)v;
        ((g8 *)p)[1] = (uint8_t)(v >> 8);
    }
}

// lib/in_cksum.c:83-111: option walk for the SSRR/LSRR final destination,
// then pseudohdr_raw.  Only reached when ip_hl != 5 (ip.h:152-160).
__device__ __noinline__ uint32_t pseudohdr_hard(uint32_t csum, const uint8_t *iph, uint32_t packet_len)
{
    const uint32_t hl = (ld_u8(iph) & 0xF) << 2;
    const uint32_t src = ld_u32_unaligned(iph + 12);
    const uint32_t proto = ld_u8(iph + 9);
    uint32_t dst = ld_u32_unaligned(iph + 16);
    uint32_t o = 20;
    while (o < hl) {
        const uint32_t t = ld_u8(iph + o);
        if (t == 1) {               // IPOPT_NOP
            o++;
            continue;
        } else if (t == 0)          // IPOPT_EOL
            break;
        if (o + 1 >= hl)
            break;
        const uint32_t l = ld_u8(iph + o + 1);
        if (l < 2 || o + l > hl)
            break;
        if ((t == 137 || t == 131) && l >= 7) {   // IPOPT_SSRR / IPOPT_LSRR
            dst = ld_u32_unaligned(iph + o + l - 4);
            break;
        }
        o += l;
    }
    return pseudohdr_raw(csum, src, dst, proto, packet_len);
}

// The destination the pseudo-header uses: the final hop of the first
// SSRR/LSRR option (in_cksum.c:86-108), else `dst`.  Options only.
__device__ __noinline__ uint32_t route_dst(const uint8_t *iph, uint32_t hl, uint32_t dst)
{
    uint32_t o = 20;
    while (o < hl) {
        const uint32_t t = ld_u8(iph + o);
        if (t == 1) {               // IPOPT_NOP
            o++;
            continue;
        } else if (t == 0)          // IPOPT_EOL
            break;
        if (o + 1 >= hl)
            break;
        const uint32_t l = ld_u8(iph + o + 1);
        if (l < 2 || o + l > hl)
            break;
        if ((t == 137 || t == 131) && l >= 7)      // IPOPT_SSRR / IPOPT_LSRR
            return ld_u32_unaligned(iph + o + l - 4);
        o += l;
    }
    return dst;
}

// pseudohdr_raw split in two (in_cksum.c:74-78): the header terms, summed
// at parse time (< 7 * 0xFFFF, no carry out of 32 bits) ...
__device__ __forceinline__ uint32_t pseudohdr_partial(uint32_t src, uint32_t dst, uint32_t proto,
                                                      uint32_t packet_len)
{
    return (src & 0xffffu) + (src >> 16) + (dst & 0xffffu) + (dst >> 16) + bswap16(packet_len & 0xFFFFu) +
           bswap16(proto & 0xFFFFu);
}
// ... and the fold with the payload checksum: equal to pseudohdr_raw(csum,
// src, dst, proto, packet_len) for ph = pseudohdr_partial(src, dst, proto,
// packet_len), as the u32 sum is order-free.
__device__ __forceinline__ uint32_t pseudohdr_ph(uint32_t csum, uint32_t ph)
{
    uint32_t c = (~csum & 0xFFFFu) + ph;
    c = (c & 0xffffu) + (c >> 16);
    return ~(c + (c >> 16)) & 0xFFFFu;
}

// include/clicknet/ip.h:152-160
__device__ __forceinline__ uint32_t pseudohdr(uint32_t csum, const uint8_t *iph, uint32_t b0,
                                              uint32_t src, uint32_t dst, uint32_t proto,
                                              uint32_t transport_len)
{
    if ((b0 & 0xF) == 5)
        return pseudohdr_raw(csum, src, dst, proto, transport_len);
    return pseudohdr_hard(csum, iph, transport_len);
}

// splitmix64 finalizer (synthetic traffic; identical to oracle_splitmix64).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

} // namespace clk
