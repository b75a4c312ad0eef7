/*
 * click_amd_cksum.h -- C ABI of the MI355X (gfx950) Internet-checksum path.
 *
 * Drop-in boundary for Click's software checksum path.  The reference has no
 * FFI for this path: the checksum functions are leaves called from element
 * simple_action()s (kohler/click 2.1, lib/in_cksum.c, include/clicknet/ip.h,
 * elements/ip, elements/tcpudp).  Each batched entry point below replaces one
 * such per-packet call, applied to a whole struct-of-arrays packet batch that
 * is resident in device memory (HBM); the element glue that would call it
 * from Click's tree is shown in INTEGRATION.md.
 *
 * Conventions
 *   - plain C: pointers, sizes, POD structs; no C++ types, no exceptions;
 *   - every function returns 0 (CLK_SUCCESS) or a negative CLK_E* code, and
 *     clk_last_error(ctx) describes the last failure on that context;
 *   - batched calls are ASYNCHRONOUS on the context's HIP stream; results are
 *     valid after clk_ctx_sync() (or an event recorded on clk_ctx_stream());
 *   - all buffers are owned by the caller; device pointers must come from
 *     hipMalloc (or any allocator with page-granular device allocations);
 *   - one context per host thread (Click RouterThread); a context is not
 *     re-entrant, distinct contexts are thread-safe.
 *
 * Byte order: 16-bit words are summed in little-endian order, like the
 * reference on x86-64, so results are bit-identical to lib/in_cksum.c and
 * are stored into the header fields exactly as the reference stores them.
 */
#ifndef CLICK_AMD_CKSUM_H
#define CLICK_AMD_CKSUM_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define CLK_ABI_VERSION 6

/* ---- return codes -------------------------------------------------------- */
#define CLK_SUCCESS 0
#define CLK_EINVAL (-1)   /* bad argument (null pointer, n too large, ...)    */
#define CLK_EHIP (-2)     /* HIP runtime error; see clk_last_error()           */
#define CLK_ENODEV (-3)   /* no such device / device is not gfx950             */

/* ---- per-packet result codes ---------------------------------------------
 * Check elements: 0 = packet passes (output 0); otherwise 1 + the element's
 * Reason enum value (the packet is dropped: output 1 if connected, else
 * killed; drops/drop_details handlers count it).                          */
enum clk_ip_verdict {                 /* CheckIPHeader::Reason, checkipheader.hh:150-158 */
    CLK_OK = 0,
    CLK_IP_MINISCULE_PACKET = 1,
    CLK_IP_BAD_VERSION = 2,
    CLK_IP_BAD_HLEN = 3,
    CLK_IP_BAD_IP_LEN = 4,
    CLK_IP_BAD_CHECKSUM = 5,
    CLK_IP_BAD_SADDR = 6
};
enum clk_l4_verdict {                 /* Check{UDP,TCP,ICMP}Header::Reason */
    CLK_L4_NOT_PROTO = 1,             /* NOT_UDP / NOT_TCP / NOT_ICMP */
    CLK_L4_BAD_LENGTH = 2,
    CLK_L4_BAD_CHECKSUM = 3
};
enum clk_set_status {                 /* Set*Checksum outcome */
    CLK_SET_OK = 0,                   /* field written; output 0                    */
    CLK_SET_OUTPUT1 = 1,              /* SetUDPChecksum: fragment or short -> output 1
                                         (setudpchecksum.cc:48-61); nothing written */
    CLK_SET_KILL = 2                  /* SetIPChecksum / SetTCPChecksum bad lengths:
                                         packet killed; nothing written            */
};
enum clk_ttl_status {                 /* DecIPTTL outcome (decipttl.cc:45-77) */
    CLK_TTL_OK = 0,                   /* ip_ttl decremented, ip_sum updated; output 0 */
    CLK_TTL_EXPIRED = 1,              /* ip_ttl <= 1: drops++, output 1 (or killed)   */
    CLK_TTL_UNCHANGED = 2             /* MULTICAST false and a multicast ip_dst, or
                                         caplen < 20: output 0, nothing written     */
};

/* ---- context ------------------------------------------------------------- */
typedef struct clk_ctx clk_ctx;

/* Number of gfx950 devices visible (HIP ordinals 0..n-1 are scanned; a
 * negative CLK_E* code on a runtime error).  An adapter maps its threads
 * to devices with it ("Devices").                          */
int clk_device_count(void);

/* Create a context on HIP device `device` with its own non-blocking stream. */
int clk_ctx_create(int device, clk_ctx **out);
int clk_ctx_destroy(clk_ctx *ctx);
/* Launch on hipStream_t `hip_stream` from now on (e.g. the stream of the
 * caller's framework; NULL is HIP's null stream, as in the HIP API).
 * clk_ctx_own_stream() returns the context's own stream, for switching back. */
int clk_ctx_set_stream(clk_ctx *ctx, void *hip_stream);
void *clk_ctx_stream(clk_ctx *ctx);
void *clk_ctx_own_stream(clk_ctx *ctx);
/* Wait for the context's stream.  Also reports a kernel's internal fault
 * flag (the IPFragmenter look-back's bounded wait timing out: CLK_EHIP). */
int clk_ctx_sync(clk_ctx *ctx);
int clk_ctx_device(clk_ctx *ctx);
/* Pre-size the context's device scratch for batches of up to max_packets
 * (4 bytes per packet: the two-phase UDP/TCP Set's work array); without it
 * the first larger batch allocates synchronously.  After a reserve, batched
 * calls of that size allocate nothing (safe inside hipGraph capture). */
int clk_ctx_reserve(clk_ctx *ctx, uint64_t max_packets);
/* Speed-only tuning of one context (tools/tune.py; defaults are the measured
 * best).  No setting changes any result: every kernel choice
 * they select is bit-exact against the reference.  Nothing is read from the
 * environment.  CLK_EINVAL for an unknown knob or an out-of-range value.   */
enum clk_tune_knob {
    CLK_TUNE_MAX_BLOCKS = 1,          /* grid cap of every launch (default 262144)       */
    CLK_TUNE_SCATTER_BLOCKS = 2,      /* grid cap of the two-phase Set's scatter (16384) */
    CLK_TUNE_SET_MODE = 3,            /* -1 auto, 0 fused Set, 1 two-phase Set           */
    CLK_TUNE_STREAM_MIN = 4,          /* len[] batches of >= this many packets run by the
                                         packet-stream kernel (65536)                     */
    CLK_TUNE_GROUP = 5,               /* lanes per packet of the fixed-geometry kernels:
                                         0 (by max_len), 1, 2, 4, ..., 64                 */
    CLK_TUNE_SET_CHUNKS = 6,          /* two-phase Set in this many packet ranges, each
                                         range's scatter on a side stream overlapping the
                                         next range's compute pass (1: one of each)       */
    CLK_TUNE_READ_SHAPE = 7,          /* clk_read_stream's load shape: 0 grid-stride, 8
                                         16 B loads per lane in flight, 8K workgroups;
                                         1 the same with 4 loads; 2 with 16 loads, 2K
                                         workgroups; 3 each wave 8 KiB contiguous per
                                         step, 4K workgroups; 4 16-lane groups each
                                         reading a 1536 B row (6 loads per lane), 16
                                         rows per workgroup step, one step per
                                         workgroup; 5 the same on 8K workgroups
                                         (bench: the best is the measured read
                                         ceiling)                                    */
    CLK_TUNE_FRAG_FLAT_MIN = 8,       /* clk_ip_fragment: batches of >= this many packets
                                         write the fragments of plain-header packets in
                                         a flat second pass (8192; 0: always)            */
    CLK_TUNE_FRAG_CHUNKS = 9          /* ... in this many tile ranges, each range's flat
                                         pass on a side stream overlapping the next
                                         range's plan (1)                                 */
};
int clk_ctx_tune(clk_ctx *ctx, int knob, int64_t value);
/* Last error text for `ctx` (or for the calling thread when ctx == NULL). */
const char *clk_last_error(clk_ctx *ctx);
int clk_abi_version(void);

/* ---- batch descriptor (struct of arrays, device-resident) ----------------
 * Packet i's bytes are [base + off_i, base + off_i + len_i) where
 *   off_i = off ? off[i] : i * stride        (byte offset of the header the
 *                                             element looks at)
 *   len_i = len ? len[i] : fixed_len          (bytes available from there to
 *                                             the packet's end_data())
 * For the IP/UDP/TCP elements the header is the packet's network (L3)
 * header; the transport header is taken at L3 + ip_hl*4, as CheckIPHeader /
 * MarkIPHeader set it.  Offsets may have any alignment (Click requires 2).
 * Set elements write their checksum field in place into `base`.
 * Readable memory: the kernels read whole 16-byte-aligned chunks, so the
 * chunk-aligned bytes around [off_i, off_i + len_i) must be readable (never
 * past its 4 KiB page).  The packet-stream kernel (below) also loads, without
 * using them, the bytes BETWEEN packets i and i+1 of one 64-packet run when
 * their offsets increase and the run's packets fill at least 8/9 of the
 * span less 1 KiB (a packed arena); such gaps must be readable too.  Every
 * packet in one device arena (the glue's staging, a registered ZEROCOPY
 * region, a generated batch) satisfies this. */
typedef struct clk_batch {
    uint8_t *base;
    const uint64_t *off;
    uint64_t stride;
    const uint32_t *len;
    uint32_t fixed_len;
    uint32_t max_len;   /* optional upper bound on len_i (0 = unknown).  With
                           len != NULL and max_len <= 16 MiB, large batches
                           run by the packet-stream kernel (whole-chunk sums,
                           lengths free per packet); others in one
                           lanes-per-packet geometry picked from max_len     */
    uint64_t n;
} clk_batch;

/* ---- checksum arithmetic ---------------------------------------------------
 * click_in_cksum(base+off_i, len_i) for every i        (lib/in_cksum.c:20-51)
 * out_sum[i] is the returned uint16_t.                                      */
int clk_in_cksum(clk_ctx *ctx, const clk_batch *ranges, uint16_t *out_sum);

/* ---- elements ------------------------------------------------------------- */

/* CheckIPHeader::simple_action (elements/ip/checkipheader.cc:161-226).
 * The batch points at each packet's data(); `offset` is the OFFSET keyword.
 * checksum = CHECKSUM keyword (0 gives CheckIPHeader2, checkipheader2.cc:27-31).
 * badsrc/gooddst: device arrays of raw (network-order) s_addr words for the
 * BADSRC/GOODDST/INTERFACES keywords (may be NULL with count 0).
 * out_verdict[i]: enum clk_ip_verdict.                                      */
typedef struct clk_ip_check_cfg {
    uint32_t offset;
    int32_t checksum;
    const uint32_t *badsrc;
    uint32_t nbadsrc;
    uint32_t ngooddst;
    const uint32_t *gooddst;
} clk_ip_check_cfg;
int clk_check_ip_header(clk_ctx *ctx, const clk_batch *batch,
                        const clk_ip_check_cfg *cfg, uint8_t *out_verdict);

/* SetIPChecksum::simple_action (elements/ip/setipchecksum.cc:74-95).
 * Writes ip_sum in place; out_status[i]: enum clk_set_status (OK or KILL);
 * out_sum (nullable): the 16-bit value stored (0 when not OK).              */
int clk_set_ip_checksum(clk_ctx *ctx, const clk_batch *batch,
                        uint8_t *out_status, uint16_t *out_sum);

/* CheckUDPHeader::simple_action (elements/tcpudp/checkudpheader.cc:84-107).
 * out_verdict[i]: 0 or enum clk_l4_verdict.                                 */
int clk_check_udp_header(clk_ctx *ctx, const clk_batch *batch, uint8_t *out_verdict);

/* SetUDPChecksum::simple_action (elements/tcpudp/setudpchecksum.cc:37-69).
 * out_status[i]: OK or OUTPUT1.                                              */
int clk_set_udp_checksum(clk_ctx *ctx, const clk_batch *batch,
                         uint8_t *out_status, uint16_t *out_sum);

/* CheckTCPHeader::simple_action (elements/tcpudp/checktcpheader.cc:85-107). */
int clk_check_tcp_header(clk_ctx *ctx, const clk_batch *batch, uint8_t *out_verdict);

/* SetTCPChecksum::simple_action (elements/tcpudp/settcpchecksum.cc:44-75);
 * fixoff = FIXOFF keyword (settcpchecksum.cc:39-41, 57-63).
 * out_status[i]: OK or KILL.                                                 */
int clk_set_tcp_checksum(clk_ctx *ctx, const clk_batch *batch, int fixoff,
                         uint8_t *out_status, uint16_t *out_sum);

/* CheckICMPHeader::simple_action (elements/icmp/checkicmpheader.cc:83-141).
 * The ICMP header is at L3 + ip_hl*4 (the transport header CheckIPHeader
 * sets); icmp_len = len_i - ip_hl*4.  out_verdict[i]: 0 or enum
 * clk_l4_verdict (NOT_ICMP, BAD_LENGTH incl. the per-type length rules,
 * BAD_CHECKSUM).                                                            */
int clk_check_icmp_header(clk_ctx *ctx, const clk_batch *batch, uint8_t *out_verdict);

/* DecIPTTL::simple_action (elements/ip/decipttl.cc:45-77) with ACTIVE true
 * (ACTIVE false passes packets without reading them: do not call).
 * multicast = MULTICAST keyword.  Decrements ip_ttl and updates ip_sum in
 * place by RFC 1624 (72-73); out_status[i]: enum clk_ttl_status; out_sum
 * (nullable): the ip_sum stored (0 when not OK).                          */
int clk_dec_ip_ttl(clk_ctx *ctx, const clk_batch *batch, int multicast,
                   uint8_t *out_status, uint16_t *out_sum);

/* ---- incremental update ------------------------------------------------------
 * click_update_in_cksum (include/clicknet/ip.h:177-185) applied in place to
 * every packet: the 16-bit word at off_i + cfg->hw_off is replaced by
 * new_hw[i] (device u16, stored as the reference stores a uint16_t) and the
 * checksum at off_i + cfg->sum_off is updated by RFC 1624 from the old and
 * new words.  With cfg->zero_fix, click_update_zero_in_cksum follows
 * (ip.h:196-201, lib/in_cksum.c:113-121): a resulting 0 over all-zero
 * data [off_i + zero_lo, off_i + len_i) becomes 0xFFFF.
 * out_status[i] (nullable): 0 updated, 1 a field past len_i (nothing
 * written), 2 updated and zero-fixed.  out_sum (nullable): the checksum
 * stored (as read back in host order).                                    */
typedef struct clk_cksum_update_cfg {
    uint32_t sum_off, hw_off;
    int32_t zero_fix;
    uint32_t zero_lo;
} clk_cksum_update_cfg;
int clk_update_in_cksum(clk_ctx *ctx, const clk_batch *batch, const clk_cksum_update_cfg *cfg,
                        const uint16_t *new_hw, uint8_t *out_status, uint16_t *out_sum);
/* click_update_zero_in_cksum alone on every packet (the ICMP responders'
 * call after their own updates, e.g. icmppingresponder.cc:89): the stored
 * checksum at off_i + sum_off becomes 0xFFFF when it is 0 and every byte of
 * [off_i + zero_lo, off_i + len_i) is 0.  Status / sums as above.          */
int clk_update_zero_in_cksum(clk_ctx *ctx, const clk_batch *batch, uint32_t sum_off, uint32_t zero_lo,
                             uint8_t *out_status, uint16_t *out_sum);

/* ---- IP output path ---------------------------------------------------------
 * The batch points at each packet's IP header (= data() for these elements
 * in an IP router graph); len_i = bytes from it to end_data().
 * cfg->my_ip: raw s_addr written by Record Route / Timestamp flg 1 and by
 *   FixIPSrc (IPGWOptions: its preferred address; IPOutputCombo / FixIPSrc:
 *   IPADDR).
 * cfg->ts: the 4 bytes a Timestamp option stores for "now" (the reference
 *   stores htonl(ms since midnight) from Timestamp::now(); the host takes it
 *   once per batch).
 * cfg->my_addrs / n_my_addrs: device array of raw s_addr, IPGWOptions'
 *   interface addresses for Timestamp flg 3 (IPOutputCombo matches my_ip).
 * cfg->mtu: IPOutputCombo's MTU.
 * out_problem (nullable): ICMP_PARAMPROB_ANNO offsets of the parameter
 *   problems (0 otherwise).  out_sum (nullable): ip_sum after the element.
 * Domain guards (as the oracle): len_i < 20 passes untouched; options are
 * not walked when ip_hl*4 > len_i; an option byte read at or past len_i
 * reads as 0. */
typedef struct clk_ip_out_cfg {
    uint32_t my_ip;
    uint32_t ts;
    const uint32_t *my_addrs;
    uint32_t n_my_addrs;
    uint32_t mtu;
} clk_ip_out_cfg;

enum clk_gwopt_status {               /* IPGWOptions outcome (ipgwoptions.cc:53-172) */
    CLK_GWOPT_OK = 0,                 /* output 0; ip_sum recomputed if an RR/TS option was met */
    CLK_GWOPT_ERROR = 1               /* parameter problem: drops++, output 1            */
};
/* IPGWOptions::simple_action (elements/ip/ipgwoptions.cc:164-172, options 53-160). */
int clk_ip_gw_options(clk_ctx *ctx, const clk_batch *batch, const clk_ip_out_cfg *cfg,
                      uint8_t *out_status, uint8_t *out_problem, uint16_t *out_sum);

/* FixIPSrc::simple_action (elements/ip/fixipsrc.cc:52-72).  anno[i] bit 0 =
 * FIX_IP_SRC_ANNO (NULL: set on every packet); the host clears the
 * annotation.  Every packet leaves on output 0.                            */
int clk_fix_ip_src(clk_ctx *ctx, const clk_batch *batch, const clk_ip_out_cfg *cfg,
                   const uint8_t *anno, uint16_t *out_sum);

/* IPOutputCombo::push (elements/ip/ipoutputcombo.cc:44-205) after its two
 * annotation-only steps, DropBroadcasts and PaintTee (the host kills
 * broadcasts and clones painted packets to output 1 before the batch):
 * IPGWOptions, FixIPSrc (flags[i] bit 0 = FIX_IP_SRC_ANNO; NULL: none), the
 * header re-checksum, DecIPTTL, the MTU test on len_i.  out_port[i]: 0,
 * 2 (parameter problem), 3 (TTL expired) or 4 (longer than MTU).          */
int clk_ip_output_combo(clk_ctx *ctx, const clk_batch *batch, const clk_ip_out_cfg *cfg,
                        const uint8_t *flags, uint8_t *out_port, uint8_t *out_problem, uint16_t *out_sum);

/* ---- IPFragmenter ------------------------------------------------------------
 * IPFragmenter::push / fragment (elements/ip/ipfragmenter.cc:88-171) on a
 * batch of packets at their IP headers (len_i = network_length()).
 * cfg->mtu / honor_df: the MTU and HONOR_DF keywords.  cfg->new_id
 * (nullable device u16 per packet): the ip_id written when HONOR_DF false
 * clears a DF bit (the reference draws click_random(), 112-115; NULL keeps
 * ip_id).
 * out_port[i]: 0 = not longer than the MTU, untouched, output 0;
 *              1 = DF with HONOR_DF, or the MTU leaves < 8 data bytes:
 *                  untouched, output 1 (drops++);
 *              2 = fragmented: packet i is rewritten IN PLACE as the first
 *                  fragment (ip_len, IP_MF, DF/ip_id, ip_sum) and keeps its
 *                  first out_first_len[i] bytes; its other fragments are
 *                  appended to `out`.
 *              3 = CLK_FRAG_NOROOM: its fragments do not all fit out->arena /
 *                  out->max_frags: nothing of it is written, the packet
 *                  keeps its bytes (size the buffers from `totals`, retry);
 *              0xFF = CLK_FRAG_FAULT: internal fault (the single-pass tile
 *                  look-back timed out, also reported by clk_ctx_sync):
 *                  the packet keeps its bytes, nothing of it is written.
 * out_first_len[i]: packet i's length after the element.
 * out_frag_first[i] (nullable): index of packet i's first appended fragment.
 * out->arena == NULL makes a sizing call: out_port, out_first_len and totals
 * are produced and nothing is written (packets untouched).
 * Appended fragments are packed in packet order at 16 B-aligned offsets of
 * out->arena; fragment k is out->frag_len[k] bytes at out->frag_off[k],
 * cut from packet out->frag_src[k].  totals (device u64[2]) receives the
 * fragments and arena bytes the batch needs; a packet whose fragments would
 * pass out->max_frags or out->arena_bytes is left whole (CLK_FRAG_NOROOM).
 * Domain guards (as the oracle): len_i < 20 with len_i > MTU -> port 1;
 * fragment bytes past len_i (ip_len > network_length) are written as 0.
 * Batches of at least CLK_TUNE_FRAG_FLAT_MIN packets (8192) that write
 * fragments run two kernels (plan/scan, then the flat payload pass) and
 * grow the context's device scratch by 16 B per out->max_frags. */
#define CLK_FRAG_NOROOM 3
#define CLK_FRAG_FAULT 0xFF
typedef struct clk_frag_cfg {
    uint32_t mtu;
    int32_t honor_df;
    const uint16_t *new_id;
} clk_frag_cfg;
typedef struct clk_frag_out {
    uint8_t *arena;
    uint64_t arena_bytes;
    uint64_t *frag_off;
    uint32_t *frag_len;
    uint32_t *frag_src;
    uint64_t max_frags;
} clk_frag_out;
int clk_ip_fragment(clk_ctx *ctx, const clk_batch *batch, const clk_frag_cfg *cfg, uint8_t *out_port,
                    uint32_t *out_first_len, uint64_t *out_frag_first, const clk_frag_out *out,
                    uint64_t *totals);

/* ---- zero-copy host packet memory --------------------------------------------
 * Register a host memory region (a DPDK mempool's hugepage area, a pcap
 * ring, any buffer the packets live in) so that kernels read and write the
 * packets in place over PCIe, with no staging copy: a batch may then use
 * base = *dev_base (the region's device address) and off_i = the packet's
 * offset from the region's host start.  Set elements then write their
 * fields straight into host memory.  Wraps hipHostRegister(Mapped) +
 * hipHostGetDevicePointer; regions are recorded process-wide so that the
 * element glue can find them (clk_host_lookup).                            */
int clk_host_register(clk_ctx *ctx, void *host, size_t bytes, void **dev_base);
int clk_host_unregister(clk_ctx *ctx, void *host);
/* The registered region containing [p, p + len): its host start, size and
 * device base (each nullable); returns 0, or CLK_EINVAL when no registered
 * region contains it.                                                      */
int clk_host_lookup(const void *p, size_t len, void **host_start, size_t *bytes, void **dev_base);

/* ---- batch utilities ------------------------------------------------------- */

/* counts[c] += number of i with codes[i] == c, for c < ncounts (device u64). */
int clk_count_codes(clk_ctx *ctx, const uint8_t *codes, uint64_t n,
                    uint64_t *counts, uint32_t ncounts);

/* Synthetic traffic (bench/test source, like InfiniteSource/RandomSource):
 * writes len_i bytes of packet (first_idx + i): IPv4 header (ihl 5, ttl 64,
 * protocol `proto`: 17 UDP, 6 TCP), transport header, pseudo-random payload
 * from splitmix64; every checksum field is 0.  Bytes past len_i in a slot
 * are not touched.                                                           */
int clk_gen_packets(clk_ctx *ctx, const clk_batch *batch, int proto,
                    uint64_t seed, uint64_t first_idx);
/* Flip one payload bit in every packet whose hash(seed, i) has its low
 * `rate_log2` bits zero (1 in 2^rate_log2), for Check-mode drop tests.      */
int clk_gen_corrupt(clk_ctx *ctx, const clk_batch *batch, uint64_t seed,
                    uint32_t rate_log2);
/* The same with the pick hashed on the global index first_idx + i and the
 * flipped byte drawn from [lo, min(hi, len_i)) (hi = 0: len_i; lo = ~0u:
 * the default payload span of clk_gen_corrupt).  Calling it twice with the
 * same arguments restores the batch.                                        */
int clk_gen_corrupt_span(clk_ctx *ctx, const clk_batch *batch, uint64_t seed, uint64_t first_idx,
                         uint32_t rate_log2, uint32_t lo, uint32_t hi);

/* Sum of `bytes` starting at device `base`, read once as 16-byte loads: the
 * measured HBM read-stream ceiling for the roofline (bench only).          */
int clk_read_stream(clk_ctx *ctx, const void *base, uint64_t bytes, uint64_t *out_sum);

/* The measured copy ceiling (bench only): `bytes` from device src to dst as
 * 16-byte nontemporal loads, shape 0-3 = 4 / 8 loads in flight per lane,
 * nontemporal / plain stores; 5 = 16 in flight, plain; 6 = each wave 8 KiB
 * contiguous per step; 7 = one step per thread over a grid covering the
 * buffer; shape 4 = the IMIX Set's traffic, src read once and one 64-byte
 * block in six written back in place (dst unused, out_sum as
 * clk_read_stream's).  16-byte aligned.                                    */
int clk_copy_stream(clk_ctx *ctx, void *dst, const void *src, uint64_t bytes, int shape, uint64_t *out_sum);

#ifdef __cplusplus
}
#endif
#endif /* CLICK_AMD_CKSUM_H */
