/*
 * cksum_oracle.h -- CPU restatement of Click's Internet-checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the HIP kernels
 * in click_amd/csrc.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library never links it.
 *
 * Every function restates the reference algorithm and cites the reference
 * line it follows (paths are relative to the kohler/click tree).  Parity is
 * pinned by the golden vectors in tests/golden/, which are taken from the
 * reference's own test files (see tests/golden/make_golden.py); the
 * reference lib/in_cksum.c itself cannot be compiled here without the
 * configure-generated <click/config.h> ("Oracle").
 *
 * Byte order: like the reference on x86-64, 16-bit words are read in host
 * (little-endian) order; gfx950 is little-endian too.
 */
#ifndef CLICK_AMD_CKSUM_ORACLE_H
#define CLICK_AMD_CKSUM_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- lib/in_cksum.c and include/clicknet/ip.h ---------------------------- */
uint16_t oracle_in_cksum(const uint8_t *addr, int len);
uint16_t oracle_in_cksum_pseudohdr_raw(uint32_t csum, uint32_t src, uint32_t dst,
                                       int proto, int packet_len);
uint16_t oracle_in_cksum_pseudohdr_hard(uint32_t csum, const uint8_t *iph, int packet_len);
uint16_t oracle_in_cksum_pseudohdr(uint32_t csum, const uint8_t *iph, int transport_len);
uint16_t oracle_update_in_cksum(uint16_t csum, uint16_t old_hw, uint16_t new_hw);
uint16_t oracle_update_zero_in_cksum(uint16_t csum, const uint8_t *x, int len);

/* ---- element simple_action()s, one packet -------------------------------
 * Codes are the ones include/click_amd_cksum.h exports (CLK_*): 0 = the
 * packet leaves on output 0; otherwise 1 + the element's Reason enum value
 * (checks) or a set status (sets).                                          */
int oracle_check_ip_header(const uint8_t *data, uint32_t length, uint32_t offset,
                           int checksum, const uint32_t *badsrc, int nbadsrc,
                           const uint32_t *gooddst, int ngooddst);
int oracle_set_ip_checksum(uint8_t *nh, uint32_t plen);
int oracle_check_udp_header(const uint8_t *nh, uint32_t caplen);
int oracle_set_udp_checksum(uint8_t *nh, uint32_t caplen);
int oracle_check_tcp_header(const uint8_t *nh, uint32_t caplen);
int oracle_set_tcp_checksum(uint8_t *nh, uint32_t caplen, int fixoff);
int oracle_check_icmp_header(const uint8_t *nh, uint32_t caplen);
int oracle_dec_ip_ttl(uint8_t *nh, uint32_t caplen, int multicast);
/* The same L4 elements with the transport header where its annotation puts
 * it, th bytes past the network header (udp_header(), tcp_header(),
 * icmp_header(), transport_length(): checkudpheader.cc:84-107,
 * setudpchecksum.cc:37-69, checktcpheader.cc:85-107,
 * settcpchecksum.cc:44-75, checkicmpheader.cc:83-141); th = ip_hl*4 gives
 * the functions above.  proto 17 / 6 / 1.  has_th = 0: no transport header
 * (SetTCPChecksum kills, settcpchecksum.cc:53). */
int oracle_check_l4_at(int proto, const uint8_t *nh, uint32_t caplen, uint32_t th);
int oracle_set_l4_at(int proto, uint8_t *nh, uint32_t caplen, uint32_t th, int has_th, int fixoff);

/* ---- IP output path (ipgwoptions.cc, fixipsrc.cc, ipoutputcombo.cc) ------
 * ts = the 4 bytes stored for Timestamp::now() (htonl(ms since midnight)). */
int oracle_ip_gw_options(uint8_t *ip, uint32_t caplen, uint32_t my_ip, const uint32_t *my_addrs,
                         int n_my_addrs, uint32_t ts, int *problem, int *touched, int *changed);
int oracle_ip_gw_options_element(uint8_t *ip, uint32_t caplen, uint32_t my_ip, const uint32_t *my_addrs,
                                 int n_my_addrs, uint32_t ts, int *problem);
int oracle_fix_ip_src(uint8_t *ip, uint32_t caplen, int anno, uint32_t my_ip);
int oracle_ip_output_combo(uint8_t *ip, uint32_t caplen, uint32_t length, int flags, uint32_t my_ip,
                           uint32_t mtu, uint32_t ts, int *problem);

/* Batch form of the three (op: 0 IPGWOptions, 1 FixIPSrc, 2 IPOutputCombo);
 * flags[i] bit 0 = FIX_IP_SRC_ANNO (NULL: 0); out8 = code / port, out_prob =
 * parameter-problem offsets; out16 = the stored ip_sum. */
int oracle_ip_out_batch(int op, uint8_t *base, const uint64_t *off, uint64_t stride,
                        const uint32_t *len, uint32_t fixed_len, uint64_t n,
                        const uint8_t *flags, uint32_t my_ip, const uint32_t *my_addrs, int n_my_addrs,
                        uint32_t ts, uint32_t mtu, uint8_t *out8, uint8_t *out_prob, uint16_t *out16);

/* ---- IPFragmenter (elements/ip/ipfragmenter.cc:53-171) -------------------- */
int oracle_ip_fragment(uint8_t *ip, uint32_t caplen, uint32_t mtu, int honor_df, int new_id,
                       uint8_t *arena, uint64_t *arena_pos, uint64_t *frag_off, uint32_t *frag_len,
                       uint64_t *nfrag, uint32_t *first_len);
int oracle_ip_fragment_batch(uint8_t *base, const uint64_t *off, uint64_t stride, const uint32_t *len,
                             uint32_t fixed_len, uint64_t n, uint32_t mtu, int honor_df, const uint16_t *new_id,
                             uint8_t *out_port, uint32_t *out_first_len, uint64_t *out_frag_first,
                             uint8_t *arena, uint64_t *frag_off, uint32_t *frag_len, uint32_t *frag_src,
                             uint64_t *totals);

/* ---- batch drivers with the C-ABI's batch semantics ----------------------
 * Packet i starts at base + (off ? off[i] : i*stride) and has
 * (len ? len[i] : fixed_len) bytes.                                          */
enum {
    ORACLE_OP_IN_CKSUM = 0,   /* out16[i] = click_in_cksum(pkt, len)            */
    ORACLE_OP_CHECK_IP = 1,   /* out8[i] = verdict; arg = CHECKSUM flag         */
    ORACLE_OP_SET_IP = 2,     /* out8 status, out16 stored ip_sum               */
    ORACLE_OP_CHECK_UDP = 3,
    ORACLE_OP_SET_UDP = 4,    /* out16 stored uh_sum                             */
    ORACLE_OP_CHECK_TCP = 5,
    ORACLE_OP_SET_TCP = 6,    /* arg = FIXOFF; out16 stored th_sum               */
    ORACLE_OP_CHECK_ICMP = 7,
    ORACLE_OP_DEC_TTL = 8,    /* arg = MULTICAST; out16 stored ip_sum            */
};
int oracle_batch(int op, uint8_t *base, const uint64_t *off, uint64_t stride,
                 const uint32_t *len, uint32_t fixed_len, uint64_t n, int arg,
                 uint8_t *out8, uint16_t *out16);

/* ---- synthetic packet generator (same bytes as clk_gen_packets) ---------- */
uint64_t oracle_splitmix64(uint64_t x);
void oracle_gen_packet(uint8_t *pkt, uint32_t length, int proto, uint64_t seed, uint64_t idx);
void oracle_gen_batch(uint8_t *base, const uint64_t *off, uint64_t stride,
                      const uint32_t *len, uint32_t fixed_len, uint64_t n,
                      int proto, uint64_t seed, uint64_t first_idx);

/* ---- CPU baseline timing (bench.py cpu_baseline leg) ---------------------
 * Runs `op` over the batch `reps` times on `nthreads` threads (disjoint
 * contiguous shards) and returns the wall seconds of the timed passes.     */
double oracle_bench(int op, uint8_t *base, uint64_t stride, uint32_t fixed_len,
                    uint64_t n, int reps, int nthreads);

/* CPU baseline per BASELINE.md §2 (bench.py cpu_baseline): `nthreads`
 * threads, thread t pinned to cpus[t] (NULL: unpinned) BEFORE it allocates
 * and generates its own DRAM-resident shard of bytes_per_thread (NUMA-local
 * first touch); a warm-up pass, then `reps` passes between barriers; the
 * median / min / max pass wall time and the per-pass totals are returned.  */
struct oracle_cb_cfg {
    int op, arg, proto, imix;
    uint32_t fixed_len;
    uint64_t stride, bytes_per_thread, seed;
    int reps;
};
struct oracle_cb_result {
    double median_s, min_s, max_s, gen_s;
    uint64_t packets, bytes, ok;      /* per pass, all threads */
    int pinned;                       /* threads whose affinity call succeeded */
};
int oracle_cpu_baseline(const struct oracle_cb_cfg *cfg, const int *cpus, int nthreads,
                        struct oracle_cb_result *res);

/* bench.py self-verification: the oracle's digest of one rank's work, packet
 * by packet from global indices [first_idx, first_idx + n) (see the .c). */
enum {
    ORACLE_DG_CHECK_L4 = 0,   /* CheckUDPHeader / CheckTCPHeader on the corrupted packet */
    ORACLE_DG_SET_L4 = 1,     /* SetUDPChecksum / SetTCPChecksum                          */
    ORACLE_DG_CHECK_IP = 2,   /* CheckIPHeader, corruption in [ip_lo, ip_hi)              */
    ORACLE_DG_SET_IP = 3,     /* SetIPChecksum                                            */
    ORACLE_DG_DEC_TTL = 4,    /* DecIPTTL(MULTICAST true), ttl_runs passes from TTL 255   */
    ORACLE_DG_OUT_COMBO = 5,  /* IPOutputCombo(my_ip, mtu), ttl_runs passes from TTL 255  */
    ORACLE_DG_NLEGS = 6
};
struct oracle_digest_cfg {
    int proto, imix;
    uint32_t fixed_len;
    uint32_t legs;            /* bit mask of ORACLE_DG_* */
    uint64_t seed, first_idx, n;
    uint64_t corrupt_seed;
    uint32_t corrupt_log2, ip_lo, ip_hi;
    int ttl_runs;
    uint32_t my_ip, mtu;
};
struct oracle_digest_leg {
    uint64_t ok, packets, sum16, xor16, wsum16, wcode;
};
int oracle_digest(const struct oracle_digest_cfg *cfg, const int *cpus, int nthreads,
                  struct oracle_digest_leg *out);

#ifdef __cplusplus
}
#endif
#endif
