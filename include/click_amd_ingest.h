/*
 * click_amd_ingest.h -- host ingest of pcap files into a struct-of-arrays
 * batch ("Host ingest -> pinned SoA staging (DPDK
 * bursts, pcap)").
 *
 * clk_pcap_read() is FromDump(FILENAME, FORCE_IP b) without its timing,
 * sampling and START/END options: it reads every record of a tcpdump file
 * (elements/userlevel/fromdump.cc:202-290 file header, 328-413 records)
 * into one caller arena -- pinned, or registered with clk_host_register
 * for zero-copy -- and reports per record where its bytes are and, with
 * FORCE_IP, where its IP header is (elements/userlevel/fakepcap.cc:121-330).
 * The records' IP headers then form a clk_batch (base = arena, off[k] +
 * nh[k], caplen[k] - nh[k]) for the checksum elements.  Host code only:
 * no context, no GPU.
 */
#ifndef CLICK_AMD_INGEST_H
#define CLICK_AMD_INGEST_H
#include <stdint.h>
#include <stddef.h>
#include "click_amd_cksum.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct clk_pcap_info {
    int32_t linktype;      /* canonical DLT (fakepcap.cc:95-101: 12 -> 101)       */
    int32_t nanosecond;    /* FAKE_PCAP_MAGIC_NANO file                           */
    int32_t swapped;       /* file written with the other byte order             */
    int32_t force_ip;      /* FORCE_IP in effect (asked, or DLT_RAW: 256-257)     */
    uint64_t records;      /* records in the file (all of them, IP or not)       */
    uint64_t arena_bytes;  /* arena bytes the records need (16 B-aligned starts) */
    uint64_t ip_records;   /* records with nh[k] >= 0                            */
} clk_pcap_info;

/* Read the tcpdump file `path`.
 *   arena == NULL: sizing pass -- only *info is filled.
 *   otherwise record k's captured bytes are copied to arena + off[k]
 *   (off[k] a multiple of 16), its captured length to caplen[k] (after
 *   FromDump's caplen > len repair, 362-368), its wire length to wire_len[k]
 *   (nullable; EXTRA_LENGTH_ANNO = wire_len - caplen, 407), its timestamp in
 *   ns to ts_ns[k] (nullable), and nh[k] = the IP header's offset within the
 *   record when FORCE_IP finds one (fakepcap.cc:121-330: an IPv4 header with
 *   ip_hl >= 5 inside the record, or an IPv6 header), else -1 -- FromDump
 *   pushes such records to output 1 (461-464).  Without FORCE_IP nh[k] = -1.
 * Records past max_records are counted in info->records but not stored.
 * Errors (CLK_EINVAL, clk_last_error(NULL)): the file's own FromDump
 * messages -- "not a tcpdump file (too short)", "not a tcpdump file (bad
 * magic number)", "unknown major version N", "unknown linktype N; can't
 * force IP packets", "bad packet header; giving up" -- or an arena too small. */
int clk_pcap_read(const char *path, int force_ip, uint8_t *arena, uint64_t arena_bytes,
                  uint64_t *off, uint32_t *caplen, uint32_t *wire_len, uint64_t *ts_ns, int32_t *nh,
                  uint64_t max_records, clk_pcap_info *info);

/* FORCE_IP for one record (fakepcap.cc:121-330) on host bytes: the IP
 * header's offset within [data, data + len), or -1. */
int32_t clk_pcap_force_ip(const uint8_t *data, uint32_t len, int32_t linktype);

#ifdef __cplusplus
}
#endif
#endif
