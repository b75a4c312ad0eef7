/*
 * cksum_oracle.c -- CPU restatement of Click's Internet-checksum path.
 *
 * TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline); the
 * product library in click_amd/ never links or calls this file.
 *
 * Restated from the reference (kohler/click 2.1):
 *   lib/in_cksum.c:20-51    click_in_cksum
 *   lib/in_cksum.c:53-80    click_in_cksum_pseudohdr_raw (portable branch 74-78;
 *                           the i386 asm branch 58-72 is not on x86-64/gfx950)
 *   lib/in_cksum.c:83-111   click_in_cksum_pseudohdr_hard
 *   lib/in_cksum.c:113-121  click_update_zero_in_cksum_hard
 *   include/clicknet/ip.h:152-160  click_in_cksum_pseudohdr (dispatch)
 *   include/clicknet/ip.h:177-185  click_update_in_cksum (RFC 1624)
 *   elements/ip/checkipheader.cc:161-226   CheckIPHeader::simple_action
 *   elements/ip/setipchecksum.cc:74-95     SetIPChecksum::simple_action
 *   elements/tcpudp/checkudpheader.cc:84-107  CheckUDPHeader::simple_action
 *   elements/tcpudp/setudpchecksum.cc:37-69   SetUDPChecksum::simple_action
 *   elements/tcpudp/checktcpheader.cc:85-107  CheckTCPHeader::simple_action
 *   elements/tcpudp/settcpchecksum.cc:44-75   SetTCPChecksum::simple_action
 *
 * Built with Click's own optimisation flags (-O2 -g, userlevel/Makefile.in:85-86)
 * by oracle/Makefile.  Parity: see cksum_oracle.h and DESIGN.md.
 */
#define _GNU_SOURCE
#include "cksum_oracle.h"
#include <string.h>
#include <pthread.h>
#include <time.h>
#include <stdlib.h>

/* Codes shared with include/click_amd_cksum.h (tests assert they agree). */
#define CLK_OK 0
#define CLK_IP_MINISCULE_PACKET 1
#define CLK_IP_BAD_VERSION 2
#define CLK_IP_BAD_HLEN 3
#define CLK_IP_BAD_IP_LEN 4
#define CLK_IP_BAD_CHECKSUM 5
#define CLK_IP_BAD_SADDR 6
#define CLK_L4_NOT_PROTO 1
#define CLK_L4_BAD_LENGTH 2
#define CLK_L4_BAD_CHECKSUM 3
#define CLK_SET_OUTPUT1 1
#define CLK_SET_KILL 2
#define CLK_TTL_EXPIRED 1
#define CLK_TTL_UNCHANGED 2
#define CLK_GWOPT_ERROR 1

static inline uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline void st16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }
/* htons/ntohs on a little-endian host; the argument is truncated to 16 bits
 * exactly as glibc's __bswap_16(uint16_t) does for htons(int). */
static inline uint16_t bswap16(uint32_t v) { v &= 0xFFFF; return (uint16_t)((v >> 8) | (v << 8)); }

/* lib/in_cksum.c:20-51.  32-bit accumulator with silent wrap (25,34), odd
 * trailing byte added as the low byte of a zero word (39-42), two-step carry
 * fold (45-46), complement truncated to 16 bits (49).  `len` is an int: a
 * negative length sums nothing, exactly as the reference's while loop. */
uint16_t oracle_in_cksum(const uint8_t *addr, int len)
{
    int nleft = len;
    const uint8_t *w = addr;
    uint32_t sum = 0;
    while (nleft > 1) {
        sum += ld16(w);
        w += 2;
        nleft -= 2;
    }
    if (nleft == 1)
        sum += *w;
    sum = (sum & 0xffff) + (sum >> 16);
    sum += (sum >> 16);
    return (uint16_t)~sum;
}

/* lib/in_cksum.c:53-80, portable branch (74-78). */
uint16_t oracle_in_cksum_pseudohdr_raw(uint32_t csum, uint32_t src, uint32_t dst,
                                       int proto, int packet_len)
{
    csum = ~csum & 0xFFFF;                                  /* 57 */
    csum += (src & 0xffff) + (src >> 16);                   /* 74 */
    csum += (dst & 0xffff) + (dst >> 16);                   /* 75 */
    csum += bswap16((uint32_t)packet_len) + bswap16((uint32_t)proto); /* 76 */
    csum = (csum & 0xffff) + (csum >> 16);                  /* 77 */
    return (uint16_t)(~(csum + (csum >> 16)) & 0xFFFF);     /* 78 */
}

/* lib/in_cksum.c:83-111: option walk for the source-route final destination. */
uint16_t oracle_in_cksum_pseudohdr_hard(uint32_t csum, const uint8_t *iph, int packet_len)
{
    const uint8_t *opt = iph + 20;                          /* 86 */
    const uint8_t *end_opt = iph + ((iph[0] & 0xF) << 2);   /* 87 */
    while (opt < end_opt) {                                 /* 88 */
        if (*opt == 1) {                                    /* IPOPT_NOP, 90-92 */
            opt++;
            continue;
        } else if (*opt == 0)                               /* IPOPT_EOL, 93-94 */
            break;
        if (opt + 1 >= end_opt || opt[1] < 2 || opt + opt[1] > end_opt) /* 97-98 */
            break;
        if ((*opt == 137 || *opt == 131) && opt[1] >= 7) {  /* SSRR/LSRR, 101-105 */
            uint32_t daddr = ld32(opt + opt[1] - 4);
            return oracle_in_cksum_pseudohdr_raw(csum, ld32(iph + 12), daddr, iph[9], packet_len);
        }
        opt += opt[1];                                      /* 107 */
    }
    return oracle_in_cksum_pseudohdr_raw(csum, ld32(iph + 12), ld32(iph + 16), iph[9], packet_len); /* 110 */
}

/* include/clicknet/ip.h:152-160 */
uint16_t oracle_in_cksum_pseudohdr(uint32_t csum, const uint8_t *iph, int transport_len)
{
    if ((iph[0] & 0xF) == 5)
        return oracle_in_cksum_pseudohdr_raw(csum, ld32(iph + 12), ld32(iph + 16), iph[9], transport_len);
    return oracle_in_cksum_pseudohdr_hard(csum, iph, transport_len);
}

/* include/clicknet/ip.h:177-185 (RFC 1624). */
uint16_t oracle_update_in_cksum(uint16_t csum, uint16_t old_hw, uint16_t new_hw)
{
    uint32_t sum = (~(uint32_t)csum & 0xFFFF) + (~(uint32_t)old_hw & 0xFFFF) + new_hw;
    sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~(sum + (sum >> 16));
}

/* include/clicknet/ip.h:196-201 + lib/in_cksum.c:113-121. */
uint16_t oracle_update_zero_in_cksum(uint16_t csum, const uint8_t *x, int len)
{
    if (csum != 0)
        return csum;
    for (; len > 0; --len, ++x)
        if (*x)
            return csum;
    return (uint16_t)~0;
}

/* ---- elements ------------------------------------------------------------ */

/* elements/ip/checkipheader.cc:161-226.  `data`/`length` are the packet's
 * data() and length(); OFFSET is `offset` (checkipheader.cc:163-164). */
int oracle_check_ip_header(const uint8_t *data, uint32_t length, uint32_t offset,
                           int checksum, const uint32_t *badsrc, int nbadsrc,
                           const uint32_t *gooddst, int ngooddst)
{
    const uint8_t *ip = data + offset;
    uint32_t plen = length - offset;
    if ((int)plen < 20)                                     /* 168-170 */
        return CLK_IP_MINISCULE_PACKET;
    if ((ip[0] >> 4) != 4)                                  /* 172-173 */
        return CLK_IP_BAD_VERSION;
    uint32_t hlen = (uint32_t)(ip[0] & 0xF) << 2;           /* 175-177 */
    if (hlen < 20)
        return CLK_IP_BAD_HLEN;
    uint32_t len = bswap16(ld16(ip + 2));                   /* 179-181 */
    if (len > plen || len < hlen)
        return CLK_IP_BAD_IP_LEN;
    if (checksum && oracle_in_cksum(ip, (int)hlen) != 0)    /* 183-197, userlevel branch 193 */
        return CLK_IP_BAD_CHECKSUM;
    /* 204-206: BADSRC unless GOODDST */
    uint32_t src = ld32(ip + 12), dst = ld32(ip + 16);
    int bad = 0, good = 0;
    for (int i = 0; i < nbadsrc; i++)
        if (badsrc[i] == src) { bad = 1; break; }
    if (bad) {
        for (int i = 0; i < ngooddst; i++)
            if (gooddst[i] == dst) { good = 1; break; }
        if (!good)
            return CLK_IP_BAD_SADDR;
    }
    return CLK_OK;
}

/* elements/ip/setipchecksum.cc:74-95; `plen` = end_data() - nh_data (80). */
int oracle_set_ip_checksum(uint8_t *iph, uint32_t plen)
{
    uint32_t hlen;
    if (plen >= 20 && (hlen = (uint32_t)(iph[0] & 0xF) << 2) >= 20 && hlen <= plen) { /* 82-84 */
        st16(iph + 10, 0);                                  /* 85 */
        st16(iph + 10, oracle_in_cksum(iph, (int)hlen));    /* 86 */
        return CLK_OK;
    }
    return CLK_SET_KILL;                                    /* 90-92 */
}


/* elements/tcpudp/checkudpheader.cc:84-107.  `nh`/`caplen` are the network
 * header and the bytes from it to end_data(); the transport header is
 * nh + ip_hl*4, as CheckIPHeader/MarkIPHeader set it.  Domain guards, which
 * replace only reads the reference would make outside the packet:
 *   caplen < 20      -> BAD_LENGTH (no full base IP header to read)
 *   caplen < hl + 8  -> BAD_LENGTH (the reference returns BAD_LENGTH for any
 *                       uh_ulen it could read there, 94-98). */
int oracle_check_udp_header(const uint8_t *nh, uint32_t caplen)
{
    if (caplen < 20)
        return CLK_L4_BAD_LENGTH;
    if (nh[9] != 17)                                        /* 91-92 */
        return CLK_L4_NOT_PROTO;
    uint32_t iph_len = (uint32_t)(nh[0] & 0xF) << 2;        /* 94 */
    if (caplen < iph_len + 8)
        return CLK_L4_BAD_LENGTH;
    const uint8_t *udph = nh + iph_len;
    uint32_t len = bswap16(ld16(udph + 4));                 /* 95 */
    if (len < 8 || caplen < len + iph_len)                  /* 96-98 */
        return CLK_L4_BAD_LENGTH;
    if (ld16(udph + 6) != 0) {                              /* 100 */
        unsigned csum = oracle_in_cksum(udph, (int)len);    /* 101 */
        if (oracle_in_cksum_pseudohdr(csum, nh, (int)len) != 0) /* 102-103 */
            return CLK_L4_BAD_CHECKSUM;
    }
    return CLK_OK;
}

/* elements/tcpudp/setudpchecksum.cc:37-69.  tlen = transport_length().
 * Domain guard: caplen < 20 -> OUTPUT1 (no full base IP header). */
int oracle_set_udp_checksum(uint8_t *nh, uint32_t caplen)
{
    if (caplen < 20)
        return CLK_SET_OUTPUT1;
    uint32_t hl = (uint32_t)(nh[0] & 0xF) << 2;
    int tlen = (int)caplen - (int)hl;
    uint8_t *udph = nh + hl;
    int len;
    int isfrag = (bswap16(ld16(nh + 6)) & 0x3FFF) != 0;     /* IP_ISFRAG, ip.h:121 */
    if (isfrag || tlen < 8                                  /* 48-51 */
        || (len = bswap16(ld16(udph + 4)), tlen < len))
        return CLK_SET_OUTPUT1;                             /* 52-61 */
    st16(udph + 6, 0);                                      /* 64 */
    unsigned csum = oracle_in_cksum(udph, len);             /* 65 */
    st16(udph + 6, oracle_in_cksum_pseudohdr(csum, nh, len)); /* 66 */
    return CLK_OK;
}

/* elements/tcpudp/checktcpheader.cc:85-107.  Unsigned length arithmetic as
 * in the reference (len = ip_len - hl may wrap; click_in_cksum then takes a
 * negative int and sums nothing).  Domain guards: caplen < 20 -> BAD_LENGTH;
 * caplen < hl + 13 (th_off unreadable) -> BAD_LENGTH, which is what the
 * reference returns for every th_off it could read there unless ip_len < hl. */
int oracle_check_tcp_header(const uint8_t *nh, uint32_t caplen)
{
    if (caplen < 20)
        return CLK_L4_BAD_LENGTH;
    if (nh[9] != 6)                                         /* 92-93 */
        return CLK_L4_NOT_PROTO;
    uint32_t iph_len = (uint32_t)(nh[0] & 0xF) << 2;        /* 95 */
    uint32_t len = (uint32_t)bswap16(ld16(nh + 2)) - iph_len; /* 96 */
    if (caplen < iph_len + 13)
        return CLK_L4_BAD_LENGTH;
    const uint8_t *tcph = nh + iph_len;
    uint32_t tcph_len = (uint32_t)(tcph[12] >> 4) << 2;     /* 97 */
    if (tcph_len < 20 || len < tcph_len || caplen < len + iph_len) /* 98-100 */
        return CLK_L4_BAD_LENGTH;
    unsigned csum = oracle_in_cksum(tcph, (int)len);        /* 102 */
    if (oracle_in_cksum_pseudohdr(csum, nh, (int)len) != 0) /* 103-104 */
        return CLK_L4_BAD_CHECKSUM;
    return CLK_OK;
}

/* elements/tcpudp/settcpchecksum.cc:44-75.  Domain guard: hl > caplen
 * (negative transport_length, where the reference would read and write
 * outside the packet) -> KILL. */
int oracle_set_tcp_checksum(uint8_t *nh, uint32_t caplen, int fixoff)
{
    if (caplen < 20)
        return CLK_SET_KILL;
    uint32_t hl = (uint32_t)(nh[0] & 0xF) << 2;
    if (hl > caplen)
        return CLK_SET_KILL;
    uint8_t *tcph = nh + hl;
    uint32_t plen = (uint32_t)bswap16(ld16(nh + 2)) - hl;   /* 50 */
    uint32_t tlen = caplen - hl;
    if (plen < 20 || plen > tlen)                           /* 53-55 */
        return CLK_SET_KILL;                                /* 71-74 */
    if (fixoff) {                                           /* 57-63 */
        uint32_t off = (uint32_t)(tcph[12] >> 4) << 2;
        int isfrag = (bswap16(ld16(nh + 6)) & 0x3FFF) != 0;
        if (off < 20)
            tcph[12] = (uint8_t)((tcph[12] & 0x0F) | (5 << 4));
        else if (off > plen && !isfrag)
            tcph[12] = (uint8_t)((tcph[12] & 0x0F) | (((plen >> 2) & 0xF) << 4));
    }
    st16(tcph + 16, 0);                                     /* 65 */
    unsigned csum = oracle_in_cksum(tcph, (int)plen);       /* 66 */
    st16(tcph + 16, oracle_in_cksum_pseudohdr(csum, nh, (int)plen)); /* 67 */
    return CLK_OK;
}

/* elements/icmp/checkicmpheader.cc:83-141.  The transport header is the
 * one CheckIPHeader / MarkIPHeader set: nh + ip_hl*4 (set_ip_header).
 * Domain guards: caplen < 20 -> BAD_LENGTH (no full base IP header);
 * caplen < hl -> BAD_LENGTH (icmp_len would wrap and the reference would
 * read the type byte outside the packet). */
int oracle_check_icmp_header(const uint8_t *nh, uint32_t caplen)
{
    if (caplen < 20)
        return CLK_L4_BAD_LENGTH;
    if (nh[9] != 1)                                         /* 89-90, IP_PROTO_ICMP */
        return CLK_L4_NOT_PROTO;
    uint32_t hl = (uint32_t)(nh[0] & 0xF) << 2;
    if (caplen < hl)
        return CLK_L4_BAD_LENGTH;
    uint32_t icmp_len = caplen - hl;                        /* 92 */
    if (icmp_len < 8)                                       /* 93-94, sizeof(click_icmp) */
        return CLK_L4_BAD_LENGTH;
    const uint8_t *icmph = nh + hl;
    switch (icmph[0]) {                                     /* 96-134 */
    case 3: case 11: case 12: case 4: case 5:   /* UNREACH TIMXCEED PARAMPROB SOURCEQUENCH REDIRECT */
        if (icmp_len < 8 + 28)
            return CLK_L4_BAD_LENGTH;
        break;
    case 13: case 14:                           /* TSTAMP TSTAMPREPLY: sizeof(click_icmp_tstamp) */
        if (icmp_len != 20)
            return CLK_L4_BAD_LENGTH;
        break;
    case 15: case 16:                           /* IREQ IREQREPLY */
        if (icmp_len != 8)
            return CLK_L4_BAD_LENGTH;
        break;
    default:
        break;
    }
    if ((oracle_in_cksum(icmph, (int)icmp_len) & 0xFFFF) != 0)  /* 136-138 */
        return CLK_L4_BAD_CHECKSUM;
    return CLK_OK;
}

/* ---- the L4 elements, transport header at its annotation -------------------
 * Header fields (ip_p, ip_hl for the lengths, ip_len, ip_off) come from the
 * IP header bytes, the segment from nh + th, as the reference reads them.
 * Domain guards where the reference would read outside the packet: caplen <
 * 20 as above; the transport fields read and the summed segment must lie in
 * [0, caplen) (else BAD_LENGTH, output 1 or kill, as a short packet); the
 * pseudo-header's option walk stops at caplen.  Test infrastructure: the
 * checker of the glue's irregular-annotation path (clk_element_push_th). */
static uint16_t pseudohdr_clamped(uint32_t csum, const uint8_t *iph, uint32_t caplen, int len)
{
    uint32_t dst = ld32(iph + 16);
    uint32_t hl = (uint32_t)(iph[0] & 0xF) << 2;
    if ((iph[0] & 0xF) != 5) {                              /* ip.h:156-159 -> in_cksum.c:83-108 */
        uint32_t end = hl < caplen ? hl : caplen, o = 20;
        while (o < end) {
            if (iph[o] == 1) {
                o++;
                continue;
            } else if (iph[o] == 0)
                break;
            if (o + 1 >= end || iph[o + 1] < 2 || o + iph[o + 1] > end)
                break;
            if ((iph[o] == 137 || iph[o] == 131) && iph[o + 1] >= 7) {
                dst = ld32(iph + o + iph[o + 1] - 4);
                break;
            }
            o += iph[o + 1];
        }
    }
    return oracle_in_cksum_pseudohdr_raw(csum, ld32(iph + 12), dst, iph[9], len);
}

int oracle_check_l4_at(int proto, const uint8_t *nh, uint32_t caplen, uint32_t th)
{
    if (caplen < 20)
        return CLK_L4_BAD_LENGTH;
    if (nh[9] != proto)                                     /* NOT_UDP / NOT_TCP / NOT_ICMP */
        return CLK_L4_NOT_PROTO;
    uint32_t iph_len = (uint32_t)(nh[0] & 0xF) << 2;
    const uint8_t *t = nh + th;
    uint32_t len;
    if (proto == 17) {                                      /* checkudpheader.cc:94-104 */
        if (th + 8 > caplen)
            return CLK_L4_BAD_LENGTH;
        len = bswap16(ld16(t + 4));
        if (len < 8 || (uint64_t)caplen < (uint64_t)len + iph_len || th + len > caplen)
            return CLK_L4_BAD_LENGTH;
        if (ld16(t + 6) == 0)
            return CLK_OK;
        return pseudohdr_clamped(oracle_in_cksum(t, (int)len), nh, caplen, (int)len) ? CLK_L4_BAD_CHECKSUM : CLK_OK;
    }
    if (proto == 6) {                                       /* checktcpheader.cc:95-104 */
        if (th + 13 > caplen)
            return CLK_L4_BAD_LENGTH;
        len = (uint32_t)bswap16(ld16(nh + 2)) - iph_len;
        uint32_t tcph_len = (uint32_t)(t[12] >> 4) << 2;
        if (tcph_len < 20 || len < tcph_len || (uint64_t)caplen < (uint64_t)len + iph_len || th + len > caplen)
            return CLK_L4_BAD_LENGTH;
        return pseudohdr_clamped(oracle_in_cksum(t, (int)len), nh, caplen, (int)len) ? CLK_L4_BAD_CHECKSUM : CLK_OK;
    }
    /* checkicmpheader.cc:92-141 on the segment [th, caplen) */
    if (th > caplen || caplen - th < 8)
        return CLK_L4_BAD_LENGTH;
    len = caplen - th;
    switch (t[0]) {
    case 3: case 11: case 12: case 4: case 5:
        if (len < 8 + 28)
            return CLK_L4_BAD_LENGTH;
        break;
    case 13: case 14:
        if (len != 20)
            return CLK_L4_BAD_LENGTH;
        break;
    case 15: case 16:
        if (len != 8)
            return CLK_L4_BAD_LENGTH;
        break;
    default:
        break;
    }
    return oracle_in_cksum(t, (int)len) != 0 ? CLK_L4_BAD_CHECKSUM : CLK_OK;
}

int oracle_set_l4_at(int proto, uint8_t *nh, uint32_t caplen, uint32_t th, int has_th, int fixoff)
{
    if (caplen < 20)
        return proto == 17 ? CLK_SET_OUTPUT1 : CLK_SET_KILL;
    uint8_t *t = nh + th;
    int isfrag = (bswap16(ld16(nh + 6)) & 0x3FFF) != 0;
    if (proto == 17) {                                      /* setudpchecksum.cc:44-66 */
        int tlen = th > caplen ? -1 : (int)(caplen - th);
        int len;
        if (isfrag || tlen < 8 || (len = bswap16(ld16(t + 4)), tlen < len))
            return CLK_SET_OUTPUT1;
        st16(t + 6, 0);
        unsigned csum = oracle_in_cksum(t, len);
        st16(t + 6, pseudohdr_clamped(csum, nh, caplen, len));
        return CLK_OK;
    }
    uint32_t hl = (uint32_t)(nh[0] & 0xF) << 2;             /* settcpchecksum.cc:50-67 */
    uint32_t plen = (uint32_t)bswap16(ld16(nh + 2)) - hl;
    if (!has_th || th > caplen || plen < 20 || plen > caplen - th)
        return CLK_SET_KILL;
    if (fixoff) {
        uint32_t off = (uint32_t)(t[12] >> 4) << 2;
        if (off < 20)
            t[12] = (uint8_t)((t[12] & 0x0F) | (5 << 4));
        else if (off > plen && !isfrag)
            t[12] = (uint8_t)((t[12] & 0x0F) | (((plen >> 2) & 0xF) << 4));
    }
    st16(t + 16, 0);
    unsigned csum = oracle_in_cksum(t, (int)plen);
    st16(t + 16, pseudohdr_clamped(csum, nh, caplen, (int)plen));
    return CLK_OK;
}

/* elements/ip/decipttl.cc:45-77 with ACTIVE true (ACTIVE false returns the
 * packet before reading it; the caller does not launch).  multicast =
 * the MULTICAST keyword.  Returns CLK_OK (TTL decremented, ip_sum updated
 * by RFC 1624, output 0), CLK_TTL_EXPIRED (ip_ttl <= 1: output 1) or
 * CLK_TTL_UNCHANGED (output 0 untouched).  Domain guard: caplen < 20 ->
 * UNCHANGED (the reference asserts a network header and reads ip_ttl,
 * ip_sum and ip_dst without a length check). */
int oracle_dec_ip_ttl(uint8_t *nh, uint32_t caplen, int multicast)
{
    if (caplen < 20)
        return CLK_TTL_UNCHANGED;
    if (!multicast && (nh[16] & 0xF0) == 0xE0)             /* 51-52, is_multicast */
        return CLK_TTL_UNCHANGED;
    if (nh[8] <= 1)                                         /* 54-57 */
        return CLK_TTL_EXPIRED;
    nh[8]--;                                                /* 63 */
    uint32_t sum = (~(uint32_t)bswap16(ld16(nh + 10)) & 0xFFFF) + 0xFEFF;  /* 72 */
    st16(nh + 10, (uint16_t)~bswap16((sum + (sum >> 16)) & 0xFFFF));     /* 73 */
    return CLK_OK;
}

/* Packet i of a batch (the C ABI's clk_batch semantics). */
static inline uint64_t pkt_off(const uint64_t *off, uint64_t stride, uint64_t i)
{ return off ? off[i] : i * stride; }
static inline uint32_t pkt_len(const uint32_t *len, uint32_t fixed_len, uint64_t i)
{ return len ? len[i] : fixed_len; }

/* ---- IP output path: IPGWOptions, FixIPSrc, IPOutputCombo ----------------
 * The option walk shared by IPGWOptions::handle_options
 * (elements/ip/ipgwoptions.cc:53-160) and IPOutputCombo::push's IPGWOptions
 * step (elements/ip/ipoutputcombo.cc:59-166).  my_ip = the address RR and
 * TS flg 1 record (IPGWOptions: the preferred address; IPOutputCombo:
 * IPADDR); my_addrs = the addresses TS flg 3 matches; ts = the 4 bytes the
 * reference stores for Timestamp::now() (htonl of ms since midnight), given
 * by the caller because a parity test cannot share the clock.  `caplen` =
 * bytes from the IP header to end_data(): an option byte the reference would
 * read at or past caplen reads as 0 (domain guard; the reference reads
 * packet tailroom there).  Returns 0 (options done), 1 (error: *problem =
 * the ICMP parameter-problem offset).  *touched: 1 if any RR/TS option was
 * reached (IPGWOptions' uniqueify), *changed: 1 if a byte was rewritten
 * (IPOutputCombo's do_cksum). */
static inline uint32_t optb(const uint8_t *o, uint32_t i, uint32_t caplen) { return i < caplen ? o[i] : 0; }

int oracle_ip_gw_options(uint8_t *ip, uint32_t caplen, uint32_t my_ip, const uint32_t *my_addrs,
                         int n_my_addrs, uint32_t ts, int *problem, int *touched, int *changed)
{
    int hlen = (ip[0] & 0xF) << 2;                          /* caller: hlen <= caplen */
    *touched = 0;
    *changed = 0;
    int oi;
    for (oi = 20; oi < hlen;) {
        unsigned type = ip[oi];
        if (type == 1) {                                    /* IPOPT_NOP */
            oi++;
            continue;
        } else if (type == 0)                               /* IPOPT_EOL */
            break;
        int xlen = (int)optb(ip, (uint32_t)oi + 1, caplen);
        if (xlen < 2 || oi + xlen > hlen) {                 /* bad length */
            *problem = oi + 1;
            return 1;
        } else if (type != 7 && type != 68) {               /* not IPOPT_RR / IPOPT_TS */
            oi += xlen;
            continue;
        }
        *touched = 1;
        if (type == 7) {                                    /* Record Route */
            int p = (int)optb(ip, (uint32_t)oi + 2, caplen) - 1;
            if (p >= 3 && p + 4 <= xlen) {
                memcpy(ip + oi + p, &my_ip, 4);
                ip[oi + 2] += 4;
                *changed = 1;
            } else if (p != xlen) {
                *problem = oi + 2;
                return 1;
            }
        } else {                                            /* Timestamp */
            int p = (int)optb(ip, (uint32_t)oi + 2, caplen) - 1;
            int oflw = (int)optb(ip, (uint32_t)oi + 3, caplen) >> 4;
            int flg = (int)optb(ip, (uint32_t)oi + 3, caplen) & 0xF;
            int overflowed = 0;
            if (p < 4) {
                *problem = oi + 2;
                return 1;
            } else if (flg == 0) {
                if (p + 4 <= xlen) {
                    memcpy(ip + oi + p, &ts, 4);
                    ip[oi + 2] += 4;
                    *changed = 1;
                } else
                    overflowed = 1;
            } else if (flg == 1) {
                if (p + 8 <= xlen) {
                    memcpy(ip + oi + p, &my_ip, 4);
                    memcpy(ip + oi + p + 4, &ts, 4);
                    ip[oi + 2] += 8;
                    *changed = 1;
                } else
                    overflowed = 1;
            } else if (flg == 3 && p + 8 <= xlen) {
                uint32_t addr = ld32(ip + oi + p);
                int mine = 0;
                for (int k = 0; k < n_my_addrs; k++)
                    if (my_addrs[k] == addr)
                        mine = 1;
                if (mine) {
                    memcpy(ip + oi + p + 4, &ts, 4);
                    ip[oi + 2] += 8;
                    *changed = 1;
                }
            } else {
                *problem = oi + 3;
                return 1;
            }
            if (overflowed) {
                if (oflw < 15) {
                    ip[oi + 3] = (uint8_t)(((oflw + 1) << 4) | flg);
                    *changed = 1;
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

/* elements/ip/ipgwoptions.cc:164-172 + 53-160.  Returns CLK_OK (output 0;
 * ip_sum recomputed when an RR/TS option was reached, 155-159) or
 * CLK_GWOPT_ERROR (output 1, *problem = ICMP_PARAMPROB_ANNO).  Domain guard:
 * caplen < 20 -> CLK_OK untouched (the reference asserts an IP header). */
int oracle_ip_gw_options_element(uint8_t *ip, uint32_t caplen, uint32_t my_ip, const uint32_t *my_addrs,
                                 int n_my_addrs, uint32_t ts, int *problem)
{
    int touched, changed;
    *problem = 0;
    if (caplen < 20 || ((ip[0] & 0xF) << 2) <= 20)          /* 168 */
        return CLK_OK;
    if ((uint32_t)((ip[0] & 0xF) << 2) > caplen)            /* domain guard: options past the packet */
        return CLK_OK;
    if (oracle_ip_gw_options(ip, caplen, my_ip, my_addrs, n_my_addrs, ts, problem, &touched, &changed))
        return CLK_GWOPT_ERROR;                             /* 162-165 */
    if (touched) {                                          /* 155-159 */
        int hlen = (ip[0] & 0xF) << 2;
        st16(ip + 10, 0);
        st16(ip + 10, oracle_in_cksum(ip, hlen));
    }
    return CLK_OK;
}

/* elements/ip/fixipsrc.cc:52-72: with FIX_IP_SRC_ANNO set, ip_src = IPADDR
 * and the header checksum is recomputed (hlen from ip_hl, no length check;
 * domain guard: caplen < 20 or hlen > caplen -> unchanged, CLK_OK). */
int oracle_fix_ip_src(uint8_t *ip, uint32_t caplen, int anno, uint32_t my_ip)
{
    if (!anno || caplen < 20)
        return CLK_OK;
    int hlen = (ip[0] & 0xF) << 2;
    if ((uint32_t)hlen > caplen)
        return CLK_OK;
    memcpy(ip + 12, &my_ip, 4);
    st16(ip + 10, 0);
    st16(ip + 10, oracle_in_cksum(ip, hlen));
    return CLK_OK;
}

/* elements/ip/ipoutputcombo.cc:44-205 after DropBroadcasts and PaintTee
 * (annotation-only steps the host takes): IPGWOptions (59-166, TS flg 3
 * matches IPADDR only), FixIPSrc (168-173), the header re-checksum when
 * either changed a byte (176-179, summed from data() = the IP header),
 * DecIPTTL (181-191), the MTU test (194-197; `length` = p->length()).
 * flags bit 0 = FIX_IP_SRC_ANNO.  Returns the output port: 0, 2 (*problem
 * set), 3 (TTL expired) or 4 (length > MTU).  Domain guard: caplen < 20 ->
 * port 0 untouched. */
int oracle_ip_output_combo(uint8_t *ip, uint32_t caplen, uint32_t length, int flags, uint32_t my_ip,
                           uint32_t mtu, uint32_t ts, int *problem)
{
    int touched = 0, changed = 0;
    *problem = 0;
    if (caplen < 20)
        return 0;
    int hlen = (ip[0] & 0xF) << 2;
    if (hlen > 20 && (uint32_t)hlen <= caplen &&           /* domain guard: options past the packet */
        oracle_ip_gw_options(ip, caplen, my_ip, &my_ip, 1, ts, problem, &touched, &changed))
        return 2;                                           /* 202-204 */
    if (flags & 1) {                                        /* 169-173 */
        memcpy(ip + 12, &my_ip, 4);
        changed = 1;
    }
    if (changed && (uint32_t)hlen <= caplen) {              /* 176-179 */
        st16(ip + 10, 0);
        st16(ip + 10, oracle_in_cksum(ip, hlen));
    }
    if (ip[8] <= 1)                                         /* 182-184 */
        return 3;
    ip[8]--;                                                /* 186 */
    uint32_t sum = (~(uint32_t)bswap16(ld16(ip + 10)) & 0xFFFF) + 0xFEFF;   /* 189 */
    st16(ip + 10, (uint16_t)~bswap16((sum + (sum >> 16)) & 0xFFFF));       /* 190 */
    if (length > mtu)                                       /* 194-197 */
        return 4;
    return 0;
}

/* ---- IPFragmenter ---------------------------------------------------------
 * elements/ip/ipfragmenter.cc:53-86 (optcopy): copy the options whose
 * copied-flag (0x80) is set, skip NOPs, stop at EOL or a malformed option,
 * pad to a multiple of 4 with EOL.  Returns the bytes written. */
static int frag_optcopy(const uint8_t *ip, uint8_t *oout)
{
    const uint8_t *oin = ip + 20;
    const uint8_t *oin_end = ip + ((ip[0] & 0xF) << 2);        /* 60 */
    int outpos = 0;
    while (oin < oin_end) {                                     /* 64 */
        if (*oin == 1)                                          /* NOP: not copied, 65-66 */
            ++oin;
        else if (*oin == 0 || oin + 1 == oin_end || oin[1] < 2 || oin + oin[1] > oin_end) /* 67-71 */
            break;
        else {
            if (*oin & 0x80) {                                  /* 73-77 */
                if (oout)
                    memcpy(oout + outpos, oin, oin[1]);
                outpos += oin[1];
            }
            oin += oin[1];                                      /* 78 */
        }
    }
    for (; (outpos & 3) != 0; outpos++)                         /* 81-83 */
        if (oout)
            oout[outpos] = 0;
    return outpos;
}

/* elements/ip/ipfragmenter.cc:88-171 (push + fragment) on one packet whose
 * IP header is at `ip` with `caplen` = network_length() bytes.  Returns the
 * port: 0 (network_length <= MTU, untouched), 1 (DF with HONOR_DF, or the
 * first fragment would carry < 8 data bytes: output 1), 2 (fragmented: the
 * packet becomes the first fragment in place, *first_len bytes from the IP
 * header; the others are appended at 16 B-aligned offsets of `arena`
 * starting at *arena_pos, descriptors at frag_off/frag_len[*nfrag ...]).
 * new_id (>= 0) replaces ip_id when DF is cleared (the reference uses
 * click_random(), 112-115; -1 keeps ip_id).  Domain guards: caplen < 20 with caplen > MTU
 * -> port 1; fragment bytes past caplen (ip_len > network_length, which
 * CheckIPHeader excludes) are written as 0.  With arena == NULL only the
 * counts are produced. */
int oracle_ip_fragment(uint8_t *ip, uint32_t caplen, uint32_t mtu, int honor_df, int new_id,
                       uint8_t *arena, uint64_t *arena_pos, uint64_t *frag_off, uint32_t *frag_len,
                       uint64_t *nfrag, uint32_t *first_len)
{
    *first_len = caplen;
    if (caplen <= mtu)                                          /* 167-168 */
        return 0;
    if (caplen < 20)
        return 1;
    int hlen = (ip[0] & 0xF) << 2;                              /* 92 */
    int first_dlen = ((int)mtu - hlen) & ~7;                    /* 93 */
    int in_dlen = (int)bswap16(ld16(ip + 2)) - hlen;            /* 94 */
    if (((ip[6] & 0x40) && honor_df) || first_dlen < 8)         /* 96-102: ip_off & htons(IP_DF) */
        return 1;
    if (ip[6] & 0x40) {                                         /* 112-115 */
        if (new_id >= 0)
            st16(ip + 4, (uint16_t)new_id);
        ip[6] &= (uint8_t)~0x40;
    }
    int had_mf = (ip[6] & 0x20) != 0;                           /* 116 */
    st16(ip + 2, bswap16((uint32_t)(hlen + first_dlen)));      /* 117 */
    ip[6] |= 0x20;                                              /* 118 */
    st16(ip + 10, 0);                                           /* 119 */
    st16(ip + 10, oracle_in_cksum(ip, hlen));                   /* 120 */
    *first_len = (uint32_t)(hlen + first_dlen);                 /* 121-122 */
    int out_hlen = 20 + frag_optcopy(ip, 0);                    /* 127 */
    const uint8_t *th = ip + hlen;
    for (int off = first_dlen; off < in_dlen;) {                /* 129 */
        int out_dlen = ((int)mtu - out_hlen) & ~7;              /* 131 */
        if (out_dlen + off > in_dlen)                           /* 132-133 */
            out_dlen = in_dlen - off;
        uint32_t qlen = (uint32_t)(out_hlen + out_dlen);
        if (arena) {
            uint8_t *q = arena + *arena_pos;
            memcpy(q, ip, 20);                                  /* 140 */
            frag_optcopy(ip, q + 20);                           /* 141 */
            for (int k = 0; k < out_dlen; k++) {                /* 142 */
                uint32_t s = (uint32_t)(hlen + off + k);
                q[out_hlen + k] = s < caplen ? th[off + k] : 0;
            }
            q[0] = (uint8_t)((q[0] & 0xF0) | ((out_hlen >> 2) & 0xF)); /* 144 */
            st16(q + 6, bswap16(bswap16(ld16(ip + 6)) + (uint32_t)(off >> 3))); /* 145 */
            if (out_dlen + off >= in_dlen && !had_mf)           /* 146-147 */
                q[6] &= (uint8_t)~0x20;
            st16(q + 2, bswap16(qlen));                         /* 148 */
            st16(q + 10, 0);                                    /* 149 */
            st16(q + 10, oracle_in_cksum(q, out_hlen));         /* 150 */
            frag_off[*nfrag] = *arena_pos;
            frag_len[*nfrag] = qlen;
        }
        *arena_pos += (qlen + 15) & ~15u;
        ++*nfrag;
        off += out_dlen;                                        /* 158 */
    }
    return 2;
}

/* Batch form: packets in order; fragments appended in packet order.
 * out_port[i], out_first_len[i]; out_frag_first[i] = index of packet i's
 * first appended fragment; totals[0] = fragments, totals[1] = arena bytes.
 * new_id (nullable: ip_id kept) per packet. */
int oracle_ip_fragment_batch(uint8_t *base, const uint64_t *off, uint64_t stride, const uint32_t *len,
                             uint32_t fixed_len, uint64_t n, uint32_t mtu, int honor_df, const uint16_t *new_id,
                             uint8_t *out_port, uint32_t *out_first_len, uint64_t *out_frag_first,
                             uint8_t *arena, uint64_t *frag_off, uint32_t *frag_len, uint32_t *frag_src,
                             uint64_t *totals)
{
    uint64_t pos = 0, nf = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t before = nf;
        out_frag_first[i] = nf;
        out_port[i] = (uint8_t)oracle_ip_fragment(base + pkt_off(off, stride, i), pkt_len(len, fixed_len, i),
                                                  mtu, honor_df, new_id ? (int)new_id[i] : -1, arena, &pos,
                                                  frag_off, frag_len, &nf, &out_first_len[i]);
        if (arena && frag_src)
            for (uint64_t k = before; k < nf; k++)
                frag_src[k] = (uint32_t)i;
    }
    totals[0] = nf;
    totals[1] = pos;
    return 0;
}

/* ---- batch drivers ------------------------------------------------------- */


static int run_one(int op, uint8_t *p, uint32_t l, int arg, uint16_t *sum)
{
    int r = 0;
    switch (op) {
    case ORACLE_OP_IN_CKSUM:
        *sum = oracle_in_cksum(p, (int)l);
        return 0;
    case ORACLE_OP_CHECK_IP:
        return oracle_check_ip_header(p, l, 0, arg, 0, 0, 0, 0);
    case ORACLE_OP_SET_IP:
        r = oracle_set_ip_checksum(p, l);
        *sum = r == 0 ? ld16(p + 10) : 0;
        return r;
    case ORACLE_OP_CHECK_UDP:
        return oracle_check_udp_header(p, l);
    case ORACLE_OP_SET_UDP:
        r = oracle_set_udp_checksum(p, l);
        *sum = r == 0 ? ld16(p + ((p[0] & 0xF) << 2) + 6) : 0;
        return r;
    case ORACLE_OP_CHECK_TCP:
        return oracle_check_tcp_header(p, l);
    case ORACLE_OP_SET_TCP:
        r = oracle_set_tcp_checksum(p, l, arg);
        *sum = r == 0 ? ld16(p + ((p[0] & 0xF) << 2) + 16) : 0;
        return r;
    case ORACLE_OP_CHECK_ICMP:
        return oracle_check_icmp_header(p, l);
    case ORACLE_OP_DEC_TTL:
        r = oracle_dec_ip_ttl(p, l, arg);
        *sum = r == 0 ? ld16(p + 10) : 0;
        return r;
    }
    return -1;
}

int oracle_batch(int op, uint8_t *base, const uint64_t *off, uint64_t stride,
                 const uint32_t *len, uint32_t fixed_len, uint64_t n, int arg,
                 uint8_t *out8, uint16_t *out16)
{
    for (uint64_t i = 0; i < n; i++) {
        uint16_t s = 0;
        int r = run_one(op, base + pkt_off(off, stride, i), pkt_len(len, fixed_len, i), arg, &s);
        if (r < 0)
            return -1;
        if (out8)
            out8[i] = (uint8_t)r;
        if (out16)
            out16[i] = s;
    }
    return 0;
}

int oracle_ip_out_batch(int op, uint8_t *base, const uint64_t *off, uint64_t stride,
                        const uint32_t *len, uint32_t fixed_len, uint64_t n,
                        const uint8_t *flags, uint32_t my_ip, const uint32_t *my_addrs, int n_my_addrs,
                        uint32_t ts, uint32_t mtu, uint8_t *out8, uint8_t *out_prob, uint16_t *out16)
{
    for (uint64_t i = 0; i < n; i++) {
        uint8_t *p = base + pkt_off(off, stride, i);
        uint32_t l = pkt_len(len, fixed_len, i);
        int f = flags ? flags[i] : 0, prob = 0, r;
        if (op == 0)
            r = oracle_ip_gw_options_element(p, l, my_ip, my_addrs, n_my_addrs, ts, &prob);
        else if (op == 1)
            r = oracle_fix_ip_src(p, l, f & 1, my_ip);
        else if (op == 2)
            r = oracle_ip_output_combo(p, l, l, f, my_ip, mtu, ts, &prob);
        else
            return -1;
        if (out8)
            out8[i] = (uint8_t)r;
        if (out_prob)
            out_prob[i] = (uint8_t)prob;
        if (out16)
            out16[i] = l >= 20 ? ld16(p + 10) : 0;
    }
    return 0;
}

/* ---- synthetic packets (bench.py / tests) ----------------
 * Byte 8w..8w+7 of packet idx is splitmix64 of counter (idx << 13 | w), then
 * the IPv4 + UDP/TCP header fields overwrite the front.  All checksum fields
 * are left 0; the Set elements fill them.  Identical to clk_gen_packets. */
uint64_t oracle_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t gen_word(uint64_t seed, uint64_t idx, uint64_t w)
{ return oracle_splitmix64(seed ^ ((idx << 13) | (w & 0x1FFF))); }

static inline void put_be16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

void oracle_gen_packet(uint8_t *pkt, uint32_t length, int proto, uint64_t seed, uint64_t idx)
{
    uint8_t hdr[40];
    for (uint32_t i = 0; i < length; i += 8) {
        uint64_t h = gen_word(seed, idx, i >> 3);
        if (i + 8 <= length) {
            memcpy(pkt + i, &h, 8);              /* little-endian host: bytes h >> 8k */
        } else {
            for (uint32_t k = 0; i + k < length; k++)
                pkt[i + k] = (uint8_t)(h >> (8 * k));
        }
    }
    /* header words use counters past the payload's (w = 0x1FFF, 0x1FFE) */
    uint64_t a = gen_word(seed, idx, 0x1FFF), b = gen_word(seed, idx, 0x1FFE);
    memset(hdr, 0, sizeof hdr);
    hdr[0] = 0x45;
    put_be16(hdr + 2, length);
    put_be16(hdr + 4, (uint32_t)(idx & 0xFFFF));
    hdr[8] = 64;
    hdr[9] = (uint8_t)proto;
    /* src 10.x.y.z, dst 192.168.x.y -- stored big-endian like s_addr */
    uint32_t src = 0x0A000000u | (uint32_t)(a & 0xFFFFFF);
    uint32_t dst = 0xC0A80000u | (uint32_t)((a >> 24) & 0xFFFF);
    put_be16(hdr + 12, src >> 16); put_be16(hdr + 14, src);
    put_be16(hdr + 16, dst >> 16); put_be16(hdr + 18, dst);
    uint32_t hlen = 20;
    if (proto == 17) {
        put_be16(hdr + 20, (uint32_t)(a >> 40));
        put_be16(hdr + 22, (uint32_t)(a >> 56) | 0x400);
        put_be16(hdr + 24, length >= 20 ? length - 20 : 0);
        hlen = 28;
    } else if (proto == 6) {
        put_be16(hdr + 20, (uint32_t)(a >> 40));
        put_be16(hdr + 22, 80);
        memcpy(hdr + 24, &b, 8);                 /* seq, ack */
        hdr[32] = 0x50;                          /* th_off = 5 */
        hdr[33] = 0x10;                          /* ACK */
        put_be16(hdr + 34, (uint32_t)(a >> 48)); /* window */
        hlen = 40;
    }
    for (uint32_t i = 0; i < hlen && i < length; i++)
        pkt[i] = hdr[i];
}

void oracle_gen_batch(uint8_t *base, const uint64_t *off, uint64_t stride,
                      const uint32_t *len, uint32_t fixed_len, uint64_t n,
                      int proto, uint64_t seed, uint64_t first_idx)
{
    for (uint64_t i = 0; i < n; i++)
        oracle_gen_packet(base + pkt_off(off, stride, i), pkt_len(len, fixed_len, i),
                          proto, seed, first_idx + i);
}

/* ---- CPU baseline --------------------------------------------------------- */

struct bench_arg {
    int op, reps, arg;
    uint8_t *base;
    uint64_t stride, lo, hi;
    uint32_t fixed_len;
    volatile uint64_t sink;
};

/* Run fn over args[0..n-1] (elements of `size` bytes): args[1..] on threads
 * of their own, args[0] on the caller's.  The threads wait at a gate until
 * every one of them was created, so a failed pthread_create leaves no thread
 * running (or stuck at a barrier of the job) and nothing joined that was not
 * started: the job is not run and -1 is returned. */
struct gate {
    pthread_mutex_t m;
    pthread_cond_t c;
    int state;                       /* 0 wait, 1 go, -1 abort */
};
struct gated {
    struct gate *g;
    void *(*fn)(void *);
    void *arg;
};
static void *gated_entry(void *p)
{
    struct gated *x = p;
    pthread_mutex_lock(&x->g->m);
    while (x->g->state == 0)
        pthread_cond_wait(&x->g->c, &x->g->m);
    const int go = x->g->state > 0;
    pthread_mutex_unlock(&x->g->m);
    return go ? x->fn(x->arg) : 0;
}
static int run_threads(int n, void *(*fn)(void *), void *args, size_t size)
{
    struct gate g = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0};
    pthread_t *th = calloc((size_t)n, sizeof *th);
    struct gated *x = calloc((size_t)n, sizeof *x);
    if (!th || !x) {
        free(th);
        free(x);
        return -1;
    }
    int started = 1;
    for (int t = 1; t < n; t++, started++) {
        x[t] = (struct gated){&g, fn, (char *)args + (size_t)t * size};
        if (pthread_create(&th[t], 0, gated_entry, &x[t]) != 0)
            break;
    }
    pthread_mutex_lock(&g.m);
    g.state = started == n ? 1 : -1;
    pthread_cond_broadcast(&g.c);
    pthread_mutex_unlock(&g.m);
    if (started == n)
        fn(args);
    for (int t = 1; t < started; t++)
        pthread_join(th[t], 0);
    free(th);
    free(x);
    return started == n ? 0 : -1;
}

static void *bench_thread(void *vp)
{
    struct bench_arg *a = (struct bench_arg *)vp;
    uint64_t acc = 0;
    for (int r = 0; r < a->reps; r++)
        for (uint64_t i = a->lo; i < a->hi; i++) {
            uint16_t s = 0;
            acc += (uint64_t)run_one(a->op, a->base + i * a->stride, a->fixed_len, a->arg, &s) + s;
        }
    a->sink = acc;
    return 0;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double oracle_bench(int op, uint8_t *base, uint64_t stride, uint32_t fixed_len,
                    uint64_t n, int reps, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    struct bench_arg *args = calloc((size_t)nthreads, sizeof *args);
    for (int t = 0; t < nthreads; t++) {
        args[t].op = op; args[t].reps = reps; args[t].arg = 1;
        args[t].base = base; args[t].stride = stride; args[t].fixed_len = fixed_len;
        args[t].lo = n * (uint64_t)t / (uint64_t)nthreads;
        args[t].hi = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
    }
    double t0 = now_s();
    const int rc = run_threads(nthreads, bench_thread, args, sizeof *args);
    double dt = rc ? -1.0 : now_s() - t0;
    free(args);
    return dt;
}

/* ---- CPU baseline per BASELINE.md §2 ---------------------------------------
 * One thread per entry of cpus[] (the caller passes one logical CPU of each
 * physical core), pinned before it allocates and generates its own shard, so
 * every shard is first-touched on the thread's NUMA node.  Each shard holds
 * bytes_per_thread of packets -- sized by the caller well above the last-level
 * cache, so the timed passes stream from DRAM -- generated with the same
 * splitmix64 packets as the GPU (oracle_gen_packet, global index
 * t * npkt + i), checksums set, then: one warm-up pass, and `reps` timed
 * passes, each between two barriers (all threads start together; a pass ends
 * when the slowest shard is done).  imix = 1: packet sizes 64/576/1500 by
 * the same hash and 7:4:1 odds as bench.py's C4 layout, packed at 64-byte
 * aligned offsets; otherwise fixed_len-byte packets in stride-byte slots. */
struct cb_thread {
    const struct oracle_cb_cfg *cfg;
    int t, cpu;
    pthread_barrier_t *bar;
    double *rep_s;               /* thread 0 writes the pass times */
    uint64_t packets, bytes, ok, gen_ns;
    int pinned, err;
};

static uint64_t imix_len(uint64_t seed, uint64_t i)
{
    /* bench.py imix_layout: splitmix64 finalizer of i*golden + seed, mod 12 */
    uint64_t x = i * 0x9E3779B97F4A7C15ull + seed;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    const uint64_t r = x % 12;
    return r < 7 ? 64 : (r < 11 ? 576 : 1500);
}

static void *cb_run(void *vp)
{
    struct cb_thread *a = (struct cb_thread *)vp;
    const struct oracle_cb_cfg *c = a->cfg;
    if (a->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(a->cpu, &set);
        a->pinned = pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0;
    }
    /* shard layout: fixed slots, or IMIX packed at 64 B-aligned offsets */
    uint64_t n, bytes;
    uint64_t *off = 0;
    uint32_t *len = 0;
    if (c->imix) {
        /* packets until the shard bytes are used; mean slot ~ 384 B */
        uint64_t cap = c->bytes_per_thread / 64 + 1;
        off = malloc(cap * sizeof *off);
        len = malloc(cap * sizeof *len);
        if (!off || !len) { a->err = 1; free(off); free(len); return 0; }
        uint64_t pos = 0, k = 0;
        const uint64_t first = (uint64_t)a->t * cap;
        for (; k < cap; k++) {
            const uint64_t L = imix_len(c->seed, first + k);
            const uint64_t slot = (L + 63) & ~63ull;
            if (pos + slot > c->bytes_per_thread)
                break;
            off[k] = pos;
            len[k] = (uint32_t)L;
            pos += slot;
        }
        n = k;
        bytes = pos;
    } else {
        n = c->bytes_per_thread / c->stride;
        bytes = n * c->stride;
    }
    uint8_t *arena = 0;
    if (posix_memalign((void **)&arena, 4096, bytes ? bytes : 4096)) {
        a->err = 1;
        free(off); free(len);
        return 0;
    }
    struct timespec g0, g1;
    clock_gettime(CLOCK_MONOTONIC, &g0);
    /* first touch + generation on this thread's node */
    const uint64_t first_idx = (uint64_t)a->t * (n + 1);
    oracle_gen_batch(arena, off, c->stride, len, c->fixed_len, n, c->proto, c->seed, first_idx);
    uint16_t s;
    for (uint64_t i = 0; i < n; i++) {
        uint8_t *p = arena + (off ? off[i] : i * c->stride);
        const uint32_t l = len ? len[i] : c->fixed_len;
        run_one(ORACLE_OP_SET_IP, p, l, 1, &s);
        if (l >= 28)
            run_one(c->proto == 6 ? ORACLE_OP_SET_TCP : ORACLE_OP_SET_UDP, p, l, 0, &s);
    }
    clock_gettime(CLOCK_MONOTONIC, &g1);
    a->gen_ns = (uint64_t)((g1.tv_sec - g0.tv_sec) * 1000000000ll + (g1.tv_nsec - g0.tv_nsec));
    a->packets = n;
    uint64_t sum_len = 0;
    for (uint64_t i = 0; i < n; i++)
        sum_len += len ? len[i] : c->fixed_len;
    a->bytes = sum_len;
    uint64_t ok = 0;
    for (int r = -1; r < c->reps; r++) {          /* r = -1: warm-up */
        pthread_barrier_wait(a->bar);
        struct timespec t0, t1;
        if (a->t == 0)
            clock_gettime(CLOCK_MONOTONIC, &t0);
        ok = 0;
        for (uint64_t i = 0; i < n; i++) {
            uint8_t *p = arena + (off ? off[i] : i * c->stride);
            ok += run_one(c->op, p, len ? len[i] : c->fixed_len, c->arg, &s) == 0;
        }
        pthread_barrier_wait(a->bar);
        if (a->t == 0 && r >= 0) {
            clock_gettime(CLOCK_MONOTONIC, &t1);
            a->rep_s[r] = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        }
    }
    a->ok = ok;
    free(arena);
    free(off);
    free(len);
    return 0;
}

static int cmp_double(const void *x, const void *y)
{
    const double a = *(const double *)x, b = *(const double *)y;
    return a < b ? -1 : a > b;
}

int oracle_cpu_baseline(const struct oracle_cb_cfg *cfg, const int *cpus, int nthreads,
                        struct oracle_cb_result *res)
{
    if (!cfg || !res || nthreads < 1 || cfg->reps < 1 || cfg->reps > 64 ||
        (!cfg->imix && (cfg->stride == 0 || cfg->fixed_len > cfg->stride)))
        return -1;
    memset(res, 0, sizeof *res);
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, 0, (unsigned)nthreads);
    struct cb_thread *a = calloc((size_t)nthreads, sizeof *a);
    double rep_s[64];
    for (int t = 0; t < nthreads; t++) {
        a[t].cfg = cfg;
        a[t].t = t;
        a[t].cpu = cpus ? cpus[t] : -1;
        a[t].bar = &bar;
        a[t].rep_s = rep_s;
    }
    int err = run_threads(nthreads, cb_run, a, sizeof *a) ? 1 : 0;
    pthread_barrier_destroy(&bar);
    for (int t = 0; t < nthreads; t++) {
        err |= a[t].err;
        res->packets += a[t].packets;
        res->bytes += a[t].bytes;
        res->ok += a[t].ok;
        res->pinned += a[t].pinned;
        if ((double)a[t].gen_ns * 1e-9 > res->gen_s)
            res->gen_s = (double)a[t].gen_ns * 1e-9;
    }
    qsort(rep_s, (size_t)cfg->reps, sizeof rep_s[0], cmp_double);
    res->median_s = rep_s[cfg->reps / 2];
    res->min_s = rep_s[0];
    res->max_s = rep_s[cfg->reps - 1];
    free(a);
    return err ? -2 : 0;
}

/* ---- bench.py self-verification -------------------------
 * The oracle's digest of exactly the work one rank of bench.py did, computed
 * packet by packet from the global packet index, so a full-size GPU result
 * is checked without holding the batch in host memory.  Per packet g in
 * [first_idx, first_idx + n): generate it (oracle_gen_packet; C4: length
 * imix_len(seed, g)), SetIPChecksum, then the L4 Set of `proto` (the bench's
 * untimed preparation; their results are the Set elements' results, since a
 * Set zeroes its field before summing).  Check legs: the packet with the
 * bench's corruption applied (corrupt_kernel's pick and bit), then the
 * element.  DecIPTTL / IPOutputCombo legs: TTL 255 + SetIPChecksum, then
 * ttl_runs passes of the element; the last pass's code.
 * Digest per leg: ok (code 0), packets, sum16 = sum of checksums, xor16,
 * wsum16 = sum of checksum * w(g), wcode = sum of code * w(g), with
 * w(g) = (g * 40503) mod 2^16 (position-weighted: a permutation of results
 * changes it).  Threads take contiguous index ranges. */
/* corrupt_kernel (click_amd/csrc/cksum_kernels.hh) on one packet of global
 * index g: picked when the low rate_log2 bits of h are zero; flips bit
 * (h >> 8) & 7 of byte lo + (h >> 20) % (hi' - lo).  Flipping twice
 * restores it.  Returns 1 when a bit was flipped. */
static int corrupt_one(uint8_t *p, uint32_t len, uint64_t seed, uint64_t g, uint32_t rate_log2,
                       uint32_t lo_arg, uint32_t hi_arg)
{
    const uint64_t h = oracle_splitmix64(seed ^ (g * 0xD1B54A32D192ED03ull));
    const uint64_t mask = rate_log2 >= 64 ? ~0ull : ((1ull << rate_log2) - 1);
    if ((h & mask) != 0)
        return 0;
    const uint32_t lo = lo_arg != ~0u ? lo_arg : (len > 40 ? 40 : (len > 20 ? 20 : 0));
    const uint32_t hi = hi_arg && hi_arg < len ? hi_arg : len;
    if (hi <= lo)
        return 0;
    const uint32_t pos = lo + (uint32_t)((h >> 20) % (uint64_t)(hi - lo));
    p[pos] ^= (uint8_t)(1u << ((h >> 8) & 7));
    return 1;
}

struct dg_thread {
    const struct oracle_digest_cfg *cfg;
    uint64_t lo, hi;
    struct oracle_digest_leg leg[ORACLE_DG_NLEGS];
    int err;
};

static void dg_add(struct oracle_digest_leg *l, uint64_t g, int code, uint16_t sum)
{
    const uint64_t w = (g * 40503u) & 0xFFFF;
    l->packets++;
    l->ok += code == 0;
    l->sum16 += sum;
    l->xor16 ^= sum;
    l->wsum16 += (uint64_t)sum * w;
    l->wcode += (uint64_t)(uint8_t)code * w;
}

static void *dg_run(void *vp)
{
    struct dg_thread *a = (struct dg_thread *)vp;
    const struct oracle_digest_cfg *c = a->cfg;
    uint8_t *buf = 0;
    if (posix_memalign((void **)&buf, 64, 65536 + 64)) {
        a->err = 1;
        return 0;
    }
    const int set_l4 = c->proto == 6 ? ORACLE_OP_SET_TCP : ORACLE_OP_SET_UDP;
    const int check_l4 = c->proto == 6 ? ORACLE_OP_CHECK_TCP : ORACLE_OP_CHECK_UDP;
    for (uint64_t g = a->lo; g < a->hi; g++) {
        const uint32_t L = c->imix ? (uint32_t)imix_len(c->seed, g) : c->fixed_len;
        if (L > 65536) { a->err = 1; break; }
        oracle_gen_packet(buf, L, c->proto, c->seed, g);
        uint16_t s_ip = 0, s_l4 = 0;
        const int r_ip = run_one(ORACLE_OP_SET_IP, buf, L, 0, &s_ip);
        const int r_l4 = run_one(set_l4, buf, L, 0, &s_l4);
        if (c->legs & (1u << ORACLE_DG_SET_IP))
            dg_add(&a->leg[ORACLE_DG_SET_IP], g, r_ip, s_ip);
        if (c->legs & (1u << ORACLE_DG_SET_L4))
            dg_add(&a->leg[ORACLE_DG_SET_L4], g, r_l4, s_l4);
        uint16_t z;
        if (c->legs & (1u << ORACLE_DG_CHECK_L4)) {
            const int f = corrupt_one(buf, L, c->corrupt_seed, g, c->corrupt_log2, ~0u, 0);
            dg_add(&a->leg[ORACLE_DG_CHECK_L4], g, run_one(check_l4, buf, L, 1, &z), 0);
            if (f)
                corrupt_one(buf, L, c->corrupt_seed, g, c->corrupt_log2, ~0u, 0);
        }
        if (c->legs & (1u << ORACLE_DG_CHECK_IP)) {
            const int f = corrupt_one(buf, L, c->corrupt_seed, g, c->corrupt_log2, c->ip_lo, c->ip_hi);
            dg_add(&a->leg[ORACLE_DG_CHECK_IP], g, run_one(ORACLE_OP_CHECK_IP, buf, L, 1, &z), 0);
            if (f)
                corrupt_one(buf, L, c->corrupt_seed, g, c->corrupt_log2, c->ip_lo, c->ip_hi);
        }
        if (c->legs & (1u << ORACLE_DG_DEC_TTL)) {
            buf[8] = 255;
            run_one(ORACLE_OP_SET_IP, buf, L, 0, &z);
            int r = 0;
            for (int k = 0; k < c->ttl_runs; k++)
                r = run_one(ORACLE_OP_DEC_TTL, buf, L, 1, &z);
            dg_add(&a->leg[ORACLE_DG_DEC_TTL], g, r, 0);
        }
        if (c->legs & (1u << ORACLE_DG_OUT_COMBO)) {
            buf[8] = 255;
            run_one(ORACLE_OP_SET_IP, buf, L, 0, &z);
            int r = 0, prob = 0;
            for (int k = 0; k < c->ttl_runs; k++)
                r = oracle_ip_output_combo(buf, L, L, 0, c->my_ip, c->mtu, 0, &prob);
            dg_add(&a->leg[ORACLE_DG_OUT_COMBO], g, r, 0);
        }
    }
    free(buf);
    return 0;
}

int oracle_digest(const struct oracle_digest_cfg *cfg, const int *cpus, int nthreads,
                  struct oracle_digest_leg *out)
{
    if (!cfg || !out || nthreads < 1 || (!cfg->imix && cfg->fixed_len > 65536))
        return -1;
    memset(out, 0, ORACLE_DG_NLEGS * sizeof *out);
    struct dg_thread *a = calloc((size_t)nthreads, sizeof *a);
    if (!a) {
        free(a);
        return -2;
    }
    for (int t = 0; t < nthreads; t++) {
        a[t].cfg = cfg;
        a[t].lo = cfg->first_idx + cfg->n * (uint64_t)t / (uint64_t)nthreads;
        a[t].hi = cfg->first_idx + cfg->n * (uint64_t)(t + 1) / (uint64_t)nthreads;
    }
    int err = run_threads(nthreads, dg_run, a, sizeof *a) ? 1 : 0;
    (void)cpus;
    for (int t = 0; t < nthreads; t++) {
        err |= a[t].err;
        for (int l = 0; l < ORACLE_DG_NLEGS; l++) {
            out[l].ok += a[t].leg[l].ok;
            out[l].packets += a[t].leg[l].packets;
            out[l].sum16 += a[t].leg[l].sum16;
            out[l].xor16 ^= a[t].leg[l].xor16;
            out[l].wsum16 += a[t].leg[l].wsum16;
            out[l].wcode += a[t].leg[l].wcode;
        }
    }
    free(a);
    return err ? -3 : 0;
}
