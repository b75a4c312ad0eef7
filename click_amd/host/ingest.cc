// ingest.cc -- pcap file ingest into a struct-of-arrays batch
// (include/click_amd_ingest.h).  Host code; restates FromDump's file and
// record handling (elements/userlevel/fromdump.cc) and FORCE_IP
// (elements/userlevel/fakepcap.cc:121-330) without Click's Packet.
#include "click_amd_ingest.h"

#include <cerrno>
#include <cstdio>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <cstring>
#include <string>
#include <vector>

extern "C" int clk_ctx_set_error_internal(clk_ctx *ctx, const char *msg);

namespace {

// fakepcap.hh:7-31
constexpr uint32_t PCAP_MAGIC = 0xA1B2C3D4u, PCAP_MAGIC_NANO = 0xA1B23C4Du, MODIFIED_PCAP_MAGIC = 0xA1B2CD34u;
enum {
    DLT_NULL = 0, DLT_EN10MB = 1, DLT_PPP = 9, DLT_FDDI = 10, DLT_PPP_HDLC = 50, DLT_ATM_RFC1483 = 100,
    DLT_RAW = 101, DLT_C_HDLC = 104, DLT_IEEE802_11 = 105, DLT_LINUX_SLL = 113, DLT_PRISM_HEADER = 119,
    DLT_SUNATM = 123, DLT_IEEE802_11_RADIO = 127, DLT_HOST_RAW = 12
};

uint32_t swap32(uint32_t v) { return __builtin_bswap32(v); }
uint16_t swap16(uint16_t v) { return __builtin_bswap16(v); }
uint32_t net16(const uint8_t *p) { return (uint32_t)p[0] << 8 | p[1]; }   // unaligned_net_short, fakepcap.cc:107-112
bool ip_ethertype(const uint8_t *p) { return net16(p) == 0x0800 || net16(p) == 0x86DD; }   // 116

int fail(const std::string &msg)
{
    clk_ctx_set_error_internal(nullptr, msg.c_str());
    return CLK_EINVAL;
}

// fakepcap.cc:83-92
bool dlt_force_ipable(int dlt)
{
    return dlt == DLT_RAW || dlt == DLT_HOST_RAW || dlt == DLT_EN10MB || dlt == DLT_SUNATM || dlt == DLT_FDDI ||
           dlt == DLT_ATM_RFC1483 || dlt == DLT_LINUX_SLL || dlt == DLT_C_HDLC || dlt == DLT_IEEE802_11 ||
           dlt == DLT_PRISM_HEADER || dlt == DLT_PPP_HDLC || dlt == DLT_PPP || dlt == DLT_NULL ||
           dlt == DLT_IEEE802_11_RADIO;
}

// fakepcap.cc:95-101
int canonical_dlt(int dlt) { return dlt == DLT_HOST_RAW ? DLT_RAW : dlt; }

}  // namespace

// fakepcap.cc:121-330.  The label structure follows the reference's
// switch, whose cases jump into one another (FDDI and 802.11 into RFC 1483,
// RFC 1483 SNAP into Ethernet or FDDI, PPP-HDLC into C-HDLC).  x86-64 has
// indifferent alignment, so the reference's realignment (304-316) is off.
extern "C" int32_t clk_pcap_force_ip(const uint8_t *p, uint32_t len, int32_t dlt)
{
    const uint8_t *data = p, *end = p + len;
    const uint8_t *iph = nullptr;
    switch (dlt) {
    case DLT_RAW:
    case DLT_HOST_RAW:
        iph = data;
        break;
    ethernet:
    case DLT_EN10MB:
        if (data + 14 <= end) {
            if (ip_ethertype(data + 12))
                iph = data + 14;
            else if (net16(data + 12) == 0x8100 && data + 18 <= end) {   // one 802.1Q tag
                if (ip_ethertype(data + 16))
                    iph = data + 18;
            }
        }
        break;
    fddi:
    case DLT_FDDI:
        if (data + 21 > end || (data[0] & 0xF0) != 0x50)      // sizeof(click_fddi_snap); FDDI_FC_LLC_ASYNC
            break;
        data += 13;                                          // sizeof(click_fddi)
        goto rfc1483;
    case DLT_SUNATM:
        data += 4;
        goto rfc1483;
    rfc1483:
    case DLT_ATM_RFC1483:
        if (data + 8 <= end && memcmp(data, "\xAA\xAA\x03\x00\x00\x00", 6) == 0 && ip_ethertype(data + 6))
            iph = data + 8;
        else if (data + 4 <= end && data[0] == 0x06 && data[1] == 0x06)     // LLC_IP_LSAP
            iph = data + 4;
        else if (data + 8 <= end && data[0] == 0xAA && data[1] == 0xAA) {   // LLC_SNAP_LSAP
            const uint32_t org = (uint32_t)data[3] << 16 | (uint32_t)data[4] << 8 | data[5];
            if (org == 0x000000 || org == 0x0000f8) {        // OUI_ENCAP_ETHER, OUI_CISCO_90
                data = data + 6 - 12;
                goto ethernet;
            } else if (org == 0x0080c2) {                    // OUI_RFC2684
                const uint32_t et = net16(data + 6);
                if (et == 0x0001 || et == 0x0007) {
                    data += 8;
                    goto ethernet;
                } else if (et == 0x0004 || et == 0x000a) {
                    data += 9;
                    goto fddi;
                }
            }
        }
        break;
    case DLT_LINUX_SLL:                                      // 16-byte cooked header
        if (data + 16 <= end && ip_ethertype(data + 14))
            iph = data + 16;
        break;
    c_hdlc:
    case DLT_C_HDLC:
        if (data + 4 <= end && ip_ethertype(data + 2))
            iph = data + 4;
        break;
    case DLT_PPP_HDLC:
        if (data + 4 > end)
            ;
        else if (data[0] == 0xff) {                          // PPP_ADDRESS
            if (data[2] == 0 && (data[3] == 0x21 || data[3] == 0x57))
                iph = data + 4;
        } else if (data[0] == 0x0F || data[0] == 0x8F)
            goto c_hdlc;
        break;
    case DLT_PPP:
        if (data + 2 <= end && data[0] == 0xff && data[1] == 0x03)
            data += 2;
        if (data + 2 > end)
            ;
        else if (data[0] == 0x21 || data[0] == 0x57)
            iph = data + 1;
        else if (data[0] == 0 && (data[1] == 0x21 || data[1] == 0x57))
            iph = data + 2;
        break;
    case DLT_PRISM_HEADER:
        data += 144;
        goto ieee802_11;
    ieee802_11:
    case DLT_IEEE802_11:
        if (data + 24 <= end && (data[0] & 0x0c) == 0x08) {  // WIFI_FC0_TYPE_DATA
            data += (data[1] & 0x03) == 0x03 ? 30 : 24;
            goto rfc1483;
        }
        break;
    case DLT_IEEE802_11_RADIO: {
        uint32_t l;
        if (data + 4 <= end && (l = (uint32_t)data[3] << 8 | data[2]) >= 8) {
            data += l;
            goto ieee802_11;
        }
        break;
    }
    case DLT_NULL: {
        if (data + 4 > end)
            break;
        int family = data[0] | (data[1] << 8);
        if (family == 0)
            family = (data[2] << 8) | data[3];
        if (family == 2 || family == 24 || family == 28 || family == 30)
            iph = data + 4;
        break;
    }
    default:
        break;
    }
    // 318-330: an IPv4 header with ip_hl >= 5 inside the packet, or IPv6.
    // A jump past `end` leaves iph beyond the data: no byte of it is read.
    if (!iph || iph < p || iph >= end)
        return -1;
    const uint32_t v = iph[0] >> 4;
    if (v == 4) {
        const uint32_t hl = iph[0] & 0xF;
        if (hl >= 5 && iph + (hl << 2) <= end)
            return (int32_t)(iph - p);
    } else if (v == 6) {
        if (iph + 40 <= end)
            return (int32_t)(iph - p);
    }
    return -1;
}

extern "C" int clk_pcap_read(const char *path, int force_ip, uint8_t *arena, uint64_t arena_bytes, uint64_t *off,
                             uint32_t *caplen_out, uint32_t *wire_len, uint64_t *ts_ns, int32_t *nh,
                             uint64_t max_records, clk_pcap_info *info)
{
    if (!path || !info)
        return fail("clk_pcap_read: null path or info");
    if (arena && max_records && (!off || !caplen_out || !nh))
        return fail("clk_pcap_read: off, caplen and nh are required with an arena");
    memset(info, 0, sizeof *info);
    // the whole file, mapped (regular files) or read (pipes, "-" style sources)
    struct Source {
        const uint8_t *p = nullptr;
        size_t n = 0;
        void *map = nullptr;
        std::vector<uint8_t> buf;
        ~Source() { if (map) munmap(map, n); }
    } src;
    {
        const int fd = open(path, O_RDONLY);
        if (fd < 0)
            return fail(std::string(path) + ": " + strerror(errno));
        struct stat sb;
        if (fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode) && sb.st_size > 0) {
            void *m = mmap(nullptr, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m != MAP_FAILED) {
                src.map = m;
                src.n = (size_t)sb.st_size;
                src.p = (const uint8_t *)m;
                madvise(m, src.n, MADV_SEQUENTIAL);
            }
        }
        if (!src.map) {
            uint8_t tmp[1 << 16];
            ssize_t r;
            while ((r = read(fd, tmp, sizeof tmp)) > 0)
                src.buf.insert(src.buf.end(), tmp, tmp + r);
            src.p = src.buf.data();
            src.n = src.buf.size();
        }
        close(fd);
    }
    const uint8_t *const file = src.p;
    const size_t fsize = src.n;
    const std::string fn(path);
    // fromdump.cc:226-250: file header, byte order, magic, version
    if (fsize < 24)
        return fail(fn + ": not a tcpdump file (too short)");
    uint32_t magic, linktype;
    uint16_t vmaj, vmin;
    memcpy(&magic, file, 4);
    memcpy(&vmaj, file + 4, 2);
    memcpy(&vmin, file + 6, 2);
    memcpy(&linktype, file + 20, 4);
    bool swapped = false;
    if (magic != PCAP_MAGIC && magic != PCAP_MAGIC_NANO && magic != MODIFIED_PCAP_MAGIC) {
        magic = swap32(magic);
        vmaj = swap16(vmaj);
        vmin = swap16(vmin);
        linktype = swap32(linktype);
        swapped = true;
    }
    if (magic != PCAP_MAGIC && magic != PCAP_MAGIC_NANO && magic != MODIFIED_PCAP_MAGIC)
        return fail(fn + ": not a tcpdump file (bad magic number)");
    const uint32_t extra = magic == MODIFIED_PCAP_MAGIC ? 8u : 0u;   // sizeof(fake_modified_pcap_pkthdr) - 16
    const bool nano = magic == PCAP_MAGIC_NANO;
    if (vmaj != 2)                                                    // FAKE_PCAP_VERSION_MAJOR
        return fail(fn + ": unknown major version " + std::to_string(vmaj));
    const int dlt = canonical_dlt((int)linktype);
    if (force_ip) {                                                   // 252-257
        if (!dlt_force_ipable(dlt))
            return fail(fn + ": unknown linktype " + std::to_string(dlt) + "; can't force IP packets");
    } else if (dlt == DLT_RAW)
        force_ip = 1;
    info->linktype = dlt;
    info->nanosecond = nano;
    info->swapped = swapped;
    info->force_ip = force_ip != 0;
    // fromdump.cc:328-413: records
    uint64_t pos = 24, k = 0, need = 0;
    int rc = CLK_SUCCESS;
    while (pos + 16 <= fsize) {
        uint32_t h[4];
        memcpy(h, file + pos, 16);
        if (swapped)
            for (auto &x : h)
                x = swap32(x);
        uint32_t len, cap;
        if (vmin > 3 || (vmin == 3 && h[2] <= h[3])) {               // 348-355
            len = h[3];
            cap = h[2];
        } else {
            len = h[2];
            cap = h[3];
        }
        uint32_t skip = 0;
        if ((int32_t)cap > 65535 || (int32_t)cap < 0) {              // 362-364 (int caplen)
            clk_ctx_set_error_internal(nullptr, (fn + ": bad packet header; giving up").c_str());
            rc = 1;
            break;
        } else if ((int32_t)cap > (int32_t)len) {                    // 365-368
            skip = cap - len;
            cap = len;
        }
        pos += 16 + extra;                                            // 371
        if (pos + cap > fsize)                                   // short final record: get_packet fails
            break;
        const uint64_t at = (need + 15) & ~15ull;
        if (arena && k < max_records) {
            if (at + cap > arena_bytes)
                return fail("clk_pcap_read: arena too small (size it with arena = NULL)");
            memcpy(arena + at, file + pos, cap);
            off[k] = at;
            caplen_out[k] = cap;
            if (wire_len)
                wire_len[k] = len;
            if (ts_ns) {
                const int64_t sec = (int32_t)h[0], sub = (int32_t)h[1];
                ts_ns[k] = (uint64_t)(sec * 1000000000 + (nano ? sub : sub * 1000));
            }
            nh[k] = force_ip ? clk_pcap_force_ip(arena + at, cap, dlt) : -1;
            if (nh[k] >= 0)
                info->ip_records++;
        } else if (!arena && force_ip && clk_pcap_force_ip(file + pos, cap, dlt) >= 0) {
            info->ip_records++;
        }
        need = at + cap;
        pos += cap + skip;                                            // 408
        k++;
    }
    info->records = k;
    info->arena_bytes = (need + 15) & ~15ull;
    return rc;
}
