"""A second, independent restatement of the checksum path in pure Python.

Test infrastructure: used only to cross-check the C oracle on small inputs
(two restatements written separately must agree before either is trusted
as the checker for the HIP kernels).  Follows the same reference lines as
oracle/cksum_oracle.c, but is written from RFC 1071 / RFC 791 terms:
big-endian one's-complement arithmetic is NOT used here either, because the
reference's u32-wrap behaviour differs from it past 131,074 bytes.
"""
import struct

M32 = 0xFFFFFFFF


def in_cksum(b, length=None):
    """lib/in_cksum.c:20-51 on bytes `b` (length may be negative/int)."""
    n = len(b) if length is None else length
    s = 0
    i = 0
    while n > 1:
        s = (s + (b[i] | (b[i + 1] << 8))) & M32
        i += 2
        n -= 2
    if n == 1:
        s = (s + b[i]) & M32
    s = (s & 0xFFFF) + (s >> 16)
    s += s >> 16
    return (~s) & 0xFFFF


def bswap16(v):
    v &= 0xFFFF
    return ((v >> 8) | (v << 8)) & 0xFFFF


def pseudohdr_raw(csum, src, dst, proto, plen):
    """lib/in_cksum.c:74-78."""
    c = (~csum) & 0xFFFF
    c += (src & 0xFFFF) + (src >> 16)
    c += (dst & 0xFFFF) + (dst >> 16)
    c += bswap16(plen) + bswap16(proto)
    c = (c & 0xFFFF) + (c >> 16)
    return (~(c + (c >> 16))) & 0xFFFF


def u32le(b, o):
    return struct.unpack_from("<I", b, o)[0]


def final_dst(iph):
    """lib/in_cksum.c:86-110 option walk."""
    hl = (iph[0] & 0xF) * 4
    o = 20
    while o < hl:
        t = iph[o]
        if t == 1:
            o += 1
            continue
        if t == 0:
            break
        if o + 1 >= hl or iph[o + 1] < 2 or o + iph[o + 1] > hl:
            break
        ln = iph[o + 1]
        if t in (137, 131) and ln >= 7:
            return u32le(iph, o + ln - 4)
        o += ln
    return u32le(iph, 16)


def pseudohdr(csum, iph, plen):
    """include/clicknet/ip.h:152-160."""
    dst = u32le(iph, 16) if (iph[0] & 0xF) == 5 else final_dst(iph)
    return pseudohdr_raw(csum, u32le(iph, 12), dst, iph[9], plen)


def be16(b, o):
    return (b[o] << 8) | b[o + 1]


def check_ip(data, length, offset=0, checksum=True, badsrc=(), gooddst=()):
    ip = data[offset:]
    plen = (length - offset) & M32
    if plen >= 0x80000000 or plen < 20:
        return 1
    if ip[0] >> 4 != 4:
        return 2
    hl = (ip[0] & 0xF) * 4
    if hl < 20:
        return 3
    ln = be16(ip, 2)
    if ln > plen or ln < hl:
        return 4
    if checksum and in_cksum(ip[:hl]) != 0:
        return 5
    if u32le(ip, 12) in badsrc and u32le(ip, 16) not in gooddst:
        return 6
    return 0


def set_ip(b, plen):
    """Returns (status, new bytes)."""
    b = bytearray(b)
    if plen >= 20:
        hl = (b[0] & 0xF) * 4
        if 20 <= hl <= plen:
            b[10:12] = b"\0\0"
            struct.pack_into("<H", b, 10, in_cksum(b[:hl]))
            return 0, bytes(b)
    return 2, bytes(b)


def check_udp(b, caplen):
    if caplen < 20:
        return 2
    if b[9] != 17:
        return 1
    hl = (b[0] & 0xF) * 4
    if caplen < hl + 8:
        return 2
    ln = be16(b, hl + 4)
    if ln < 8 or caplen < ln + hl:
        return 2
    if b[hl + 6] | b[hl + 7]:
        if pseudohdr(in_cksum(b[hl:hl + ln]), b, ln) != 0:
            return 3
    return 0


def set_udp(b, caplen):
    b = bytearray(b)
    if caplen < 20:
        return 1, bytes(b)
    hl = (b[0] & 0xF) * 4
    tlen = caplen - hl
    frag = be16(b, 6) & 0x3FFF
    if frag or tlen < 8:
        return 1, bytes(b)
    ln = be16(b, hl + 4)
    if tlen < ln:
        return 1, bytes(b)
    b[hl + 6:hl + 8] = b"\0\0"
    struct.pack_into("<H", b, hl + 6, pseudohdr(in_cksum(b[hl:hl + ln]), b, ln))
    return 0, bytes(b)


def _as_int(u):
    u &= M32
    return u - (1 << 32) if u & 0x80000000 else u


def check_tcp(b, caplen):
    if caplen < 20:
        return 2
    if b[9] != 6:
        return 1
    hl = (b[0] & 0xF) * 4
    ln = (be16(b, 2) - hl) & M32
    if caplen < hl + 13:
        return 2
    thl = (b[hl + 12] >> 4) * 4
    if thl < 20 or ln < thl or caplen < ((ln + hl) & M32):
        return 2
    n = _as_int(ln)
    seg = b[hl:hl + max(n, 0)]
    if pseudohdr(in_cksum(seg, n), b, n) != 0:
        return 3
    return 0


def set_tcp(b, caplen, fixoff=False):
    b = bytearray(b)
    if caplen < 20:
        return 2, bytes(b)
    hl = (b[0] & 0xF) * 4
    if hl > caplen:
        return 2, bytes(b)
    plen = (be16(b, 2) - hl) & M32
    tlen = caplen - hl
    if plen < 20 or plen > tlen:
        return 2, bytes(b)
    if fixoff:
        off = (b[hl + 12] >> 4) * 4
        frag = be16(b, 6) & 0x3FFF
        if off < 20:
            b[hl + 12] = (b[hl + 12] & 0xF) | 0x50
        elif off > plen and not frag:
            b[hl + 12] = (b[hl + 12] & 0xF) | (((plen >> 2) & 0xF) << 4)
    b[hl + 16:hl + 18] = b"\0\0"
    struct.pack_into("<H", b, hl + 16, pseudohdr(in_cksum(b[hl:hl + plen]), b, plen))
    return 0, bytes(b)


def check_icmp(b, caplen):
    """CheckICMPHeader (checkicmpheader.cc:83-141) with the oracle's guards."""
    if caplen < 20:
        return 2
    if b[9] != 1:
        return 1
    hl = (b[0] & 0xF) * 4
    if caplen < hl or caplen - hl < 8:
        return 2
    ilen = caplen - hl
    t = b[hl]
    need = {3: (">=", 36), 4: (">=", 36), 5: (">=", 36), 11: (">=", 36), 12: (">=", 36),
            13: ("==", 20), 14: ("==", 20), 15: ("==", 8), 16: ("==", 8)}.get(t)
    if need and ((need[0] == ">=" and ilen < need[1]) or (need[0] == "==" and ilen != need[1])):
        return 2
    return 3 if in_cksum(b[hl:hl + ilen]) != 0 else 0


def dec_ttl(b, caplen, multicast=True):
    """DecIPTTL (decipttl.cc:45-77): returns (status, new bytes).  The
    checksum is updated with the general RFC 1624 form (ip.h:177-185) for
    the 16-bit word {ttl, proto}, not the reference's 0xFEFF shortcut."""
    b = bytearray(b)
    if caplen < 20 or (not multicast and (b[16] & 0xF0) == 0xE0):
        return 2, bytes(b)
    if b[8] <= 1:
        return 1, bytes(b)
    old_hw = be16(b, 8)
    b[8] -= 1
    new_hw = be16(b, 8)
    hc = be16(b, 10)
    s = ((~hc) & 0xFFFF) + ((~old_hw) & 0xFFFF) + new_hw
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    struct.pack_into(">H", b, 10, (~s) & 0xFFFF)
    return 0, bytes(b)


# ---- IP output path (RFC 791 Record Route / Timestamp processing) ----------
def _ip_resum(b, hl):
    """ip_sum = 0, then the header checksum over hl bytes."""
    b[10:12] = b"\0\0"
    struct.pack_into("<H", b, 10, in_cksum(bytes(b[:hl])))


def gw_walk(b, caplen, my_ip, my_addrs, ts):
    """Process RR (7) and TS (68) options in place.  Returns (problem or
    None, touched, changed).  Option bytes at/after caplen read as 0."""
    hl = (b[0] & 0xF) * 4
    at = lambda i: b[i] if i < caplen else 0            # noqa: E731
    mine_b = struct.pack("<I", my_ip)
    ts_b = struct.pack("<I", ts)
    touched = changed = False
    i = 20
    while i < hl:
        kind = b[i]
        if kind == 0:
            break
        if kind == 1:
            i += 1
            continue
        olen = at(i + 1)
        if olen < 2 or i + olen > hl:
            return i + 1, touched, changed
        if kind not in (7, 68):
            i += olen
            continue
        touched = True
        ptr = at(i + 2)               # 1-origin pointer to the next free slot
        if kind == 7:
            if ptr >= 4 and ptr - 1 + 4 <= olen:
                b[i + ptr - 1:i + ptr + 3] = mine_b
                b[i + 2] = (ptr + 4) & 0xFF
                changed = True
            elif ptr - 1 != olen:                          # not simply full
                return i + 2, touched, changed
        else:
            of, flag = at(i + 3) >> 4, at(i + 3) & 0xF
            slot = ptr - 1
            full = False
            if slot < 4:
                return i + 2, touched, changed
            if flag == 0:
                if slot + 4 <= olen:
                    b[i + slot:i + slot + 4] = ts_b
                    b[i + 2] = (ptr + 4) & 0xFF
                    changed = True
                else:
                    full = True
            elif flag == 1:
                if slot + 8 <= olen:
                    b[i + slot:i + slot + 4] = mine_b
                    b[i + slot + 4:i + slot + 8] = ts_b
                    b[i + 2] = (ptr + 8) & 0xFF
                    changed = True
                else:
                    full = True
            elif flag == 3 and slot + 8 <= olen:
                if u32le(bytes(b), i + slot) in my_addrs:
                    b[i + slot + 4:i + slot + 8] = ts_b
                    b[i + 2] = (ptr + 8) & 0xFF
                    changed = True
            else:
                return i + 3, touched, changed
            if full:
                if of >= 15:
                    return i + 3, touched, changed
                b[i + 3] = ((of + 1) << 4) | flag
                changed = True
        i += olen
    return None, touched, changed


def ip_gw_options(b, caplen, my_ip, my_addrs, ts):
    """IPGWOptions: returns (code, problem, new bytes)."""
    b = bytearray(b)
    hl = (b[0] & 0xF) * 4 if caplen >= 20 else 0
    if caplen < 20 or hl <= 20 or hl > caplen:
        return 0, 0, bytes(b)
    prob, touched, _ = gw_walk(b, caplen, my_ip, set(my_addrs), ts)
    if prob is not None:
        return 1, prob, bytes(b)
    if touched:
        _ip_resum(b, hl)
    return 0, 0, bytes(b)


def fix_ip_src(b, caplen, anno, my_ip):
    b = bytearray(b)
    if anno and caplen >= 20 and (b[0] & 0xF) * 4 <= caplen:
        b[12:16] = struct.pack("<I", my_ip)
        _ip_resum(b, (b[0] & 0xF) * 4)
    return bytes(b)


def ip_output_combo(b, caplen, flags, my_ip, mtu, ts):
    """IPOutputCombo after DropBroadcasts/PaintTee: (port, problem, bytes).
    The TTL step uses the general RFC 1624 update (ip.h:177-185)."""
    b = bytearray(b)
    if caplen < 20:
        return 0, 0, bytes(b)
    hl = (b[0] & 0xF) * 4
    changed = False
    if 20 < hl <= caplen:
        prob, _, changed = gw_walk(b, caplen, my_ip, {my_ip}, ts)
        if prob is not None:
            return 2, prob, bytes(b)
    if flags & 1:
        b[12:16] = struct.pack("<I", my_ip)
        changed = True
    if changed and hl <= caplen:
        _ip_resum(b, hl)
    if b[8] <= 1:
        return 3, 0, bytes(b)
    st, nb = dec_ttl(bytes(b), caplen)
    assert st == 0
    return (4 if caplen > mtu else 0), 0, nb


# ---- IPFragmenter (RFC 791 fragmentation) ----------------------------------
def _copied_options(h):
    """Options with the copied flag, NOPs dropped, EOL-padded to 4 bytes."""
    hl = (h[0] & 0xF) * 4
    out = bytearray()
    i = 20
    while i < hl:
        k = h[i]
        if k == 1:
            i += 1
            continue
        if k == 0 or i + 1 == hl or h[i + 1] < 2 or i + h[i + 1] > hl:
            break
        if k & 0x80:
            out += h[i:i + h[i + 1]]
        i += h[i + 1]
    while len(out) % 4:
        out.append(0)
    return bytes(out)


def ip_fragment(pkt, mtu, honor_df=False, new_id=None):
    """Returns (port, first fragment bytes or None, [other fragments])."""
    n = len(pkt)
    if n <= mtu:
        return 0, None, []
    if n < 20:
        return 1, None, []
    b = bytearray(pkt)
    hl = (b[0] & 0xF) * 4
    per = (mtu - hl) // 8 * 8 if mtu >= hl else -1
    total_data = be16(b, 2) - hl
    if (b[6] & 0x40 and honor_df) or per < 8:
        return 1, None, []
    if b[6] & 0x40:
        if new_id is not None:
            struct.pack_into("<H", b, 4, new_id)
        b[6] &= 0xBF
    more = bool(b[6] & 0x20)
    struct.pack_into(">H", b, 2, hl + per)
    b[6] |= 0x20
    struct.pack_into("<H", b, 10, 0)
    struct.pack_into("<H", b, 10, in_cksum(bytes(b[:hl])))
    first = bytes(b[:hl + per])
    opts = _copied_options(b)
    qhl = 20 + len(opts)
    frags = []
    pos = per
    payload = bytes(b[hl:]) + bytes(max(0, hl + total_data - n))
    while pos < total_data:
        size = min((mtu - qhl) // 8 * 8, total_data - pos)
        q = bytearray(b[:20]) + opts + payload[pos:pos + size]
        q[0] = (q[0] & 0xF0) | (qhl // 4)
        fo = (be16(b, 6) + pos // 8) & 0xFFFF
        if pos + size >= total_data and not more:
            fo &= ~0x2000
        struct.pack_into(">H", q, 6, fo)
        struct.pack_into(">H", q, 2, qhl + size)
        struct.pack_into("<H", q, 10, 0)
        struct.pack_into("<H", q, 10, in_cksum(bytes(q[:qhl])))
        frags.append(bytes(q))
        pos += size
    return 2, first, frags


# ---------------------------------------------------------------------------
# pcap ingest: FromDump's record loop (elements/userlevel/fromdump.cc:226-290,
# 328-413) and FORCE_IP (elements/userlevel/fakepcap.cc:121-330), written
# from the pcap format and the link-layer headers.
# ---------------------------------------------------------------------------
FORCE_IPABLE = {101, 12, 1, 123, 10, 100, 113, 104, 105, 119, 50, 9, 0, 127}


def _is_ip_ethertype(b, i):
    return i + 2 <= len(b) and ((b[i] << 8) | b[i + 1]) in (0x0800, 0x86DD)


def force_ip(rec, dlt):
    """Offset of the IP header FORCE_IP finds in record bytes `rec`, or -1."""
    n = len(rec)

    def eth(i):
        if i + 14 <= n:
            et = (rec[i + 12] << 8) | rec[i + 13]
            if et in (0x0800, 0x86DD):
                return i + 14
            if et == 0x8100 and i + 18 <= n and _is_ip_ethertype(rec, i + 16):
                return i + 18
        return None

    def fddi(i):
        if i + 21 > n or (rec[i] & 0xF0) != 0x50:
            return None
        return rfc1483(i + 13)

    def rfc1483(i):
        if i + 8 <= n and bytes(rec[i:i + 6]) == b"\xAA\xAA\x03\x00\x00\x00" and _is_ip_ethertype(rec, i + 6):
            return i + 8
        if i + 4 <= n and rec[i] == 0x06 and rec[i + 1] == 0x06:
            return i + 4
        if i + 8 <= n and rec[i] == 0xAA and rec[i + 1] == 0xAA:
            org = (rec[i + 3] << 16) | (rec[i + 4] << 8) | rec[i + 5]
            if org in (0, 0xF8):
                return eth(i - 6)
            if org == 0x0080C2:
                et = (rec[i + 6] << 8) | rec[i + 7]
                if et in (1, 7):
                    return eth(i + 8)
                if et in (4, 0xA):
                    return fddi(i + 9)
        return None

    def wifi(i):
        if i + 24 <= n and (rec[i] & 0x0C) == 0x08:
            return rfc1483(i + (30 if (rec[i + 1] & 3) == 3 else 24))
        return None

    def chdlc(i):
        return i + 4 if i + 4 <= n and _is_ip_ethertype(rec, i + 2) else None

    ip = None
    if dlt in (101, 12):
        ip = 0
    elif dlt == 1:
        ip = eth(0)
    elif dlt == 10:
        ip = fddi(0)
    elif dlt == 123:
        ip = rfc1483(4)
    elif dlt == 100:
        ip = rfc1483(0)
    elif dlt == 113:
        ip = 16 if n >= 16 and _is_ip_ethertype(rec, 14) else None
    elif dlt == 104:
        ip = chdlc(0)
    elif dlt == 50:
        if n >= 4:
            if rec[0] == 0xFF:
                ip = 4 if rec[2] == 0 and rec[3] in (0x21, 0x57) else None
            elif rec[0] in (0x0F, 0x8F):
                ip = chdlc(0)
    elif dlt == 9:
        i = 2 if n >= 2 and rec[0] == 0xFF and rec[1] == 0x03 else 0
        if i + 2 <= n:
            if rec[i] in (0x21, 0x57):
                ip = i + 1
            elif rec[i] == 0 and rec[i + 1] in (0x21, 0x57):
                ip = i + 2
    elif dlt == 119:
        ip = wifi(144)
    elif dlt == 105:
        ip = wifi(0)
    elif dlt == 127:
        if n >= 4:
            ln = (rec[3] << 8) | rec[2]
            if ln >= 8:
                ip = wifi(ln)
    elif dlt == 0:
        if n >= 4:
            fam = rec[0] | (rec[1] << 8)
            if fam == 0:
                fam = (rec[2] << 8) | rec[3]
            if fam in (2, 24, 28, 30):
                ip = 4
    # fakepcap.cc:318-330 (plus the domain guard: the header byte must exist)
    if ip is None or ip < 0 or ip >= n:
        return -1
    v = rec[ip] >> 4
    if v == 4:
        hl = rec[ip] & 0xF
        return ip if hl >= 5 and ip + 4 * hl <= n else -1
    if v == 6:
        return ip if ip + 40 <= n else -1
    return -1


def read_pcap(data, want_force_ip=True):
    """(info, records): records = [(bytes, wire_len, ts_ns, nh)] as FromDump
    would emit them, or raises ValueError(message)."""
    if len(data) < 24:
        raise ValueError("not a tcpdump file (too short)")
    magics = (0xA1B2C3D4, 0xA1B23C4D, 0xA1B2CD34)
    end = "<"
    magic = struct.unpack_from("<I", data, 0)[0]
    if magic not in magics:
        end = ">"
        magic = struct.unpack_from(">I", data, 0)[0]
    if magic not in magics:
        raise ValueError("not a tcpdump file (bad magic number)")
    vmaj, vmin = struct.unpack_from(end + "HH", data, 4)
    dlt = struct.unpack_from(end + "I", data, 20)[0]
    if vmaj != 2:
        raise ValueError("unknown major version %d" % vmaj)
    dlt = 101 if dlt == 12 else dlt
    fip = want_force_ip
    if fip and dlt not in FORCE_IPABLE:
        raise ValueError("unknown linktype %d; can't force IP packets" % dlt)
    if dlt == 101:
        fip = True
    extra = 8 if magic == 0xA1B2CD34 else 0
    nano = magic == 0xA1B23C4D
    pos, recs, stopped = 24, [], False
    while pos + 16 <= len(data):
        sec, sub, a, b = struct.unpack_from(end + "iiII", data, pos)
        if vmin > 3 or (vmin == 3 and a <= b):
            cap, ln = a, b
        else:
            cap, ln = b, a
        if cap > 65535:
            stopped = True
            break
        skip = 0
        if cap > ln:
            skip, cap = cap - ln, ln
        pos += 16 + extra
        if pos + cap > len(data):
            break
        rec = data[pos:pos + cap]
        recs.append((rec, ln, sec * 1000000000 + (sub if nano else sub * 1000),
                     force_ip(rec, dlt) if fip else -1))
        pos += cap + skip
    return {"linktype": dlt, "nanosecond": int(nano), "swapped": int(end == ">"), "force_ip": int(fip),
            "stopped": stopped}, recs


def write_pcap(records, linktype=1, magic=0xA1B2C3D4, big_endian=False, vmin=4, lens=None, raw_headers=None):
    """A tcpdump file: records = [(bytes, sec, subsec)]; lens = wire lengths
    (default: the captured length); raw_headers[k] = (a, b) written as the
    record's caplen/len words verbatim."""
    e = ">" if big_endian else "<"
    out = bytearray(struct.pack(e + "IHHiIII", magic, 2, vmin, 0, 0, 65535, linktype))
    for k, (rec, sec, sub) in enumerate(records):
        ln = len(rec) if lens is None else lens[k]
        a, b = (len(rec), ln) if raw_headers is None or raw_headers[k] is None else raw_headers[k]
        out += struct.pack(e + "iiII", sec, sub, a, b)
        if magic == 0xA1B2CD34:
            out += bytes(8)
        out += rec
    return bytes(out)
