"""Seeded packet batches that exercise every branch of the checksum elements.

Test infrastructure.  Packets are built with zero checksum fields, made
valid by the ORACLE's Set elements, then mutated (bit flips, bad versions
and header lengths, IP options incl. SSRR/LSRR/NOP/EOL/malformed, bad
ip_len/uh_ulen/th_off, fragments, uh_sum = 0, truncated caplen), and placed
at arbitrary byte alignments in one arena.
"""
import numpy as np

from tests import oracle_lib


def _options(rng, words):
    """`words` 32-bit words of IP options, mixing the kinds the option walk
    distinguishes (lib/in_cksum.c:88-108)."""
    n = 4 * words
    out = bytearray(n)
    o = 0
    while o < n:
        kind = rng.integers(0, 8)
        room = n - o
        if kind == 0:                         # NOP
            out[o] = 1
            o += 1
        elif kind == 1:                       # EOL, then garbage after it
            out[o] = 0
            o += 1
            if rng.integers(0, 2):
                out[o:n] = rng.integers(0, 256, room - 1, dtype=np.uint8).tobytes()
                o = n
        elif kind in (2, 3) and room >= 7:    # SSRR / LSRR with >= 1 address
            naddr = int(rng.integers(1, (room - 3) // 4 + 1))
            ln = 3 + 4 * naddr
            out[o] = 137 if kind == 2 else 131
            out[o + 1] = ln if rng.integers(0, 8) else int(rng.integers(0, 256))
            out[o + 2] = 4
            out[o + 3:o + ln] = rng.integers(0, 256, ln - 3, dtype=np.uint8).tobytes()
            o += ln
        elif kind == 4 and room >= 4:         # record route / other with length
            ln = int(rng.integers(2, room + 1))
            out[o] = int(rng.choice([7, 68, 130, 148]))
            out[o + 1] = ln
            out[o + 2:o + ln] = rng.integers(0, 256, ln - 2, dtype=np.uint8).tobytes()
            o += ln
        elif kind == 5:                       # malformed length (< 2 or past the end)
            out[o] = int(rng.choice([137, 131, 7]))
            if o + 1 < n:
                out[o + 1] = int(rng.choice([0, 1, room + 1, 255]))
            o = n
        else:
            out[o] = 1
            o += 1
    return bytes(out)


ICMP_TYPES = [0, 3, 4, 5, 8, 9, 11, 12, 13, 14, 15, 16, 17, 18, 42]


def build(rng, proto, total, opt_words=0):
    """One well-formed IPv4 packet of `total` bytes (checksums zero)."""
    hl = 20 + 4 * opt_words
    tl = max(total, hl + (8 if proto in (1, 17) else 20))
    if proto == 1:
        itype = int(rng.choice(ICMP_TYPES))
        if itype in (13, 14) and rng.random() < 0.7:      # exact-size types (checkicmpheader.cc:96-134)
            tl = hl + 20
        elif itype in (15, 16) and rng.random() < 0.7:
            tl = hl + 8
        elif itype in (3, 4, 5, 11, 12) and rng.random() < 0.3:
            tl = hl + int(rng.integers(8, 44))
    b = bytearray(rng.integers(0, 256, tl, dtype=np.uint8).tobytes())
    b[0] = 0x40 | (hl // 4)
    b[1] = 0
    b[2:4] = tl.to_bytes(2, "big")
    b[6:8] = b"\0\0"
    b[8] = 64
    b[9] = proto
    b[10:12] = b"\0\0"
    b[20:hl] = _options(rng, opt_words)
    if proto == 17:
        b[hl + 4:hl + 6] = (tl - hl).to_bytes(2, "big")
        b[hl + 6:hl + 8] = b"\0\0"
    elif proto == 1:
        b[hl] = itype
        b[hl + 2:hl + 4] = b"\0\0"
    else:
        b[hl + 12] = (5 + int(rng.integers(0, 3))) << 4 | (b[hl + 12] & 0xF)
        b[hl + 16:hl + 18] = b"\0\0"
    return bytes(b)


def _mutate(rng, b, proto):
    b = bytearray(b)
    hl = (b[0] & 0xF) * 4
    r = rng.random()
    if r < 0.06:
        b[0] = (b[0] & 0x0F) | (int(rng.integers(0, 16)) << 4)          # version
    elif r < 0.12:
        b[0] = (b[0] & 0xF0) | int(rng.integers(0, 16))                 # ip_hl
    elif r < 0.18:
        b[2:4] = int(rng.integers(0, 65536)).to_bytes(2, "big")         # ip_len
    elif r < 0.24 and len(b) > hl + 13:
        if proto == 17:
            b[hl + 4:hl + 6] = int(rng.choice([0, 7, 8, len(b) - hl + 1, int(rng.integers(0, 65536))])).to_bytes(2, "big")
        elif proto == 1:
            b[hl] = int(rng.choice(ICMP_TYPES))
        else:
            b[hl + 12] = (int(rng.integers(0, 16)) << 4) | (b[hl + 12] & 0xF)
    elif r < 0.30:
        b[6] |= int(rng.choice([0x20, 0x01, 0x80, 0x40]))               # MF / offset / RF / DF
    elif r < 0.36 and proto == 17 and len(b) >= hl + 8:
        b[hl + 6:hl + 8] = b"\0\0"                                       # uh_sum = 0
    elif r < 0.48:
        k = int(rng.integers(0, len(b)))
        b[k] ^= 1 << int(rng.integers(0, 8))                             # bit flip
    elif r < 0.52:
        b[9] = int(rng.integers(0, 256))                                 # protocol
    return bytes(b)


def make_batch(rng, n, proto, max_total=1600, opt_frac=0.2, mutate_frac=0.5, tiny_frac=0.05,
               trunc_frac=0.08, align="any", set_checksums=True, fixed_stride=None):
    """Returns (arena uint8, off uint64, length uint32, max_len)."""
    pkts = []
    for _ in range(n):
        if rng.random() < tiny_frac:
            tl = int(rng.integers(0, 48))
            pkts.append(rng.integers(0, 256, tl, dtype=np.uint8).tobytes())
            continue
        ow = int(rng.integers(1, 11)) if rng.random() < opt_frac else 0
        tl = int(rng.integers(20 + 4 * ow + 20, max_total + 1))
        pkts.append(build(rng, proto, tl, ow))
    caplen = np.array([len(p) for p in pkts], np.uint32)
    if fixed_stride:
        off = np.arange(n, dtype=np.uint64) * np.uint64(fixed_stride)
        size = n * fixed_stride + 64
    else:
        off = np.zeros(n, np.uint64)
        pos = 0
        for i, p in enumerate(pkts):
            if align == "any":
                pos += int(rng.integers(0, 16))
            elif align == "even":
                pos += 2 * int(rng.integers(0, 8))
            elif align == 64:                  # 64 B-aligned packet starts (the benches' layouts)
                pos = (pos + 63) // 64 * 64
            off[i] = pos
            pos += len(p) + int(rng.integers(0, 24))
        size = pos + 64
    arena = np.zeros(size, np.uint8)
    for i, p in enumerate(pkts):
        arena[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
    if set_checksums:
        oracle_lib.batch("set_ip", arena, n, off=off, length=caplen)
        if proto == 1:
            set_icmp_checksums(arena, off, caplen)
        else:
            oracle_lib.batch("set_udp" if proto == 17 else "set_tcp", arena, n, off=off, length=caplen, arg=0)
    for i in range(n):
        if rng.random() < mutate_frac and caplen[i] >= 20:
            o = int(off[i])
            mb = _mutate(rng, arena[o:o + caplen[i]].tobytes(), proto)
            arena[o:o + caplen[i]] = np.frombuffer(mb, np.uint8)
        if rng.random() < trunc_frac and caplen[i] > 0:
            caplen[i] = int(rng.integers(0, caplen[i]))
    return arena, off, caplen, int(caplen.max()) if n else 0


def set_icmp_checksums(arena, off, caplen):
    """icmp_cksum over [th, end) as ICMPPingEncap does (icmppingencap.cc:85,99);
    Click has no SetICMPChecksum element, so fixtures set it here."""
    L = oracle_lib.load_oracle()
    for i in range(len(off)):
        o, c = int(off[i]), int(caplen[i])
        if c < 20:
            continue
        hl = (int(arena[o]) & 0xF) * 4
        if hl < 20 or c < hl + 4:
            continue
        arena[o + hl + 2:o + hl + 4] = 0
        seg = arena[o + hl:o + c].tobytes()
        v = L.oracle_in_cksum(seg, len(seg))
        arena[o + hl + 2] = v & 0xFF
        arena[o + hl + 3] = v >> 8


def vary_ttl(rng, arena, off, caplen, frac=0.4):
    """DecIPTTL inputs: TTLs at the 0/1/2/255 edges and multicast
    destinations (decipttl.cc:51-57) in a fraction of the packets."""
    for i in range(len(off)):
        o = int(off[i])
        if caplen[i] < 20 or rng.random() >= frac:
            continue
        r = rng.random()
        if r < 0.5:
            arena[o + 8] = int(rng.choice([0, 1, 2, 255]))
        elif r < 0.8:
            arena[o + 16] = 0xE0 | int(rng.integers(0, 16))
        else:
            arena[o + 10] = int(rng.integers(0, 256))          # stale ip_sum: updated all the same


def _gw_options(rng, words, my_ip):
    """`words` 32-bit words of options built around Record Route (7) and
    Timestamp (68) at every pointer / flag / overflow edge
    (ipgwoptions.cc:59-153), mixed with NOP/EOL/other/malformed options."""
    n = 4 * words
    out = bytearray(n)
    o = 0
    while o < n:
        room = n - o
        kind = int(rng.integers(0, 10))
        if kind <= 3 and room >= 3:                       # Record Route
            ln = int(rng.integers(3, room + 1))
            out[o], out[o + 1] = 7, ln
            out[o + 2] = int(rng.choice([4, 4 + 4 * int(rng.integers(0, 8)), ln + 1, ln - 2, 0, 1, 3,
                                         int(rng.integers(0, 256))]))
            out[o + 3:o + ln] = rng.integers(0, 256, ln - 3, dtype=np.uint8).tobytes()
            o += ln
        elif kind <= 6 and room >= 4:                     # Timestamp
            ln = int(rng.integers(4, room + 1))
            flg = int(rng.choice([0, 1, 3, 2, 4]))
            of = int(rng.choice([0, 1, 14, 15]))
            out[o], out[o + 1] = 68, ln
            out[o + 2] = int(rng.choice([5, 5 + 4 * int(rng.integers(0, 9)), ln + 1, ln - 3, 4, 1,
                                         int(rng.integers(0, 256))]))
            out[o + 3] = (of << 4) | flg
            out[o + 4:o + ln] = rng.integers(0, 256, ln - 4, dtype=np.uint8).tobytes()
            if flg == 3 and ln >= 12 and rng.random() < 0.6:
                p = out[o + 2] - 1
                if 4 <= p and p + 8 <= ln:
                    out[o + p:o + p + 4] = int(my_ip).to_bytes(4, "little")
            o += ln
        elif kind == 7:
            out[o] = 1
            o += 1
        elif kind == 8:
            out[o] = 0
            o += 1
        else:                                             # other / malformed length
            out[o] = int(rng.choice([130, 148, 7, 68]))
            if o + 1 < n:
                out[o + 1] = int(rng.choice([0, 1, room + 1, 2, min(room, 255)]))
            o = n
    return bytes(out)


def gw_batch(rng, n, my_ip, max_total=200, opt_frac=0.7, tiny_frac=0.03, trunc_frac=0.05):
    """Batch for IPGWOptions / FixIPSrc / IPOutputCombo: valid IPv4 headers
    (ip_sum set) with RR/TS options on most packets, TTLs at the 0/1/2
    edges, a few tiny or truncated packets; arbitrary alignments.  Returns
    (arena, off, length, flags) with flags bit 0 = FIX_IP_SRC_ANNO."""
    pkts = []
    for _ in range(n):
        if rng.random() < tiny_frac:
            pkts.append(rng.integers(0, 256, int(rng.integers(0, 24)), dtype=np.uint8).tobytes())
            continue
        ow = int(rng.integers(1, 11)) if rng.random() < opt_frac else 0
        tl = int(rng.integers(20 + 4 * ow + 8, max_total + 1))
        b = bytearray(build(rng, 17, tl, 0))
        b[0] = 0x40 | (5 + ow)
        b[20:20 + 4 * ow] = _gw_options(rng, ow, my_ip)
        if rng.random() < 0.2:
            b[8] = int(rng.choice([0, 1, 2]))
        pkts.append(bytes(b))
    caplen = np.array([len(p) for p in pkts], np.uint32)
    off = np.zeros(n, np.uint64)
    pos = 0
    for i, p in enumerate(pkts):
        pos += int(rng.integers(0, 8))
        off[i] = pos
        pos += len(p) + int(rng.integers(0, 8))
    arena = np.zeros(pos + 64, np.uint8)
    for i, p in enumerate(pkts):
        arena[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
    oracle_lib.batch("set_ip", arena, n, off=off, length=caplen)
    for i in range(n):
        if rng.random() < trunc_frac and caplen[i] > 0:
            caplen[i] = int(rng.integers(0, caplen[i]))
    flags = (rng.random(n) < 0.3).astype(np.uint8)
    return arena, off, caplen, flags


def frag_batch(rng, n, max_total=3000):
    """Batch for IPFragmenter: IPv4 packets with copied / uncopied / NOP /
    malformed options, DF / MF / nonzero fragment offsets, ip_len below and
    above the captured length, tiny packets; arbitrary alignments.  Returns
    (arena, off, length)."""
    pkts = []
    for _ in range(n):
        if rng.random() < 0.03:
            pkts.append(rng.integers(0, 256, int(rng.integers(0, 30)), dtype=np.uint8).tobytes())
            continue
        ow = int(rng.integers(1, 11)) if rng.random() < 0.4 else 0
        tl = int(rng.integers(20 + 4 * ow + 8, max_total + 1))
        b = bytearray(build(rng, int(rng.choice([6, 17])), tl, 0))
        b[0] = 0x40 | (5 + ow)
        opts = bytearray(_options(rng, ow))
        for k in range(len(opts)):                      # set the copied flag on some kinds
            if opts[k] in (137, 131, 7, 68, 130, 148) and rng.random() < 0.5:
                opts[k] |= 0x80
        b[20:20 + 4 * ow] = opts
        r = rng.random()
        if r < 0.15:
            b[6] |= 0x40                                # DF
        elif r < 0.3:
            b[6] |= 0x20                                # MF
        elif r < 0.4:
            b[6:8] = (int(rng.integers(1, 0x1FFF)) | (0x2000 if rng.random() < 0.5 else 0)).to_bytes(2, "big")
        if rng.random() < 0.08:
            b[2:4] = int(rng.integers(0, tl + 64)).to_bytes(2, "big")
        pkts.append(bytes(b))
    caplen = np.array([len(p) for p in pkts], np.uint32)
    off = np.zeros(n, np.uint64)
    pos = 0
    for i, p in enumerate(pkts):
        pos += int(rng.integers(0, 16))
        off[i] = pos
        pos += len(p)
    arena = np.zeros(pos + 64, np.uint8)
    for i, p in enumerate(pkts):
        arena[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
    oracle_lib.batch("set_ip", arena, n, off=off, length=caplen)
    return arena, off, caplen
