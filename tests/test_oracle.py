"""CPU tests: pin the oracle (oracle/cksum_oracle.c) before it checks the GPU.

1. every golden vector extracted from the reference's own files
   (tests/golden/golden_vectors.json, made by tests/golden/make_golden.py);
2. agreement with a second, independently written restatement (tests/pyref.py)
   on randomized and fuzzed inputs, including the u32-wrap overflow case;
3. the synthetic-traffic generator's invariants.
"""
import ctypes
import json
import os
import struct

import numpy as np
import pytest

from tests import oracle_lib, pyref, fuzz

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")


def golden_vectors():
    with open(GOLDEN) as f:
        return json.load(f)["vectors"]


def run_vector_oracle(v):
    """Returns (result, bytes after) for one golden vector on the oracle."""
    if "fill" in v:
        data = bytes([v["fill"]]) * v["caplen"]
    else:
        data = bytes.fromhex(v["l3"])
    arena = np.frombuffer(data + b"\0" * 8, np.uint8).copy()
    op = v["op"]
    if op == "set_tcp_then_rfc1071":
        codes, sums = oracle_lib.batch("set_tcp", arena, 1, stride=0, fixed_len=v["caplen"], arg=0)
        return int(codes[0]), arena[:v["caplen"]].tobytes()
    codes, sums = oracle_lib.batch(op, arena, 1, stride=0, fixed_len=v["caplen"], arg=v.get("arg", 1))
    if op == "in_cksum" or op.startswith("set_"):
        res = int(sums[0])
    else:
        res = int(codes[0])
    return res, arena[:v["caplen"]].tobytes()


def rfc1071_tcp_ok(pkt, final_dst):
    """Independent verification in RFC 793/1071 terms (big-endian one's
    complement sum over pseudo-header + segment), as tcpdump does."""
    hl = (pkt[0] & 0xF) * 4
    seg = pkt[hl:]
    dst = bytes(int(x) for x in final_dst.split("."))
    ph = pkt[12:16] + dst + bytes([0, pkt[9]]) + len(seg).to_bytes(2, "big")
    data = ph + seg + (b"\0" if len(seg) % 2 else b"")
    s = 0
    for i in range(0, len(data), 2):
        s += (data[i] << 8) | data[i + 1]
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s == 0xFFFF


@pytest.mark.parametrize("v", golden_vectors(), ids=lambda v: v["name"])
def test_golden_vector(v):
    res, after = run_vector_oracle(v)
    if v["op"] == "set_tcp_then_rfc1071":
        assert res == 0
        assert rfc1071_tcp_ok(after, v["final_dst"]), v["source"]
    else:
        assert res == v["expect"], v["source"]


def test_golden_covers_every_op():
    ops = {v["op"] for v in golden_vectors()}
    assert {"in_cksum", "check_ip", "set_ip", "check_udp", "set_udp", "check_tcp", "set_tcp"} <= ops
    pins = {v["pin"] for v in golden_vectors()}
    assert {"reference-output", "reference-accepts", "captured", "survey-ref-run", "tcpdump-ok"} <= pins


def test_in_cksum_matches_pyref_random():
    L = oracle_lib.load_oracle()
    rng = np.random.default_rng(1)
    for _ in range(400):
        n = int(rng.integers(0, 3000))
        kind = rng.integers(0, 4)
        if kind == 0:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            b = b"\0" * n
        elif kind == 2:
            b = b"\xff" * n
        else:
            b = bytes(rng.integers(250, 256, n, dtype=np.uint8))
        assert L.oracle_in_cksum(b, n) == pyref.in_cksum(b)


@pytest.mark.parametrize("n", [131072, 131074, 131076, 200000, 262147])
def test_in_cksum_u32_wrap(n):
    """The reference's u32 accumulator wraps past 131,074 bytes of 0xFF."""
    L = oracle_lib.load_oracle()
    b = b"\xff" * n
    assert L.oracle_in_cksum(b, n) == pyref.in_cksum(b)


def test_in_cksum_edge_lengths():
    L = oracle_lib.load_oracle()
    assert L.oracle_in_cksum(b"", 0) == 0xFFFF
    assert L.oracle_in_cksum(b"\x12", 1) == (~0x12) & 0xFFFF
    assert L.oracle_in_cksum(b"\x12\x34", 2) == (~0x3412) & 0xFFFF
    assert L.oracle_in_cksum(b"\x12\x34\x56", 3) == (~(0x3412 + 0x56)) & 0xFFFF
    assert L.oracle_in_cksum(b"abcd", -4) == 0xFFFF         # negative int len sums nothing
    # a nonzero input whose folded sum is 0xFFFF yields 0x0000
    assert L.oracle_in_cksum(b"\xff\xff", 2) == 0


def test_pseudohdr_matches_pyref_random():
    L = oracle_lib.load_oracle()
    rng = np.random.default_rng(2)
    for _ in range(3000):
        csum = int(rng.integers(0, 65536))
        src, dst = (int(x) for x in rng.integers(0, 2 ** 32, 2, dtype=np.uint64))
        proto = int(rng.integers(0, 256))
        plen = int(rng.integers(-70000, 70000))
        assert L.oracle_in_cksum_pseudohdr_raw(csum, src, dst, proto, plen) == \
            pyref.pseudohdr_raw(csum, src, dst, proto, plen & 0xFFFFFFFF)


def test_pseudohdr_hard_matches_pyref_options():
    L = oracle_lib.load_oracle()
    rng = np.random.default_rng(3)
    for _ in range(3000):
        words = int(rng.integers(0, 11))
        hdr = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes()) + fuzz._options(rng, words)
        hdr[0] = 0x40 | (5 + words)
        csum = int(rng.integers(0, 65536))
        plen = int(rng.integers(0, 65536))
        assert L.oracle_in_cksum_pseudohdr(csum, bytes(hdr), plen) == pyref.pseudohdr(csum, bytes(hdr), plen)


def test_update_in_cksum_rfc1624():
    """ip.h:177-185: an incremental update equals a recomputation (except the
    0x0000/0xFFFF representation, ip.h:166-176)."""
    L = oracle_lib.load_oracle()
    rng = np.random.default_rng(4)
    for _ in range(500):
        hdr = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
        hdr[10:12] = b"\0\0"
        s = L.oracle_in_cksum(bytes(hdr), 20)
        struct.pack_into("<H", hdr, 10, s)
        k = 2 * int(rng.integers(0, 10))
        if k == 10:
            continue
        old = struct.unpack_from("<H", hdr, k)[0]
        new = int(rng.integers(0, 65536))
        struct.pack_into("<H", hdr, k, new)
        upd = L.oracle_update_in_cksum(s, old, new)
        hdr2 = bytearray(hdr)
        hdr2[10:12] = b"\0\0"
        full = L.oracle_in_cksum(bytes(hdr2), 20)
        assert upd == full or {upd, full} == {0, 0xFFFF}
    assert L.oracle_update_zero_in_cksum(0, b"\0\0\0\0", 4) == 0xFFFF
    assert L.oracle_update_zero_in_cksum(0, b"\0\1\0\0", 4) == 0


@pytest.mark.parametrize("proto", [17, 6])
def test_elements_match_pyref_fuzz(proto):
    rng = np.random.default_rng(10 + proto)
    arena, off, caplen, _ = fuzz.make_batch(rng, 600, proto, max_total=400)
    n = len(off)
    ops = ["check_ip", "set_ip"] + (["check_udp", "set_udp"] if proto == 17 else ["check_tcp", "set_tcp"])
    for op in ops:
        a = arena.copy()
        codes, sums = oracle_lib.batch(op, a, n, off=off, length=caplen, arg=1 if op != "set_tcp" else 1)
        for i in range(n):
            o, c = int(off[i]), int(caplen[i])
            pkt = arena[o:o + c].tobytes()
            # pyref works on the caplen bytes it may read (domain guards keep
            # the oracle inside them)
            padded = pkt + b"\0" * 64
            if op == "check_ip":
                exp = pyref.check_ip(padded, c)
            elif op == "check_udp":
                exp = pyref.check_udp(padded, c)
            elif op == "check_tcp":
                exp = pyref.check_tcp(padded, c)
            else:
                fn = {"set_ip": pyref.set_ip, "set_udp": pyref.set_udp,
                      "set_tcp": lambda b, cl: pyref.set_tcp(b, cl, True)}[op]
                exp, newb = fn(padded, c)
                assert a[o:o + c].tobytes() == newb[:c], (op, i)
            assert codes[i] == exp, (op, i, pkt.hex())


def test_generator_packets_are_valid():
    """Synthetic traffic: header fields as documented; Set then Check passes."""
    for proto, L in ((17, 1500), (6, 9000), (17, 46)):
        n = 64
        stride = (L + 63) // 64 * 64
        arena = np.zeros(n * stride, np.uint8)
        oracle_lib.gen(arena, n, stride=stride, fixed_len=L, proto=proto)
        p0 = arena[:L].tobytes()
        assert p0[0] == 0x45 and p0[9] == proto and int.from_bytes(p0[2:4], "big") == L
        assert p0[10:12] == b"\0\0"
        oracle_lib.batch("set_ip", arena, n, stride=stride, fixed_len=L)
        c, _ = oracle_lib.batch("check_ip", arena, n, stride=stride, fixed_len=L)
        assert not c.any()
        if L >= 28:
            s = "set_udp" if proto == 17 else "set_tcp"
            k = "check_udp" if proto == 17 else "check_tcp"
            c, _ = oracle_lib.batch(s, arena, n, stride=stride, fixed_len=L, arg=0)
            assert not c.any()
            c, _ = oracle_lib.batch(k, arena, n, stride=stride, fixed_len=L)
            assert not c.any()


def test_oracle_bench_runs():
    L = oracle_lib.load_oracle()
    n, stride = 256, 1536
    arena = np.zeros(n * stride, np.uint8)
    oracle_lib.gen(arena, n, stride=stride, fixed_len=1500)
    dt = L.oracle_bench(oracle_lib.OP_SET_UDP, arena.ctypes.data, stride, 1500, n, 2, 2)
    assert dt > 0


@pytest.mark.parametrize("proto", [17, 6])
def test_fuzz_batches_build(proto):
    """The GPU parity tests' fuzzed batches build (same seeds as there)."""
    for max_total, align in [(96, "any"), (400, "any"), (1600, "even"), (1600, "any"), (5000, "any"),
                             (20000, "even")]:
        rng = np.random.default_rng(proto * 1000 + max_total + (align == "any"))
        n = 3000 if max_total <= 1600 else 400
        arena, off, caplen, ml = fuzz.make_batch(rng, n, proto, max_total=max_total, align=align)
        assert len(off) == n and ml <= max(max_total, 60)


def test_icmp_and_dec_ttl_match_pyref_fuzz():
    """CheckICMPHeader and DecIPTTL: the C oracle against the independent
    Python restatement (pyref) on fuzzed ICMP / TTL-edge batches.  The
    ICMP per-type length rules are pinned by these two restatements of
    checkicmpheader.cc:96-134 (the reference's tests hold no ICMP bytes);
    the checksum arithmetic is in_cksum, pinned by the golden vectors."""
    rng = np.random.default_rng(123)
    arena, off, caplen, _ = fuzz.make_batch(rng, 1500, 1, max_total=300)
    n = len(off)
    codes, _ = oracle_lib.batch("check_icmp", arena.copy(), n, off=off, length=caplen)
    exp = [pyref.check_icmp(arena[int(off[i]):int(off[i]) + int(caplen[i])].tobytes(), int(caplen[i]))
           for i in range(n)]
    assert np.array_equal(codes, np.array(exp))
    assert set(np.unique(codes)) == {0, 1, 2, 3}
    fuzz.vary_ttl(rng, arena, off, caplen)
    for multicast in (0, 1):
        a = arena.copy()
        codes, sums = oracle_lib.batch("dec_ttl", a, n, off=off, length=caplen, arg=multicast)
        for i in range(n):
            o, c = int(off[i]), int(caplen[i])
            st, nb = pyref.dec_ttl(arena[o:o + c].tobytes(), c, bool(multicast))
            assert codes[i] == st and a[o:o + c].tobytes() == nb, (i, multicast)
        assert set(np.unique(codes)) == {0, 1, 2}


def test_dec_ttl_on_reference_headers():
    """DecIPTTL on the IPv4 headers the reference's own files hold (golden
    vectors that CheckIPHeader accepts): TTL drops by one and the RFC 1624
    update equals a full recomputation (the header still checks)."""
    L = oracle_lib.load_oracle()
    seen = 0
    for v in golden_vectors():
        if v["op"] != "check_ip" or v["expect"] != 0 or "l3" not in v:
            continue
        pkt = np.frombuffer(bytes.fromhex(v["l3"]), np.uint8).copy()
        if pkt[8] <= 1:
            continue
        ttl = int(pkt[8])
        codes, sums = oracle_lib.batch("dec_ttl", pkt, 1, off=np.zeros(1, np.uint64),
                                       length=np.array([v["caplen"]], np.uint32))
        assert codes[0] == 0 and pkt[8] == ttl - 1, v["name"]
        hl = (int(pkt[0]) & 0xF) * 4
        assert L.oracle_in_cksum(pkt[:hl].tobytes(), hl) == 0, v["name"]
        seen += 1
    assert seen >= 3


MY_IP = 0x18041A12          # 18.26.4.24 as a raw s_addr word (network order in memory)
TS = 0x40E20100


@pytest.mark.parametrize("op", ["ip_gw_options", "fix_ip_src", "ip_output_combo"])
def test_ip_output_path_matches_pyref(op):
    """IPGWOptions / FixIPSrc / IPOutputCombo: the C oracle against the
    independent Python restatement on option-heavy fuzzed batches; every
    outcome (ports 0/2/3/4, parameter-problem offsets) is exercised."""
    rng = np.random.default_rng(321)
    arena, off, caplen, flags = fuzz.gw_batch(rng, 3000, MY_IP)
    n = len(off)
    addrs = np.array([MY_IP, 0x01020304], np.uint32)
    a = arena.copy()
    codes, prob, sums = oracle_lib.ip_out_batch(op, a, n, off=off, length=caplen, flags=flags, my_ip=MY_IP,
                                                my_addrs=addrs, ts=TS, mtu=120)
    for i in range(n):
        o, c = int(off[i]), int(caplen[i])
        pk = arena[o:o + c].tobytes()
        if op == "ip_gw_options":
            code, p, nb = pyref.ip_gw_options(pk, c, MY_IP, addrs.tolist(), TS)
        elif op == "fix_ip_src":
            code, p, nb = 0, 0, pyref.fix_ip_src(pk, c, flags[i] & 1, MY_IP)
        else:
            code, p, nb = pyref.ip_output_combo(pk, c, int(flags[i]), MY_IP, 120, TS)
        assert (codes[i], prob[i]) == (code, p), (op, i, codes[i], prob[i], code, p)
        assert a[o:o + c].tobytes() == nb, (op, i)
    got = set(np.unique(codes).tolist())
    assert got == {"ip_gw_options": {0, 1}, "fix_ip_src": {0}, "ip_output_combo": {0, 2, 3, 4}}[op], got


def test_iprouter_output_equivalence():
    """iprouter-01.clicktest: the IP output chain IPGWOptions -> FixIPSrc ->
    DecIPTTL and its click-xform replacement IPOutputCombo give the same
    bytes (the test expects OUTA == OUTB), on fuzzed headers with and
    without RR/TS options that pass both without error."""
    rng = np.random.default_rng(99)
    arena, off, caplen, flags = fuzz.gw_batch(rng, 2000, MY_IP)
    n = len(off)
    a1, a2 = arena.copy(), arena.copy()
    g, _, _ = oracle_lib.ip_out_batch("ip_gw_options", a1, n, off=off, length=caplen, my_ip=MY_IP,
                                      my_addrs=np.array([MY_IP], np.uint32), ts=TS)
    oracle_lib.ip_out_batch("fix_ip_src", a1, n, off=off, length=caplen, flags=flags, my_ip=MY_IP)
    d, _ = oracle_lib.batch("dec_ttl", a1, n, off=off, length=caplen)
    port, _, _ = oracle_lib.ip_out_batch("ip_output_combo", a2, n, off=off, length=caplen, flags=flags,
                                         my_ip=MY_IP, ts=TS, mtu=1 << 20)
    same = 0
    for i in range(n):
        o, c = int(off[i]), int(caplen[i])
        if c < 20 or g[i] != 0:
            continue
        # IPGWOptions re-checksums whenever it meets an RR/TS option, the
        # combo only when a byte changed: equal for headers that were valid
        hl = (int(arena[o]) & 0xF) * 4
        if hl < 20 or hl > c or pyref.in_cksum(arena[o:o + hl].tobytes()) != 0:
            continue
        assert port[i] == (3 if d[i] == 1 else 0), i
        assert a1[o:o + c].tobytes() == a2[o:o + c].tobytes(), i
        same += 1
    assert same > 500


def fragment_cases():
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")))["fragment_cases"]


@pytest.mark.parametrize("case", fragment_cases(), ids=lambda c: c["name"])
def test_fragmenter_reproduces_reference_output(case):
    """IPFragmenter-01/02.clicktest: the oracle's fragments are the bytes
    Click itself printed (first fragment rewritten in place, the others
    appended), at several alignments."""
    pkt = bytes.fromhex(case["in"])
    for shift in (0, 1, 2, 3, 13):
        arena = np.zeros(shift + len(pkt) + 16, np.uint8)
        arena[shift:shift + len(pkt)] = np.frombuffer(pkt, np.uint8)
        r = oracle_lib.ip_fragment(arena, 1, case["mtu"], case["honor_df"], off=np.array([shift], np.uint64),
                                   length=np.array([len(pkt)], np.uint32))
        assert r["port"][0] == 2
        got = [arena[shift:shift + int(r["first_len"][0])].tobytes()] + r["frags"]
        assert [g.hex() for g in got] == case["fragments"], (case["name"], shift)


@pytest.mark.parametrize("mtu,honor_df", [(576, False), (1500, True), (68, False), (40, True)])
def test_fragmenter_matches_pyref_fuzz(mtu, honor_df):
    """The C oracle's fragmenter against the independent Python one on
    fuzzed packets (options, DF/MF/offsets, short and long ip_len)."""
    rng = np.random.default_rng(mtu + honor_df)
    arena, off, caplen = fuzz.frag_batch(rng, 600)
    n = len(off)
    nid = rng.integers(0, 65536, n).astype(np.uint16)
    a = arena.copy()
    r = oracle_lib.ip_fragment(a, n, mtu, honor_df, off=off, length=caplen, new_id=nid)
    ports = set()
    for i in range(n):
        o, c = int(off[i]), int(caplen[i])
        port, first, frags = pyref.ip_fragment(arena[o:o + c].tobytes(), mtu, honor_df, int(nid[i]))
        ports.add(port)
        assert r["port"][i] == port, i
        k0 = int(r["frag_first"][i])
        if port == 2:
            assert a[o:o + int(r["first_len"][i])].tobytes() == first, i
            assert r["frags"][k0:k0 + len(frags)] == frags, i
            assert all(r["frag_src"][k0:k0 + len(frags)] == i)
        else:
            assert a[o:o + c].tobytes() == arena[o:o + c].tobytes()
    assert ports == ({0, 1, 2} if honor_df else {0, 2})


def test_config1_fake_iprouter_plumbing_on_cpu():
    """BASELINE config 1 (conf/fake-iprouter.click, CPU, no GPU): the
    forwarding path of its 600,000 frames through the CPU restatement --
    Strip(14) + CheckIPHeader(INTERFACES ...) -> IPGWOptions -> FixIPSrc ->
    DecIPTTL -> IPFragmenter(300), and the click-xform combos
    IPInputCombo -> IPOutputCombo(1, 18.26.4.24, 300) -- forwards every
    frame (iprouter-01 expects 600000) with identical bytes both ways."""
    L = oracle_lib.load_oracle()
    v = [g for g in golden_vectors() if g["name"] == "fake-iprouter-ip-check"][0]
    frame = bytes.fromhex("0000c0ae67ef0000000000000800") + bytes.fromhex(v["l3"])
    n, fl = 600000, len(frame)
    outs = []
    for combo in (False, True):
        arena = np.tile(np.frombuffer(frame, np.uint8), n).copy()
        bad = np.array([0xFF041A12, 0x00041A12, 0xFF071A12, 0x00071A12, 0, 0xFFFFFFFF], np.uint32)
        good = np.array([0x01041A12, 0x01071A12], np.uint32)
        ok = [L.oracle_check_ip_header(arena[i * fl:].ctypes.data, fl, 14, 1, bad.ctypes.data, len(bad),
                                       good.ctypes.data, len(good)) for i in range(0, n, 997)]
        assert not any(ok)                      # a sample: every frame is the same
        ip = arena.reshape(n, fl)[:, 14:].copy().reshape(-1)
        if combo:
            port, _, _ = oracle_lib.ip_out_batch("ip_output_combo", ip, n, stride=fl - 14, fixed_len=fl - 14,
                                                 my_ip=0x18041A12, mtu=300)
            assert not port.any()
        else:
            st, _, _ = oracle_lib.ip_out_batch("ip_gw_options", ip, n, stride=fl - 14, fixed_len=fl - 14,
                                               my_ip=0x18041A12, my_addrs=np.array([0x18041A12], np.uint32))
            assert not st.any()
            oracle_lib.ip_out_batch("fix_ip_src", ip, n, stride=fl - 14, fixed_len=fl - 14,
                                    flags=np.zeros(n, np.uint8), my_ip=0x18041A12)
            st, _ = oracle_lib.batch("dec_ttl", ip, n, stride=fl - 14, fixed_len=fl - 14)
            assert not st.any()
            r = oracle_lib.ip_fragment(ip, n, 300, True, stride=fl - 14, fixed_len=fl - 14)
            assert not r["port"].any() and not r["frags"]
        outs.append(ip)
    assert np.array_equal(outs[0], outs[1])
    assert int(outs[0].reshape(n, -1)[:, 8].astype(np.int64).sum()) == n * 63     # TTL 64 -> 63 on all 600000


@pytest.mark.parametrize("proto", [17, 6, 1])
def test_transport_annotation_restatement_at_ip_hl(proto):
    """oracle_check_l4_at / oracle_set_l4_at (the segment at the transport
    header annotation, as udp_header() / tcp_header() / icmp_header() read
    it) with the annotation at ip_hl are the element restatements above:
    same verdicts and, for the Set elements, the same bytes."""
    L = oracle_lib.load_oracle()
    rng = np.random.default_rng(40 + proto)
    arena, off, cap, _ = fuzz.make_batch(rng, 1200, proto, max_total=900)
    a2 = arena.copy()
    base, base2 = arena.ctypes.data, a2.ctypes.data
    check = {17: L.oracle_check_udp_header, 6: L.oracle_check_tcp_header, 1: L.oracle_check_icmp_header}[proto]
    for f in (check, L.oracle_set_udp_checksum, L.oracle_set_tcp_checksum):
        f.restype = ctypes.c_int
    for i in range(len(off)):
        o, c = int(off[i]), int(cap[i])
        hl = int(arena[o] & 15) * 4 if c else 0
        assert L.oracle_check_l4_at(proto, base + o, c, hl) == check(ctypes.c_void_p(base + o), c), i
        if proto == 17:
            assert L.oracle_set_l4_at(17, base + o, c, hl, 1, 0) == \
                L.oracle_set_udp_checksum(ctypes.c_void_p(base2 + o), c), i
        elif proto == 6:
            assert L.oracle_set_l4_at(6, base + o, c, hl, 1, i & 1) == \
                L.oracle_set_tcp_checksum(ctypes.c_void_p(base2 + o), c, i & 1), i
    assert np.array_equal(arena, a2)
