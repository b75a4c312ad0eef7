"""GPU tests of the host element glue (click_amd/host/elements.cc): the
batched elements route, count, trim, write back and chatter exactly as the
reference elements would, packet by packet (the oracle decides each packet;
the routing rules are the reference's: checkipheader.cc:143-159,
setipchecksum.cc:88-93, setudpchecksum.cc:48-61, settcpchecksum.cc:71-74)."""
import ctypes

import numpy as np
import pytest

from tests import oracle_lib, fuzz

pytestmark = pytest.mark.gpu

IP_REASONS = ["tiny packet", "bad IP version", "bad IP header length", "bad IP length", "bad IP checksum",
              "bad source address"]
UDP_REASONS = ["not UDP", "bad packet length", "bad UDP checksum"]
TCP_REASONS = ["not TCP", "bad packet length", "bad TCP checksum"]


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def frames(rng, n, proto, max_total=1600, eth=14):
    """Ethernet-framed fuzzed packets in one arena: frame i at foff[i],
    flen[i] bytes, L3 at foff[i] + eth."""
    arena3, off3, cap3, _ = fuzz.make_batch(rng, n, proto, max_total=max_total)
    flen = (cap3 + eth).astype(np.uint32)
    foff = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 8)) * 2
        foff[i] = pos
        pos += int(flen[i]) + 4
    arena = np.zeros(pos + 64, np.uint8)
    for i in range(n):
        o = int(foff[i])
        arena[o:o + eth] = rng.integers(0, 256, eth, dtype=np.uint8)
        arena[o + eth:o + flen[i]] = arena3[int(off3[i]):int(off3[i]) + int(cap3[i])]
    return arena, foff, flen


def run_element(ctx, cls, config, arena, foff, flen, nh, noutputs, batch=None):
    from click_amd.elements import Element
    conf = ", ".join(c for c in (config, ("BATCH %d" % batch) if batch else "") if c)
    e = Element(ctx, cls, conf, name="e0", noutputs=noutputs)
    base = arena.ctypes.data
    for i in range(len(foff)):
        full = e.push_ptr(base + int(foff[i]), int(flen[i]), nh, token=i)
        if full:
            e.flush()
    e.flush()
    tok, port, ln = e.results()
    assert np.array_equal(tok, np.arange(len(foff))), "results out of push order"
    return e, port, ln


def expected_drop_messages(name_prefix, codes, reasons, verbose):
    msgs = []
    drops = 0
    for c in codes:
        if c:
            if drops == 0 or verbose:
                msgs.append(name_prefix + reasons[c - 1])
            drops += 1
    return msgs


@pytest.mark.parametrize("noutputs,verbose", [(2, False), (1, True)])
def test_check_ip_header_element(ctx, noutputs, verbose):
    rng = np.random.default_rng(100 + noutputs)
    arena, foff, flen = frames(rng, 2500, 17)
    e, port, ln = run_element(ctx, "CheckIPHeader", "OFFSET 14, DETAILS true, VERBOSE %s" % str(verbose).lower(),
                              arena, foff, flen, -1, noutputs, batch=700)
    L = oracle_lib.load_oracle()
    codes = np.array([L.oracle_check_ip_header(arena.ctypes.data + int(foff[i]), int(flen[i]), 14, 1,
                                               None, 0, None, 0) for i in range(len(foff))])
    exp_port = np.where(codes == 0, 0, 1 if noutputs == 2 else -1)
    assert np.array_equal(port, exp_port)
    for i in np.nonzero(codes == 0)[0]:
        o = int(foff[i])
        ip_len = (int(arena[o + 16]) << 8) | int(arena[o + 17])
        assert ln[i] == min(int(flen[i]), 14 + ip_len)
    assert e.read_handler("drops") == str(int((codes != 0).sum()))
    det = e.read_handler("drop_details").splitlines()
    assert det == ["%d\t%s" % (int((codes == k + 1).sum()), IP_REASONS[k]) for k in range(6)]
    assert e.messages() == expected_drop_messages("e0: IP header check failed: ", codes, IP_REASONS, verbose)
    assert int(e.read_handler("packets")) == len(foff) and int(e.read_handler("batches")) >= 4


def test_check_ip_header_interfaces(ctx):
    """INTERFACES 18.26.4.1/24 (checkipheader.cc:51-74): broadcast and 0/255
    sources are bad unless the destination is one of the interfaces."""
    from click_amd.elements import Element
    rng = np.random.default_rng(5)
    n = 400
    arena = np.zeros(n * 64, np.uint8)
    oracle_lib.gen(arena, n, stride=64, fixed_len=40, proto=17)
    srcs = [b"\x12\x1a\x04\xff", b"\x00\x00\x00\x00", b"\xff\xff\xff\xff", b"\x0a\x00\x00\x01"]
    dsts = [b"\x12\x1a\x04\x01", b"\x12\x1a\x07\x01", b"\x0a\x00\x00\x02"]
    for i in range(n):
        arena[i * 64 + 12:i * 64 + 16] = np.frombuffer(srcs[rng.integers(0, 4)], np.uint8)
        arena[i * 64 + 16:i * 64 + 20] = np.frombuffer(dsts[rng.integers(0, 3)], np.uint8)
    oracle_lib.batch("set_ip", arena, n, stride=64, fixed_len=40)
    e = Element(ctx, "CheckIPHeader", "INTERFACES 18.26.4.1/24 18.26.7.1/24", noutputs=2)
    for i in range(n):
        e.push_ptr(arena.ctypes.data + i * 64, 40, -1, i)
    e.flush()
    _, port, _ = e.results()
    bad = [bytes(arena[i * 64 + 12:i * 64 + 16]) in srcs[:3] and
           bytes(arena[i * 64 + 16:i * 64 + 20]) not in dsts[:2] for i in range(n)]
    assert np.array_equal(port, np.where(bad, 1, 0))
    assert sum(bad) > 0


def test_set_ip_checksum_element(ctx):
    rng = np.random.default_rng(7)
    arena, foff, flen = frames(rng, 2000, 6)
    ref = arena.copy()
    e, port, ln = run_element(ctx, "SetIPChecksum", "", arena, foff, flen, 14, 1)
    codes, _ = oracle_lib.batch("set_ip", ref, len(foff), off=foff + 14, length=flen - 14)
    assert np.array_equal(port, np.where(codes == 0, 0, -1))
    assert np.array_equal(arena, ref)
    assert e.read_handler("drops") == str(int((codes != 0).sum()))
    assert e.messages() == (["SetIPChecksum: bad input packet"] if (codes != 0).any() else [])


@pytest.mark.parametrize("proto", [17, 6])
@pytest.mark.parametrize("noutputs", [1, 2])
def test_check_l4_element(ctx, proto, noutputs):
    rng = np.random.default_rng(proto + 10 * noutputs)
    arena, foff, flen = frames(rng, 2500, proto)
    cls = "CheckUDPHeader" if proto == 17 else "CheckTCPHeader"
    e, port, ln = run_element(ctx, cls, "DETAILS true", arena, foff, flen, 14, noutputs, batch=1000)
    codes, _ = oracle_lib.batch("check_udp" if proto == 17 else "check_tcp", arena.copy(), len(foff),
                                off=foff + 14, length=flen - 14)
    assert np.array_equal(port, np.where(codes == 0, 0, 1 if noutputs == 2 else -1))
    assert np.array_equal(ln, flen)
    reasons = UDP_REASONS if proto == 17 else TCP_REASONS
    det = e.read_handler("drop_details").splitlines()
    assert det == ["%d\t%s" % (int((codes == k + 1).sum()), reasons[k]) for k in range(3)]
    prefix = "UDP header check failed: " if proto == 17 else "e0 :: CheckTCPHeader: TCP header check failed: "
    assert e.messages() == expected_drop_messages(prefix, codes, reasons, False)


@pytest.mark.parametrize("hold", [False, True])
def test_push_copies_unless_held(ctx, hold):
    """clk_element_push copies what the kernel reads at the push:
    a caller may reuse its receive buffer at once, and the verdicts are the
    packets' as pushed.  With clk_element_hold_packets the long spans are
    gathered at the flush, so a buffer overwritten before it is what is
    checked -- the caller's side of that contract (the adapter holds its
    Packets)."""
    from click_amd.elements import Element
    rng = np.random.default_rng(77)
    arena, foff, flen = frames(rng, 600, 17, max_total=1600)
    codes, _ = oracle_lib.batch("check_udp", arena.copy(), len(foff), off=foff + 14, length=flen - 14)
    e = Element(ctx, "CheckUDPHeader", "BATCH 4096", noutputs=2)
    if hold:
        e.hold_packets()
    base = arena.ctypes.data
    for i in range(len(foff)):
        e.push_ptr(base + int(foff[i]), int(flen[i]), 14, token=i)
    hl = [int(arena[int(o) + 14] & 15) * 4 for o in foff]
    usum = [int(arena[int(foff[i]) + 14 + hl[i] + 6]) | int(arena[int(foff[i]) + 14 + hl[i] + 7]) << 8
            if int(flen[i]) - 14 >= hl[i] + 8 else 0 for i in range(len(foff))]
    long_ = [i for i in range(len(foff)) if int(flen[i]) - 14 - hl[i] >= 300 and codes[i] == 0 and usum[i]]
    assert len(long_) > 50
    for i in long_:                                  # the receive buffer reused before the flush
        o = int(foff[i]) + 14 + hl[i] + 8            # UDP payload bytes
        arena[o:o + 200] ^= 0x5A
    e.flush()
    tok, port, _ = e.results()
    assert np.array_equal(tok, np.arange(len(foff)))
    if not hold:
        assert np.array_equal(port, np.where(codes == 0, 0, 1))
    else:
        assert all(port[i] == 1 for i in long_)      # the overwritten bytes were read at the flush
    e.close()


@pytest.mark.parametrize("proto,config,noutputs", [(17, "", 1), (17, "", 2), (6, "", 1), (6, "FIXOFF true", 1),
                                                   (6, "true", 1)])
def test_set_l4_element(ctx, proto, config, noutputs):
    rng = np.random.default_rng(proto * 3 + noutputs + len(config))
    arena, foff, flen = frames(rng, 2500, proto)
    ref = arena.copy()
    cls = "SetUDPChecksum" if proto == 17 else "SetTCPChecksum"
    e, port, ln = run_element(ctx, cls, config, arena, foff, flen, 14, noutputs)
    fix = 1 if "true" in config else 0
    codes, _ = oracle_lib.batch("set_udp" if proto == 17 else "set_tcp", ref, len(foff), off=foff + 14,
                                length=flen - 14, arg=fix)
    if proto == 17:
        exp = np.where(codes == 0, 0, 1 if noutputs == 2 else -1)
    else:
        exp = np.where(codes == 0, 0, -1)
    assert np.array_equal(port, exp)
    assert np.array_equal(arena, ref)
    m = e.messages()
    if proto == 17:
        assert m == (["e0 :: SetUDPChecksum: fragment or short packet"] if noutputs == 1 and (codes != 0).any()
                     else [])
    else:
        assert m == ["SetTCPChecksum: bad lengths"] * int((codes != 0).sum())


def test_no_network_header(ctx):
    """Without a network header CheckUDPHeader drops NOT_UDP
    (checkudpheader.cc:91-92) and SetTCPChecksum kills (settcpchecksum.cc:53)."""
    from click_amd.elements import Element
    buf = np.zeros(100, np.uint8)
    e = Element(ctx, "CheckUDPHeader", "DETAILS true", noutputs=2)
    e.push(buf, nh_offset=-1, token=3)
    e.flush()
    t, p, _ = e.results()
    assert list(t) == [3] and list(p) == [1]
    assert e.read_handler("drop_details").splitlines()[0] == "1\tnot UDP"
    e2 = Element(ctx, "SetTCPChecksum", "", noutputs=1)
    e2.push(buf, nh_offset=-1, token=4)
    e2.flush()
    assert list(e2.results()[1]) == [-1]


def test_configure_errors(ctx):
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    for cls, conf in [("CheckIPHeader", "OFFSET x"), ("CheckIPHeader", "BOGUS 1"), ("CheckUDPHeader", "5"),
                      ("SetTCPChecksum", "FIXOFF maybe"), ("NoSuchElement", ""),
                      ("CheckIPHeader", "INTERFACES 1.2.3.4"), ("CheckUDPHeader", "VERBOSE True")]:
        with pytest.raises(ClickAmdError):
            Element(ctx, cls, conf)
    Element(ctx, "CheckIPHeader2", "14")
    Element(ctx, "CheckIPHeader", "CHECKSUM false, OFFSET 14, VERBOSE true")


ICMP_REASONS = ["not ICMP", "bad packet length", "bad ICMP checksum"]


@pytest.mark.parametrize("noutputs", [1, 2])
def test_check_icmp_element(ctx, noutputs):
    rng = np.random.default_rng(200 + noutputs)
    arena, foff, flen = frames(rng, 2500, 1, max_total=600)
    e, port, ln = run_element(ctx, "CheckICMPHeader", "DETAILS true", arena, foff, flen, 14, noutputs, batch=900)
    codes, _ = oracle_lib.batch("check_icmp", arena.copy(), len(foff), off=foff + 14, length=flen - 14)
    assert np.array_equal(port, np.where(codes == 0, 0, 1 if noutputs == 2 else -1))
    det = e.read_handler("drop_details").splitlines()
    assert det == ["%d\t%s" % (int((codes == k + 1).sum()), ICMP_REASONS[k]) for k in range(3)]
    assert e.messages() == expected_drop_messages("e0 :: CheckICMPHeader: ICMP header check failed: ", codes,
                                                  ICMP_REASONS, False)
    assert (codes == 0).any() and (codes == 3).any()


@pytest.mark.parametrize("config,noutputs", [("", 2), ("", 1), ("MULTICAST false", 2), ("ACTIVE false", 2)])
def test_dec_ip_ttl_element(ctx, config, noutputs):
    """DecIPTTL (decipttl.cc:45-77): TTL and ip_sum rewritten in the host
    packets exactly as the oracle does; expired packets to output 1 (or
    killed); ACTIVE false passes everything untouched."""
    rng = np.random.default_rng(300 + noutputs + len(config))
    arena, foff, flen = frames(rng, 2000, 17, max_total=300)
    fuzz.vary_ttl(rng, arena, foff + 14, flen - 14, frac=0.5)
    ref = arena.copy()
    e, port, ln = run_element(ctx, "DecIPTTL", config, arena, foff, flen, 14, noutputs, batch=700)
    if "ACTIVE false" in config:
        assert np.array_equal(arena, ref) and (port == 0).all()
        assert e.read_handler("active") == "false"
        return
    mc = 0 if "MULTICAST false" in config else 1
    codes, _ = oracle_lib.batch("dec_ttl", ref, len(foff), off=foff + 14, length=flen - 14, arg=mc)
    assert np.array_equal(arena, ref)
    assert np.array_equal(port, np.where(codes == 1, 1 if noutputs == 2 else -1, 0))
    assert e.read_handler("drops") == str(int((codes == 1).sum()))
    assert (codes == 0).any() and (codes == 1).any() and (codes == 2).any()


def test_ip_input_combo_element(ctx):
    """IPInputCombo (ipinputcombo.cc:66-140) = Paint + Strip(14) +
    CheckIPHeader: bad packets are killed, the first chatters once; good
    ones leave with their length after the strip and the ip_len trim."""
    rng = np.random.default_rng(400)
    arena, foff, flen = frames(rng, 2500, 17)
    e, port, ln = run_element(ctx, "IPInputCombo", "3, INTERFACES 10.0.0.1/8", arena, foff, flen, -1, 1, batch=800)
    L = oracle_lib.load_oracle()
    bad = np.array([0xFFFFFFFF, 0, 0x0AFFFFFF], np.uint32)    # INTERFACES 10.0.0.1/8 (checkipheader.cc:51-74)
    bad_be = bad.byteswap()
    good = np.array([0x0A000001], np.uint32).byteswap()
    codes = np.array([L.oracle_check_ip_header(arena.ctypes.data + int(foff[i]), int(flen[i]), 14, 1,
                                               bad_be.ctypes.data, 3, good.ctypes.data, 1)
                      for i in range(len(foff))])
    assert np.array_equal(port, np.where(codes == 0, 0, -1))
    for i in np.nonzero(codes == 0)[0]:
        o = int(foff[i])
        ip_len = (int(arena[o + 16]) << 8) | int(arena[o + 17])
        assert ln[i] == min(int(flen[i]) - 14, ip_len)
    assert e.read_handler("drops") == str(int((codes != 0).sum()))
    assert e.read_handler("color") == "3"
    assert e.messages() == (["IP checksum failed"] if (codes != 0).any() else [])


def test_new_element_configure_errors(ctx):
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    for cls, conf in [("IPInputCombo", ""), ("IPInputCombo", "x"), ("DecIPTTL", "ACTIVE maybe"),
                      ("DecIPTTL", "3"), ("CheckICMPHeader", "VERBOSE 2")]:
        with pytest.raises(ClickAmdError):
            Element(ctx, cls, conf)
    Element(ctx, "IPInputCombo", "COLOR 1, 18.26.4.255 18.26.7.255")
    Element(ctx, "DecIPTTL", "MULTICAST false, ACTIVE true")


@pytest.mark.parametrize("cls,config,noutputs,reasons,prefix", [
    ("CheckIPHeader", "OFFSET 14", 2, IP_REASONS, "e0: IP header check failed: "),
    ("SetUDPChecksum", "", 1, None, "e0 :: SetUDPChecksum: fragment or short packet")])
def test_shared_messages_speak_once(ctx, cls, config, noutputs, reasons, prefix):
    """Two glue elements standing for one reference element (the Click
    adapter's per-thread elements) share their once-only chatter
    (clk_element_share_messages): the first drop's reason, or
    SetUDPChecksum's fragment warning (once per router,
    setudpchecksum.cc:52-58), is said once over both -- by whichever element
    meets it first -- and each keeps its own drop counter."""
    from click_amd.elements import Element
    rng = np.random.default_rng(7)
    arena, foff, flen = frames(rng, 1200, 17)
    half = len(foff) // 2
    a = Element(ctx, cls, config, name="e0", noutputs=noutputs)
    b = Element(ctx, cls, config, name="e0", noutputs=noutputs).share_messages(a)
    base = arena.ctypes.data
    nh = -1 if cls == "CheckIPHeader" else 14
    ref = arena.copy()
    for e, rng_ in ((a, range(half)), (b, range(half, len(foff)))):
        for i in rng_:
            e.push_ptr(base + int(foff[i]), int(flen[i]), nh, token=i)
        e.flush()
        e.results()
    msgs = a.messages() + b.messages()
    if cls == "CheckIPHeader":
        L = oracle_lib.load_oracle()
        rb = ref.ctypes.data
        codes = np.array([L.oracle_check_ip_header(rb + int(foff[i]), int(flen[i]), 14, 1, None, 0, None, 0)
                          for i in range(len(foff))])
        assert (codes[:half] != 0).any() and (codes[half:] != 0).any()
        assert msgs == expected_drop_messages(prefix, codes, reasons, False)
        assert int(a.read_handler("drops")) + int(b.read_handler("drops")) == int((codes != 0).sum())
    else:
        codes, _ = oracle_lib.batch("set_udp", ref, len(foff), off=foff + 14, length=flen - 14, arg=0)
        assert (codes[:half] != 0).any() and (codes[half:] != 0).any()
        assert msgs == [prefix]


@pytest.mark.parametrize("cls,conf,proto,noutputs", [
    ("CheckUDPHeader", "", 17, 2), ("CheckTCPHeader", "", 6, 2), ("CheckICMPHeader", "", 1, 2),
    ("SetUDPChecksum", "", 17, 2), ("SetTCPChecksum", "", 6, 1), ("SetTCPChecksum", "FIXOFF true", 6, 1)])
def test_transport_header_annotation(ctx, cls, conf, proto, noutputs):
    """The L4 elements read the segment at the transport header annotation
    (udp_header() / tcp_header() / icmp_header(), checkudpheader.cc:87,
    setudpchecksum.cc:45, checktcpheader.cc:88, settcpchecksum.cc:49,
    checkicmpheader.cc:85) and ip_hl from the header bytes.  Packets pushed
    with clk_element_push_th: a third at ip_hl (the kernels' path), a third
    with ip_hl rewritten after marking (a corrupted header: RandomBitErrors
    in a graph), a third at an arbitrary offset; verdicts and every byte
    against the oracle's annotation-aware restatement."""
    from click_amd.elements import Element
    L = oracle_lib.load_oracle()
    rng = np.random.default_rng(300 + proto + len(conf))
    arena, off3, cap3, _ = fuzz.make_batch(rng, 1500, proto, max_total=1200, mutate_frac=0.2)
    n = len(off3)
    th = np.zeros(n, np.int64)
    for i in range(n):
        o, c = int(off3[i]), int(cap3[i])
        hl = int(arena[o] & 15) * 4 if c else 20
        k = i % 3
        if k == 0 or c < 20:
            th[i] = hl
        elif k == 1:
            th[i] = hl
            arena[o] = (arena[o] & 0xF0) | int(rng.choice([4, 6, 7, 9, 15, 2]))
        else:
            th[i] = int(rng.integers(0, min(c, 80) + 1))
    ref = arena.copy()
    set_ = cls.startswith("Set")
    fix = 1 if "FIXOFF" in conf else 0
    codes = []
    for i in range(n):
        o, c = int(off3[i]), int(cap3[i])
        nh = ref.ctypes.data + o
        if set_:
            codes.append(L.oracle_set_l4_at(proto, nh, c, int(th[i]), 1, fix))
        else:
            codes.append(L.oracle_check_l4_at(proto, nh, c, int(th[i])))
    codes = np.array(codes)
    e = Element(ctx, cls, ", ".join(x for x in (conf, "BATCH 700") if x), noutputs=noutputs)
    base = arena.ctypes.data
    for i in range(n):
        rc = e.push_th(base + int(off3[i]), int(cap3[i]), 0, int(th[i]), token=i)
        assert rc >= 0, e.last_error()
        if rc == 1:
            e.flush()
    e.flush()
    tok, port, _ = e.results()
    assert np.array_equal(tok, np.arange(n))
    if set_:
        from click_amd import _abi
        exp = np.where(codes == 0, 0, np.where(codes == _abi.CLK_SET_OUTPUT1, 1 if noutputs == 2 else -1, -1))
    else:
        exp = np.where(codes == 0, 0, 1 if noutputs == 2 else -1)
    bad = np.nonzero(port != exp)[0]
    assert len(bad) == 0, [(int(i), int(codes[i]), int(port[i]), int(th[i]), int(cap3[i])) for i in bad[:8]]
    if set_:
        diff = np.nonzero(arena != ref)[0]
        assert len(diff) == 0, diff[:10]
    kinds = {(i % 3, int(codes[i] == 0)) for i in range(n)}
    assert (1, 1) in kinds and (2, 1) in kinds and (1, 0) in kinds, kinds
    e.close()


def test_transport_header_annotation_zerocopy_refused(ctx):
    """ZEROCOPY reads packets in place: a packet whose annotation is not at
    ip_hl cannot be, and the push is refused (clk_element_push_th)."""
    import ctypes as ct
    from click_amd.elements import Element
    pkt = np.zeros(64, np.uint8)
    oracle_lib.gen(pkt, 1, stride=64, fixed_len=60, proto=17)
    pkt[0] = 0x44                                    # ip_hl 4 written after the header was marked at 20
    e = Element(ctx, "CheckUDPHeader", "ZEROCOPY true", noutputs=2)
    assert e.push_th(pkt.ctypes.data, 60, 0, 20, token=0) < 0
    assert "annotation" in e.last_error()
    e.close()
