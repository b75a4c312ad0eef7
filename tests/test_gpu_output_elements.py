"""GPU tests of the output-path element glue (click_amd/host/elements.cc):
IPGWOptions, FixIPSrc, IPOutputCombo and IPFragmenter route, write back,
count and chatter as the reference elements (ipgwoptions.cc:161-172,
fixipsrc.cc:69-73, ipoutputcombo.cc:44-205, ipfragmenter.cc:88-171) on
host packets, each decided by the oracle; and the fake-iprouter forwarding
path run through the glue both as separate elements and as the click-xform
combos (test/userlevel/iprouter-01.clicktest)."""
import numpy as np
import pytest

from tests import fuzz, oracle_lib

pytestmark = pytest.mark.gpu

MY_IP = 0x18041A12          # 18.26.4.24
MY_IP_TXT = "18.26.4.24"


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def framed(arena3, off3, cap3, rng, eth=14):
    """The L3 packets behind an Ethernet header: (arena, foff, flen)."""
    n = len(off3)
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


def push_all(e, arena, foff, flen, nh=14, anno=None, batch_flush=None):
    base = arena.ctypes.data
    for i in range(len(foff)):
        a = int(anno[i]) if anno is not None else 0
        rc = e.lib.clk_element_push_anno(e.h, base + int(foff[i]), int(flen[i]), nh, a, i)
        assert rc >= 0
        if rc == 1 or (batch_flush and (i + 1) % batch_flush == 0):
            e.flush()
    e.flush()
    return e.results(aux=True)


@pytest.mark.parametrize("noutputs", [2, 1])
def test_ip_gw_options_element(ctx, noutputs):
    from click_amd.elements import Element
    rng = np.random.default_rng(40 + noutputs)
    a3, o3, c3, _ = fuzz.gw_batch(rng, 2000, MY_IP)
    arena, foff, flen = framed(a3, o3, c3, rng)
    ref = arena.copy()
    addrs = np.array([0x01020304, MY_IP], np.uint32)
    e = Element(ctx, "IPGWOptions", "%s, 4.3.2.1, BATCH 600" % MY_IP_TXT, noutputs=noutputs)
    tok, port, ln, aux = push_all(e, arena, foff, flen)
    assert np.array_equal(tok, np.arange(len(foff)))
    drops = 0
    for i in range(len(foff)):
        o = int(foff[i]) + 14
        c = int(flen[i]) - 14
        # routing does not depend on the Timestamp value ("now")
        codes, prob, _ = oracle_lib.ip_out_batch("ip_gw_options", ref[o:o + c].copy(), 1, fixed_len=c,
                                                 my_ip=MY_IP, my_addrs=addrs, ts=0)
        if codes[0] == 1:
            drops += 1
            assert port[i] == (1 if noutputs == 2 else -1) and aux[i] == prob[0], i
        else:
            assert port[i] == 0 and aux[i] == 0, i
    assert int(e.read_handler("drops")) == drops > 0


def test_ip_gw_options_bytes(ctx):
    """Written bytes equal the oracle's with the Timestamp value the element
    used (recovered from one TS flg-0 option it filled)."""
    from click_amd.elements import Element
    hdr = bytearray(60)
    hdr[0] = 0x4F
    hdr[2:4] = (60).to_bytes(2, "big")
    hdr[8], hdr[9] = 64, 17
    hdr[20:24] = bytes([68, 8, 5, 0])          # TS flg 0, room for one stamp
    rng = np.random.default_rng(3)
    a3, o3, c3, _ = fuzz.gw_batch(rng, 800, MY_IP)
    n = len(o3)
    cat = np.concatenate([np.frombuffer(bytes(hdr), np.uint8), a3])
    o3 = np.concatenate([[0], o3 + 60]).astype(np.uint64)
    c3 = np.concatenate([[60], c3]).astype(np.uint32)
    oracle_lib.batch("set_ip", cat, 1, off=o3[:1], length=c3[:1])
    arena, foff, flen = framed(cat, o3, c3, rng)
    ref = arena.copy()
    e = Element(ctx, "IPGWOptions", MY_IP_TXT, noutputs=2)
    push_all(e, arena, foff, flen)
    ts = int.from_bytes(arena[int(foff[0]) + 14 + 24:int(foff[0]) + 14 + 28].tobytes(), "little")
    for i in range(n + 1):
        o, c = int(foff[i]) + 14, int(flen[i]) - 14
        exp = ref[o:o + c].copy()
        oracle_lib.ip_out_batch("ip_gw_options", exp, 1, fixed_len=c, my_ip=MY_IP,
                                my_addrs=np.array([MY_IP], np.uint32), ts=ts)
        assert arena[o:o + c].tobytes() == exp.tobytes(), i


def test_fix_ip_src_element(ctx):
    from click_amd.elements import Element, ANNO_FIX_IP_SRC
    rng = np.random.default_rng(8)
    a3, o3, c3, flags = fuzz.gw_batch(rng, 1500, MY_IP)
    arena, foff, flen = framed(a3, o3, c3, rng)
    ref = arena.copy()
    e = Element(ctx, "FixIPSrc", "IPADDR " + MY_IP_TXT, noutputs=1)
    tok, port, ln, aux = push_all(e, arena, foff, flen, anno=flags * ANNO_FIX_IP_SRC)
    assert (port == 0).all()
    for i in range(len(foff)):
        o, c = int(foff[i]) + 14, int(flen[i]) - 14
        exp = ref[o:o + c].copy()
        oracle_lib.ip_out_batch("fix_ip_src", exp, 1, fixed_len=c, flags=flags[i:i + 1], my_ip=MY_IP)
        assert arena[o:o + c].tobytes() == exp.tobytes(), i


def test_ip_output_combo_element(ctx):
    """Ports 0-4 with the reference's order: broadcast killed, painted clone
    on 1 before the packet, parameter problem 2 (aux offset), TTL 3, MTU 4."""
    from click_amd.elements import Element, ANNO_BCAST, ANNO_FIX_IP_SRC, AUX_CLONE, anno_paint
    rng = np.random.default_rng(12)
    a3, o3, c3, flags = fuzz.gw_batch(rng, 2500, MY_IP)
    n = len(o3)
    arena, foff, flen = framed(a3, o3, c3, rng)
    ref = arena.copy()
    bcast = rng.random(n) < 0.05
    paint = rng.integers(0, 3, n)
    anno = flags * ANNO_FIX_IP_SRC + bcast * ANNO_BCAST + np.array([anno_paint(int(p)) for p in paint])
    mtu = 120
    e = Element(ctx, "IPOutputCombo", "2, %s, %d" % (MY_IP_TXT, mtu), noutputs=5)
    tok, port, ln, aux = push_all(e, arena, foff, flen, anno=anno, batch_flush=777)
    k = 0
    seen = set()
    for i in range(n):
        o, c = int(foff[i]) + 14, int(flen[i]) - 14
        if bcast[i]:
            assert (tok[k], port[k]) == (i, -1)
            k += 1
            continue
        if paint[i] == 2:
            assert (tok[k], port[k], aux[k]) == (i, 1, AUX_CLONE)
            k += 1
        exp = ref[o:o + c].copy()                 # routing does not depend on the Timestamp value
        pc, prob, _ = oracle_lib.ip_out_batch("ip_output_combo", exp, 1, fixed_len=c, flags=flags[i:i + 1],
                                              my_ip=MY_IP, mtu=0xFFFFFFFF, ts=0)
        want = int(pc[0])
        if want == 0 and flen[i] > mtu:
            want = 4
        assert (tok[k], port[k]) == (i, want), (i, port[k], want)
        if want == 2:
            assert aux[k] == prob[0]
        seen.add(want)
        k += 1
    assert k == len(tok)
    assert seen == {0, 2, 3, 4}


def test_ip_fragmenter_element(ctx):
    from click_amd.elements import Element
    rng = np.random.default_rng(21)
    a3, o3, c3 = fuzz.frag_batch(rng, 1200, max_total=2000)
    arena, foff, flen = framed(a3, o3, c3, rng)
    ref = a3.copy()
    r = oracle_lib.ip_fragment(ref, len(o3), 576, True, off=o3, length=c3)
    e = Element(ctx, "IPFragmenter", "576, true, BATCH 500", noutputs=2)
    tok, port, ln, aux = push_all(e, arena, foff, flen)
    k = 0
    nfr = ndrop = 0
    for i in range(len(o3)):
        o = int(foff[i]) + 14
        if r["port"][i] == 1:
            assert (tok[k], port[k]) == (i, 1)
            ndrop += 1
            k += 1
            continue
        if r["port"][i] == 0:
            assert (tok[k], port[k], ln[k]) == (i, 0, flen[i])
            k += 1
            continue
        first = int(r["first_len"][i])
        assert (tok[k], port[k], ln[k], aux[k]) == (i, 0, 14 + first, 0), i
        assert arena[o:o + first].tobytes() == ref[int(o3[i]):int(o3[i]) + first].tobytes(), i
        k += 1
        nfr += 1
        k0 = int(r["frag_first"][i])
        while k < len(tok) and tok[k] == i:
            b = e.take_packet(int(aux[k]))
            assert b == r["frags"][k0], (i, k0)
            assert ln[k] == len(b)
            k0 += 1
            k += 1
            nfr += 1
    assert k == len(tok)
    assert int(e.read_handler("drops")) == ndrop > 0
    assert int(e.read_handler("fragments")) == nfr > 0
    msgs = e.messages()
    assert len(msgs) == min(ndrop, 5) and msgs[0].startswith("IPFragmenter(576) DF ")


def test_fake_iprouter_through_the_glue(ctx):
    """iprouter-01: the forwarding path of conf/fake-iprouter.click through
    the element glue, once as Strip(14) + CheckIPHeader(INTERFACES ...) ->
    IPGWOptions -> FixIPSrc -> DecIPTTL -> IPFragmenter(300) and once as
    IPInputCombo(2, ...) -> IPOutputCombo(1, 18.26.4.24, 300) (xform-ip-01:282,285;
    painted 2, not redirected by the colour-1 PaintTee): all 60,000 frames
    forwarded on port 0, identical bytes both ways."""
    import json
    import os
    from click_amd.elements import Element
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")))["vectors"]
    l3 = bytes.fromhex([v for v in g if v["name"] == "fake-iprouter-ip-check"][0]["l3"])
    frame = bytes.fromhex("0000c0ae67ef0000000000000800") + l3
    n = 60000
    outs = []
    for combo in (False, True):
        arena = np.tile(np.frombuffer(frame, np.uint8), n).copy()
        foff = np.arange(n, dtype=np.uint64) * len(frame)
        flen = np.full(n, len(frame), np.uint32)
        chain = ([("IPInputCombo", "2, INTERFACES 18.26.4.1/24 18.26.7.1/24", 1, 14),
                  ("IPOutputCombo", "1, 18.26.4.24, 300", 5, 14)] if combo else
                 [("CheckIPHeader", "INTERFACES 18.26.4.1/24 18.26.7.1/24, OFFSET 14", 2, 14),
                  ("IPGWOptions", "18.26.4.24", 2, 14), ("FixIPSrc", "18.26.4.24", 1, 14),
                  ("DecIPTTL", "", 2, 14), ("IPFragmenter", "300", 2, 14)])
        for cls, conf, nout, nh in chain:
            e = Element(ctx, cls, ", ".join(x for x in (conf, "BATCH 65536") if x), noutputs=nout)
            tok, port, ln, aux = push_all(e, arena, foff, flen, nh=nh)
            assert (port == 0).all() and (tok == np.arange(n)).all(), cls
            e.close()
        outs.append(arena)
    assert np.array_equal(outs[0], outs[1])
    ref = np.frombuffer(frame, np.uint8).copy()
    oracle_lib.batch("dec_ttl", ref[14:], 1, fixed_len=len(frame) - 14)
    assert np.array_equal(outs[1].reshape(n, -1), np.broadcast_to(ref, (n, len(frame))))
