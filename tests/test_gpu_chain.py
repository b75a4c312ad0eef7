"""GPU tests of element chains (clk_chain_*, click_amd/host/chain.cc):
consecutive elements on one staged, device-resident batch must route,
rewrite and count exactly as the same elements run one after another (which
tests/test_gpu_elements.py and test_gpu_output_elements.py pin to the
oracle): the fake-iprouter forwarding path as separate elements and as the
click-xform combos (iprouter-01), fuzzed frames with every drop reason, IP
options, expiring TTLs, fragments, broadcast / painted annotations, a
check-then-set pair over whole payloads, a failed flush resumed (or its
packets killed after a rewriting member's kernel ran), and the chains the
ABI refuses."""
import ctypes

import numpy as np
import pytest

from tests import fuzz, oracle_lib

pytestmark = pytest.mark.gpu

MY_IP_TXT = "18.26.4.24"
MY_IP = 0x18041A12


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def framed(rng, a3, o3, c3, eth=14):
    n = len(o3)
    flen = (c3 + eth).astype(np.uint32)
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
        arena[o + eth:o + int(flen[i])] = a3[int(o3[i]):int(o3[i]) + int(c3[i])]
    return arena, foff, flen


def make(ctx, spec):
    from click_amd.elements import Element
    return [Element(ctx, cls, conf, name="m%d" % k, noutputs=nout) for k, (cls, conf, nout) in enumerate(spec)]


def run_separate(ctx, spec, arena, foff, flen, nh0, anno):
    """The members one after another, each flushed over what the one before
    passed on output 0 (views as the Click adapters leave them: CheckIPHeader
    sets the network header at OFFSET, IPInputCombo strips 14 bytes).
    Returns the results in the chain's order and the elements."""
    from click_amd.elements import AUX_CLONE, ANNO_BCAST
    els = make(ctx, spec)
    base = arena.ctypes.data
    n = len(foff)
    ptr = [base + int(foff[i]) for i in range(n)]
    ln = [int(flen[i]) for i in range(n)]
    nh = [nh0] * n
    anno = [int(a) for a in anno]
    out = []                                    # member-major: each member's results in its own order
    alive = list(range(n))
    clones = {}                                 # (member, token): the bytes as they reached the member
    for k, e in enumerate(els):
        if spec[k][0] == "IPOutputCombo" and k > 0:
            color = int(spec[k][1].split(",")[0])
            for i in alive:
                if not anno[i] & ANNO_BCAST and (anno[i] >> 8) & 0xFF == color and spec[k][2] >= 2:
                    o = ptr[i] - base
                    clones[(k, i)] = bytes(arena[o:o + ln[i]])
        for i in alive:
            rc = e.lib.clk_element_push_anno(e.h, ctypes.c_void_p(ptr[i]), ln[i], nh[i], anno[i], i)
            assert rc >= 0
            if rc == 1:
                e.flush()
        e.flush()
        tok, port, length, aux = e.results(aux=True)
        cls = spec[k][0]
        passed = set()
        nxt = []
        seen = set()
        for t, p, l_, a in zip(tok.tolist(), port.tolist(), length.tolist(), aux.tolist()):
            primary = t not in seen and not (cls == "IPOutputCombo" and a == AUX_CLONE)
            if primary:
                seen.add(t)
            if primary and p == 0 and k + 1 < len(els):
                passed.add(t)
                if cls in ("CheckIPHeader", "CheckIPHeader2"):
                    nh[t] = int(e.read_handler("offset"))
                if cls == "IPInputCombo":
                    ptr[t] += 14
                    nh[t] = 0
                    color = int(spec[k][1].split(",")[0])
                    anno[t] = (anno[t] & ~0xFF00) | ((color & 0xFF) << 8)    # Paint(COLOR)
                if cls == "FixIPSrc" and anno[t] & 1 and 0 <= nh[t] < ln[t]:
                    anno[t] &= ~1                                           # the fixed source clears FIX_IP_SRC
                ln[t] = l_
                nxt.append(t)
                continue
            out.append((t, k, p, l_, a))
        alive = nxt
    run_separate.clones = clones
    return out, els


def run_chain(ctx, spec, arena, foff, flen, nh0, anno, batch_flush=None, async_flush=False, flush_after=None):
    """The chain over the frames; a full batch (or every batch_flush
    packets) flushed with clk_chain_flush, or double-buffered with
    clk_chain_flush_async (async_flush), then everything flushed.
    flush_after: {i: "sync" | "async"} -- a flush of that kind after packet
    i as well (a partial batch: the adapter's deadline or stop)."""
    from click_amd.elements import Chain
    els = make(ctx, spec)
    ch = Chain(els)
    base = arena.ctypes.data
    flush_after = flush_after or {}
    for i in range(len(foff)):
        if ch.push_anno(base + int(foff[i]), int(flen[i]), nh0, int(anno[i]), i) or \
                (batch_flush and (i + 1) % batch_flush == 0):
            ch.flush_async() if async_flush else ch.flush()
        if i in flush_after:
            ch.flush_async() if flush_after[i] == "async" else ch.flush()
    ch.flush()
    tok, mem, port, length, aux = ch.results()
    return list(zip(tok.tolist(), mem.tolist(), port.tolist(), length.tolist(), aux.tolist())), els, ch


def compare_chain(ctx, spec, arena, foff, flen, nh0=-1, anno=None, batch_flush=None,
                  handlers=("drops", "fragments", "packets", "lost"), async_flush=False, flush_after=None):
    from click_amd.elements import AUX_CLONE
    anno = np.zeros(len(foff), np.uint32) if anno is None else anno
    a1, a2 = arena.copy(), arena.copy()
    r1, e1 = run_separate(ctx, spec, a1, foff, flen, nh0, anno)
    r2, e2, ch = run_chain(ctx, spec, a2, foff, flen, nh0, anno, batch_flush, async_flush, flush_after)
    assert len(r1) == len(r2)
    # each member's results in its own (push) order, as the elements one by
    # one give them (a chain flush interleaves members batch by batch)
    for k in range(len(spec)):
        x1 = [x for x in r1 if x[1] == k]
        x2 = [y for y in r2 if y[1] == k]
        assert len(x1) == len(x2), (spec[k][0], len(x1), len(x2))
        for x, y in zip(x1, x2):
            if x[:4] != y[:4]:
                raise AssertionError(("first difference", x, y))
    assert np.array_equal(a1, a2), np.nonzero(a1 != a2)[0][:10]
    clones = run_separate.clones
    for k in range(len(spec)):                  # new packets (fragments, clones), byte for byte
        for x, y in zip([x for x in r1 if x[1] == k], [y for y in r2 if y[1] == k]):
            if spec[k][0] == "IPFragmenter" and x[4] != 0:
                assert e1[k].take_packet(x[4]) == e2[k].take_packet(y[4])
            if spec[k][0] == "IPOutputCombo" and k > 0 and x[4] == AUX_CLONE and x[2] == 1:
                # a member after the head: its PaintTee clone carries the
                # bytes as they reached it (clk_element_take_packet)
                assert y[4] & AUX_CLONE and y[4] != AUX_CLONE, y
                assert e2[k].take_packet(y[4] & ~AUX_CLONE) == clones[(k, y[0])]
        for h in handlers:
            assert e1[k].read_handler(h) == e2[k].read_handler(h), (spec[k][0], h)
        assert e1[k].messages() == e2[k].messages(), spec[k][0]
    ch.close()
    for e in e1 + e2:
        e.close()
    return r2


# fake-iprouter.click's forwarding path (bench.py C1_CHAINS)
FAKE_IPROUTER = [("CheckIPHeader", "INTERFACES 18.26.4.1/24 18.26.7.1/24, OFFSET 14", 2),
                 ("IPGWOptions", MY_IP_TXT, 2), ("FixIPSrc", MY_IP_TXT, 1), ("DecIPTTL", "", 2),
                 ("IPFragmenter", "300", 2)]
COMBOS = [("IPInputCombo", "2, INTERFACES 18.26.4.1/24 18.26.7.1/24", 1),
          ("IPOutputCombo", "1, %s, 300" % MY_IP_TXT, 5)]


def no_timestamps(arena, off, caplen):
    """Timestamp options become Record Route ones: the TS value is the
    wall clock at the flush (Timestamp::now(), ipgwoptions.cc:118-119), which
    two runs cannot share; everything else about the option walk stays."""
    for i in range(len(off)):
        o, c = int(off[i]), int(caplen[i])
        if c < 20:
            continue
        hl = int(arena[o] & 0xF) * 4
        k = o + 20
        while k < o + min(hl, c):
            t = int(arena[k])
            if t == 0:
                break
            if t == 1:
                k += 1
                continue
            if k + 1 >= o + min(hl, c) or arena[k + 1] < 2:
                break
            if t == 68:
                arena[k] = 7
            k += int(arena[k + 1])
        if hl <= c:
            oracle_lib.batch("set_ip", arena[o:o + c], 1, fixed_len=c)


def fake_frames(n):
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")))["vectors"]
    l3 = bytes.fromhex([v for v in g if v["name"] == "fake-iprouter-ip-check"][0]["l3"])
    frame = np.frombuffer(bytes.fromhex("0000c0ae67ef0000000000000800") + l3, np.uint8)
    arena = np.tile(frame, n)
    return arena, np.arange(n, dtype=np.uint64) * len(frame), np.full(n, len(frame), np.uint32)


@pytest.mark.parametrize("spec", [FAKE_IPROUTER, COMBOS], ids=["elements", "combos"])
def test_fake_iprouter_chain(ctx, spec):
    """iprouter-01's frames: every one forwarded on the last member's output
    0, the same bytes as the elements one by one."""
    arena, foff, flen = fake_frames(20000)
    r = compare_chain(ctx, spec, arena, foff, flen)
    assert all(m == len(spec) - 1 and p == 0 for _, m, p, _, _ in r)


def fuzzed_frames(seed, n=3000):
    rng = np.random.default_rng(seed)
    a3, o3, c3, _ = fuzz.gw_batch(rng, n, MY_IP)
    no_timestamps(a3, o3, c3)
    arena, foff, flen = framed(rng, a3, o3, c3)
    for i in range(0, n, 7):                    # TTLs 0-2: expired on DecIPTTL / IPOutputCombo
        o = int(foff[i]) + 14
        arena[o + 8] = i % 3
        oracle_lib.batch("set_ip", arena[o:o + int(flen[i]) - 14], 1, fixed_len=int(flen[i]) - 14)
    for i in range(3, n, 11):                   # a flipped bit: CheckIPHeader's output 1
        arena[int(foff[i]) + 14 + 12] ^= 0x02
    return rng, arena, foff, flen


@pytest.mark.parametrize("batch_flush", [None, 333])
def test_fuzzed_element_chain(ctx, batch_flush):
    rng, arena, foff, flen = fuzzed_frames(5 + (batch_flush or 0))
    anno = (rng.random(len(foff)) < 0.3).astype(np.uint32)        # FIX_IP_SRC on a third
    spec = [("CheckIPHeader", "OFFSET 14, DETAILS true", 2), ("IPGWOptions", MY_IP_TXT + ", BATCH 700", 2),
            ("FixIPSrc", MY_IP_TXT, 1), ("DecIPTTL", "", 2), ("IPFragmenter", "576, HONOR_DF true", 2)]
    r = compare_chain(ctx, spec, arena, foff, flen, anno=anno, batch_flush=batch_flush)
    seen = {(m, p) for _, m, p, _, _ in r}
    assert {(0, 1), (1, 1), (3, 1), (4, 0)} <= seen, seen


@pytest.mark.parametrize("which", ["elements", "combos"])
def test_chain_double_buffered(ctx, which):
    """clk_chain_flush_async: a full batch is launched while the one before
    it is finished, two batches in flight (BATCH 1000 and 777 on the head,
    so 6000 frames make 6-8 batches): every member's results in push
    order, bytes, clones and handlers as the elements one by one."""
    from click_amd.elements import ANNO_BCAST, anno_paint
    if which == "elements":
        rng, arena, foff, flen = fuzzed_frames(21, n=6000)
        anno = (rng.random(len(foff)) < 0.3).astype(np.uint32)
        spec = [("CheckIPHeader", "OFFSET 14, DETAILS true, BATCH 1000", 2), ("IPGWOptions", MY_IP_TXT, 2),
                ("FixIPSrc", MY_IP_TXT, 1), ("DecIPTTL", "", 2), ("IPFragmenter", "576, HONOR_DF true", 2)]
    else:
        rng, arena, foff, flen = fuzzed_frames(23, n=6000)
        n = len(foff)
        anno = np.array([anno_paint(int(p)) for p in rng.integers(0, 3, n)], np.uint32) + \
            (rng.random(n) < 0.05) * ANNO_BCAST + (rng.random(n) < 0.2).astype(np.uint32)
        spec = [("IPInputCombo", "1, BATCH 777", 1), ("IPOutputCombo", "1, %s, 120" % MY_IP_TXT, 5)]
    for async_flush in (False, True):
        compare_chain(ctx, spec, arena, foff, flen, anno=anno, async_flush=async_flush,
                      handlers=("drops", "packets", "lost"))


def test_chain_host_only_batch_behind_gpu_batch(ctx):
    """a batch decided wholly on the host (IPGWOptions
    without options, FixIPSrc without the annotation) ends inside the flush
    that starts it while the batch before it -- options, on the GPU -- is
    still in flight.  Its results must come out after that batch's, none
    lost.  Groups of fuzzed frames (options, annotations) and plain
    fake-iprouter frames alternate; full batches are flushed double-buffered,
    partial ones by a synchronous or a double-buffered flush (the adapter's
    stop and deadline)."""
    rng, a1, o1, l1 = fuzzed_frames(41, n=1500)
    a2, o2, l2 = fake_frames(1500)
    arena = np.concatenate([a1, a2])
    o2 = o2 + np.uint64(len(a1))
    groups = [(0, 0, 500, None), (1, 0, 300, "sync"), (0, 500, 1000, None), (1, 300, 500, "async"),
              (1, 500, 800, "async"), (0, 1000, 1500, None), (1, 800, 1500, "sync")]
    foff, flen, anno, flush_after = [], [], [], {}
    fix = (rng.random(1500) < 0.3).astype(np.uint32)
    for g, a, b, how in groups:
        foff += list((o1 if g == 0 else o2)[a:b])
        flen += list((l1 if g == 0 else l2)[a:b])
        anno += list(fix[a:b]) if g == 0 else [0] * (b - a)
        if how:
            flush_after[len(foff) - 1] = how
    foff, flen, anno = np.array(foff, np.uint64), np.array(flen, np.uint32), np.array(anno, np.uint32)
    spec = [("IPGWOptions", MY_IP_TXT + ", BATCH 500", 2), ("FixIPSrc", MY_IP_TXT, 1)]
    r = compare_chain(ctx, spec, arena, foff, flen, nh0=14, anno=anno, async_flush=True, flush_after=flush_after,
                      handlers=("drops", "packets", "lost"))
    toks = [t for t, m, p, _, _ in r]
    assert sorted(set(toks)) == list(range(len(foff)))


def test_fuzzed_combos_chain(ctx):
    from click_amd.elements import ANNO_BCAST, anno_paint
    rng, arena, foff, flen = fuzzed_frames(9)
    n = len(foff)
    anno = np.array([anno_paint(int(p)) for p in rng.integers(0, 3, n)], np.uint32) + \
        (rng.random(n) < 0.05) * ANNO_BCAST + (rng.random(n) < 0.2).astype(np.uint32)
    spec = [("IPInputCombo", "1", 1), ("IPOutputCombo", "1, %s, 120" % MY_IP_TXT, 5)]
    r = compare_chain(ctx, spec, arena, foff, flen, anno=anno, handlers=("drops", "packets", "lost"))
    assert {p for _, m, p, _, _ in r if m == 1} >= {-1, 0, 1, 2, 3, 4}


def test_check_then_set_chain(ctx):
    """CheckUDPHeader -> SetUDPChecksum over whole UDP payloads (L3 at
    offset 0): the set runs on the packets the check passed."""
    rng = np.random.default_rng(31)
    a3, o3, c3, _ = fuzz.make_batch(rng, 2500, 17, max_total=1600)
    spec = [("CheckUDPHeader", "", 2), ("SetUDPChecksum", "", 2)]
    compare_chain(ctx, spec, a3, o3, c3, nh0=0)


@pytest.mark.parametrize("nth", [1, 2, 4, 6, 8])
def test_chain_failed_flush(ctx, nth):
    """The nth checked HIP call of a chain flush fails (fake-iprouter chain:
    1 the batch's H2D, 2 CheckIPHeader's descriptors, 4 its verdicts back,
    6 DecIPTTL's descriptors, 8 its verdicts back).  Before any kernel of a
    member that is not idempotent ran (1-6): nothing is routed, nothing
    written, push() refuses packets, and the next flush resumes and routes
    every packet exactly as a chain that never failed.  A push meanwhile
    retries the failed flush first and is staged once that goes through
    (no packet lost to a transient failure).  After DecIPTTL's
    kernel (8): its packets are killed, never decremented twice."""
    from click_amd import ClickAmdError
    from click_amd.elements import Chain
    arena, foff, flen = fake_frames(3000)
    before = arena.copy()
    els = make(ctx, FAKE_IPROUTER)
    ch = Chain(els)
    base = arena.ctypes.data
    for i in range(len(foff)):
        ch.push_anno(base + int(foff[i]), int(flen[i]), -1, 0, i)
    hook = ctx.lib.clk_glue_inject_fault_internal
    hook.argtypes, hook.restype = [ctypes.c_int], None
    hook(nth)
    try:
        with pytest.raises(ClickAmdError):
            ch.flush()
    finally:
        hook(0)
    tok, mem, port, _, _ = ch.results()
    if nth == 8:
        assert len(tok) == 3000 and (mem == 3).all() and (port == -1).all()
        assert "not retried" in ch.last_error()
        assert els[3].read_handler("lost") == "3000"
        ch.flush()
        assert len(ch.results()[0]) == 0
    else:
        assert len(tok) == 0 and np.array_equal(arena, before)
        extra, _, _ = fake_frames(1)             # a packet pushed before the retry
        ch.push_anno(extra.ctypes.data, len(extra), -1, 0, 99999)
        ch.flush()
        tok, mem, port, _, _ = ch.results()
        assert len(tok) == 3001 and (mem == 4).all() and (port == 0).all()
        assert tok.tolist() == list(range(3000)) + [99999]
        ref = before.copy()                     # the same frames through a chain that never failed
        run_chain(ctx, FAKE_IPROUTER, ref, foff, flen, -1, np.zeros(len(foff), np.uint32))
        assert np.array_equal(arena, ref)
    ch.close()


@pytest.mark.parametrize("which", ["elements", "combos", "fuzzed"])
def test_zerocopy_chain(ctx, which):
    """ZEROCOPY chains: the members' kernels read and rewrite the packets in
    registered host memory; routes, lengths, bytes and handlers equal the
    staged elements one by one."""
    from click_amd.elements import ANNO_BCAST, AUX_CLONE, anno_paint
    if which == "fuzzed":
        rng, arena0, foff, flen = fuzzed_frames(77)
        n = len(foff)
        anno = np.array([anno_paint(int(p)) for p in rng.integers(0, 3, n)], np.uint32) + \
            (rng.random(n) < 0.05) * ANNO_BCAST + (rng.random(n) < 0.2).astype(np.uint32)
        spec = [("IPInputCombo", "1", 1), ("IPOutputCombo", "1, %s, 120" % MY_IP_TXT, 5)]
    else:
        arena0, foff, flen = fake_frames(20000)
        anno = np.zeros(len(foff), np.uint32)
        spec = FAKE_IPROUTER if which == "elements" else COMBOS
    a1 = arena0.copy()
    r1, e1 = run_separate(ctx, spec, a1, foff, flen, -1, anno)
    raw = np.zeros(arena0.size + 8192, np.uint8)
    a2 = raw[(-raw.ctypes.data) % 4096:][:arena0.size]
    a2[:] = arena0
    ctx.host_register(a2)
    try:
        zspec = [(c, ", ".join(x for x in (conf, "ZEROCOPY true") if x), k) for c, conf, k in spec]
        r2, e2, ch = run_chain(ctx, zspec, a2, foff, flen, -1, anno)
        clones = run_separate.clones
        for k in range(len(spec)):
            x1 = [x[:4] for x in r1 if x[1] == k]
            x2 = [y[:4] for y in r2 if y[1] == k]
            assert x1 == x2, spec[k][0]
            for y in r2:                        # clones of a member after the head: the bytes it saw
                if y[1] == k and k > 0 and spec[k][0] == "IPOutputCombo" and y[4] & AUX_CLONE:
                    assert e2[k].take_packet(y[4] & ~AUX_CLONE) == clones[(k, y[0])]
            for h in ("drops", "packets", "lost"):
                assert e1[k].read_handler(h) == e2[k].read_handler(h), (spec[k][0], h)
        assert np.array_equal(a1, a2), np.nonzero(a1 != a2)[0][:10]
        ch.close()
        for e in e1 + e2:
            e.close()
    finally:
        ctx.host_unregister(a2)


@pytest.mark.parametrize("which", ["elements", "combos"])
def test_zerocopy_chain_two_regions(ctx, which):
    """A ZEROCOPY chain fed from two registered regions in turns (runs of 500
    frames from each, as packets from two mempools): a batch ends where the
    region changes (push's fast path hands over to the slow one), and every
    result and byte equals the staged elements one by one."""
    arena0, foff, flen = fake_frames(6000)
    n = len(foff)
    anno = np.zeros(n, np.uint32)
    spec = FAKE_IPROUTER if which == "elements" else COMBOS
    a1 = arena0.copy()
    r1, e1 = run_separate(ctx, spec, a1, foff, flen, -1, anno)
    regions, raws = [], []
    for _ in range(2):
        raw = np.zeros(arena0.size + 8192, np.uint8)
        a = raw[(-raw.ctypes.data) % 4096:][:arena0.size]
        a[:] = arena0
        ctx.host_register(a)
        regions.append(a)
        raws.append(raw)
    try:
        from click_amd.elements import Chain
        zspec = [(c, ", ".join(x for x in (conf, "ZEROCOPY true") if x), k) for c, conf, k in spec]
        els = make(ctx, zspec)
        ch = Chain(els)
        src = [(i // 500) % 2 for i in range(n)]
        for i in range(n):
            if ch.push_anno(regions[src[i]].ctypes.data + int(foff[i]), int(flen[i]), -1, 0, i):
                ch.flush_async()
        ch.flush()
        tok, mem, port, length, aux = ch.results()
        r2 = list(zip(tok.tolist(), mem.tolist(), port.tolist(), length.tolist(), aux.tolist()))
        for k in range(len(spec)):
            assert [x[:4] for x in r1 if x[1] == k] == [y[:4] for y in r2 if y[1] == k], spec[k][0]
            for h in ("drops", "packets", "lost"):
                assert e1[k].read_handler(h) == els[k].read_handler(h), (spec[k][0], h)
        for i in range(n):                      # each frame's bytes in the region it was pushed from
            o, ln = int(foff[i]), int(flen[i])
            assert np.array_equal(regions[src[i]][o:o + ln], a1[o:o + ln]), i
        ch.close()
        for e in e1 + els:
            e.close()
    finally:
        for a in regions:
            ctx.host_unregister(a)


def test_chain_refuses(ctx):
    import click_amd
    from click_amd import ClickAmdError
    from click_amd.elements import Chain, Element
    with pytest.raises(ClickAmdError, match="last element"):
        Chain(make(ctx, [("IPFragmenter", "576", 2), ("DecIPTTL", "", 2)]))
    with pytest.raises(ClickAmdError, match="all ZEROCOPY or none"):
        Chain([Element(ctx, "CheckIPHeader", "", noutputs=2), Element(ctx, "DecIPTTL", "ZEROCOPY true", noutputs=2)])
    other = click_amd.Context(0)
    with pytest.raises(ClickAmdError, match="one context"):
        Chain([Element(ctx, "CheckIPHeader", "", noutputs=2), Element(other, "DecIPTTL", "", noutputs=2)])
    other.close()


def test_chain_abandon(ctx):
    """A chain whose flush keeps failing gives its packets up
    (clk_chain_abandon): each is killed at the member it reached and counted
    by that member's "lost" handler; the chain then takes packets again."""
    from click_amd import ClickAmdError
    from click_amd.elements import Chain
    arena, foff, flen = fake_frames(2000)
    before = arena.copy()
    els = make(ctx, FAKE_IPROUTER)
    ch = Chain(els)
    base = arena.ctypes.data
    for i in range(len(foff)):
        ch.push_anno(base + int(foff[i]), int(flen[i]), -1, 0, i)
    hook = ctx.lib.clk_glue_inject_fault_internal
    hook.argtypes, hook.restype = [ctypes.c_int], None
    hook(6)                                     # DecIPTTL's descriptors: the packets wait at member 3
    try:
        with pytest.raises(ClickAmdError):
            ch.flush()
    finally:
        hook(0)
    assert ch.abandon() == 2000
    tok, mem, port, _, _ = ch.results()
    assert len(tok) == 2000 and (mem == 3).all() and (port == -1).all()
    assert np.array_equal(arena, before)
    assert els[3].read_handler("lost") == "2000" and els[0].read_handler("lost") == "0"
    assert ch.abandon() == 0
    for i in range(len(foff)):                  # the chain works again
        ch.push_anno(base + int(foff[i]), int(flen[i]), -1, 0, i)
    ch.flush()
    tok, mem, port, _, _ = ch.results()
    assert len(tok) == 2000 and (mem == 4).all() and (port == 0).all()
    ch.close()
    for e in els:
        e.close()


def test_chain_copy_back_failure(ctx):
    """The rewritten bytes' copy back fails (every frame carries FIX_IP_SRC,
    so FixIPSrc rewrites each on the GPU: calls 1 H2D, 2-5 CheckIPHeader,
    6-10 FixIPSrc, 11-15 DecIPTTL, 16 the bytes back).  No result is handed
    out before its bytes are back; push() refuses packets; the next flush
    copies them and hands every packet out, bytes as a chain that never
    failed."""
    from click_amd import ClickAmdError
    from click_amd.elements import Chain
    arena, foff, flen = fake_frames(3000)
    before = arena.copy()
    els = make(ctx, FAKE_IPROUTER)
    ch = Chain(els)
    base = arena.ctypes.data
    for i in range(len(foff)):
        ch.push_anno(base + int(foff[i]), int(flen[i]), -1, 1, i)
    hook = ctx.lib.clk_glue_inject_fault_internal
    hook.argtypes, hook.restype = [ctypes.c_int], None
    hook(16)
    try:
        with pytest.raises(ClickAmdError):
            ch.flush()
    finally:
        hook(0)
    tok, mem, port, _, _ = ch.results()
    assert len(tok) == 0
    extra, _, _ = fake_frames(1)                 # a push retries the copy back first, then is staged
    ch.push_anno(extra.ctypes.data, len(extra), -1, 1, 99999)
    tok, mem, port, _, _ = ch.results()
    assert len(tok) == 3000 and (mem == 4).all() and (port == 0).all()
    ch.flush()
    assert ch.results()[0].tolist() == [99999]
    ref = before.copy()
    run_chain(ctx, FAKE_IPROUTER, ref, foff, flen, -1, np.ones(len(foff), np.uint32))
    assert np.array_equal(arena, ref) and not np.array_equal(arena, before)
    ch.close()
    for e in els:
        e.close()


def test_ttl_then_set_chain(ctx):
    """CheckIPHeader -> DecIPTTL -> SetIPChecksum: two members whose
    verdicts carry their rewrites (the TTL and checksum written into the
    packet by route(), nothing copied back for them), one after the other on
    the same bytes -- equal to the elements one by one, byte for byte."""
    rng, arena, foff, flen = fuzzed_frames(21)
    spec = [("CheckIPHeader", "OFFSET 14", 2), ("DecIPTTL", "", 2), ("SetIPChecksum", "", 1)]
    r = compare_chain(ctx, spec, arena, foff, flen)
    seen = {(m, p) for _, m, p, _, _ in r}
    assert {(0, 1), (1, 1), (2, 0)} <= seen, seen


def test_member_destroyed_before_chain(ctx):
    """A member element destroyed while its chain lives (a caller's order, or
    a garbage collector's): the chain lets go of every member, refuses
    further work, and is then destroyed without touching them."""
    from click_amd import ClickAmdError
    from click_amd.elements import Chain
    arena, foff, flen = fake_frames(100)
    els = make(ctx, FAKE_IPROUTER)
    ch = Chain(els)
    base = arena.ctypes.data
    for i in range(len(foff)):
        ch.push_anno(base + int(foff[i]), int(flen[i]), -1, 0, i)
    els[2].close()
    with pytest.raises(ClickAmdError):
        ch.push_anno(base, int(flen[0]), -1, 0, 999)
    assert "destroyed" in ch.last_error()
    ch.close()
    for e in els:
        e.close()
    ch2 = Chain(make(ctx, FAKE_IPROUTER))       # the context and the library are fine
    ch2.push_anno(base, int(flen[0]), -1, 0, 0)
    ch2.flush()
    assert len(ch2.results()[0]) == 1
    ch2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [1, 7, 64, 100])
def test_chain_results_small_pops(ctx, cap):
    """clk_chain_results in small pops: each published batch's results are
    queued whole (chain.cc publish / pop); a pop that ends inside one batch,
    or spans several, hands out the same results in the same order as one
    pop of everything (IPInputCombo -> IPOutputCombo at BATCH 64,
    double-buffered: 13 batches, some results popped between flushes)."""
    from click_amd.elements import Chain
    spec = [(c, conf + ", BATCH 64", n) for c, conf, n in COMBOS]
    bufs = [np.empty(cap, t) for t in (np.uint64, np.int32, np.int32, np.uint32, np.uint32)]
    runs = []
    for small in (False, True):
        arena, foff, flen = fake_frames(800)
        els = make(ctx, spec)
        ch = Chain(els)
        base = arena.ctypes.data
        got = [[] for _ in range(5)]
        for i in range(len(foff)):
            if ch.push_anno(base + int(foff[i]), int(flen[i]), -1, 0, i):
                ch.flush_async()
            if small and i % 300 == 299:          # one pop of part of what is queued
                n = int(ch.lib.clk_chain_results(ch.h, *[x.ctypes.data_as(ctypes.c_void_p) for x in bufs], cap))
                assert 0 < n <= cap
                for k in range(5):
                    got[k].extend(bufs[k][:n].tolist())
        ch.flush()
        r = ch.results(cap=cap) if small else ch.results()
        for k in range(5):
            got[k].extend(r[k].tolist())
        assert len(ch.results()[0]) == 0
        runs.append((got, arena))
        ch.close()
        for e in els:
            e.close()
    (a, arena_a), (b, arena_b) = runs
    assert len(a[0]) >= 800 and a == b
    assert sorted(set(a[0]))[:3] == [0, 1, 2]
    assert np.array_equal(arena_a, arena_b)
