"""GPU tests of the element glue's device choice and failure handling.

* DEVICE keyword (SURVEY §5 "Config / flags"): an element runs on the GPU
  it names -- on a caller's context of that device, or on its own context
  when none is given -- and a GPU that does not exist is a configure error
  (CLK_ENODEV), as Click's configure() reports bad arguments.
* A flush whose HIP runtime calls fail (injected through the glue's test
  hook at every checked call of the flush path) routes NOTHING and writes
  nothing into the packets; the batch stays staged and the next flush
  routes it exactly as the oracle decides.
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def udp_packets(n, L=600, stride=640, seed=0x5EED):
    arena = np.zeros(n * stride, np.uint8)
    oracle_lib.gen(arena, n, stride=stride, fixed_len=L, proto=17, seed=seed)
    oracle_lib.batch("set_ip", arena, n, stride=stride, fixed_len=L)
    return arena, np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(stride), \
        np.full(n, L, np.uint32)


def test_device_count(ctx):
    assert ctx.lib.clk_device_count() >= 1


def test_device_keyword(ctx):
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    nd = ctx.lib.clk_device_count()
    e = Element(ctx, "CheckUDPHeader", "DEVICE 0", noutputs=2)
    assert e.read_handler("device") == "0"
    e.close()
    # no context: the element makes its own on DEVICE, and it works
    n, L, stride = 500, 600, 640
    arena, ptrs, lens = udp_packets(n, L, stride)
    ref = arena.copy()
    rc, _ = oracle_lib.batch("set_udp", ref, n, stride=stride, fixed_len=L)
    e = Element(None, "SetUDPChecksum", "DEVICE 0", noutputs=2)
    assert e.read_handler("device") == "0"
    e.push_burst(ptrs, lens, np.zeros(n, np.int32))
    e.flush()
    tok, port, _ = e.results()
    assert (tok == np.arange(n)).all() and (port == rc.astype(np.int32)).all()
    assert np.array_equal(arena, ref)
    e.close()
    # a GPU that does not exist
    for c in (None, ctx):
        with pytest.raises(ClickAmdError) as ei:
            Element(c, "CheckIPHeader", "DEVICE %d" % nd)
        assert ei.value.rc == -3 and "no such GPU" in str(ei.value)
    with pytest.raises(ClickAmdError) as ei:
        Element(ctx, "CheckIPHeader", "DEVICE -1")
    assert ei.value.rc == -1


@pytest.mark.parametrize("nth", list(range(1, 13)))
def test_flush_failure_routes_nothing(ctx, nth):
    """Fail the nth checked HIP call of a fresh element's first flush (event
    creation, H2D of packets / descriptors, event records, D2H of verdicts /
    checksums, the completion wait): the flush raises, no result is routed,
    no packet byte changes; the retry routes every packet as the oracle."""
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    n, L, stride = 300, 600, 640
    arena, ptrs, lens = udp_packets(n, L, stride, seed=nth)
    before = arena.copy()
    ref = arena.copy()
    rc, _ = oracle_lib.batch("set_udp", ref, n, stride=stride, fixed_len=L)
    e = Element(ctx, "SetUDPChecksum", "", noutputs=2)
    e.push_burst(ptrs, lens, np.zeros(n, np.int32))
    hook = ctx.lib.clk_glue_inject_fault_internal
    hook.argtypes, hook.restype = [ctypes.c_int], None
    hook(nth)
    try:
        with pytest.raises(ClickAmdError) as ei:
            e.flush()
        assert ei.value.rc == -2
        assert e.last_error()
    finally:
        hook(0)
    tok, port, _ = e.results()
    assert len(tok) == 0                       # nothing routed on stale verdicts
    assert np.array_equal(arena, before)       # nothing written back
    e.flush()                                  # the staged batch is retried
    tok, port, _ = e.results()
    assert (tok == np.arange(n)).all() and (port == rc.astype(np.int32)).all()
    assert np.array_equal(arena, ref)
    assert e.read_handler("batches") == "1"
    e.close()


def udp_600(n):
    """n synthetic 600 B UDP/IPv4 packets (valid IP checksums) in 640 B
    slots: longer than IPFragmenter(576)'s MTU."""
    L, stride = 600, 640
    arena = np.zeros(n * stride, np.uint8)
    oracle_lib.gen(arena, n, stride=stride, fixed_len=L, proto=17, seed=7)
    oracle_lib.batch("set_ip", arena, n, stride=stride, fixed_len=L)
    return arena, L, stride


# nth: the n-th checked HIP call of the flush fails (4: the packets' H2D,
# before any kernel; IPOutputCombo 11 its checksums back, 12 the rewritten
# arena back); -1: the completion wait, after the kernel ran and the
# rewritten arena was copied back
@pytest.mark.parametrize("cls,conf,nth", [("IPOutputCombo", "1, 18.26.4.24, 1500", k) for k in (4, 11, 12, -1)] +
                         [("IPFragmenter", "576", k) for k in (4, -1)] +
                         [("DecIPTTL", "", k) for k in (4, -1)])
def test_rewriting_element_retry_is_exact(ctx, cls, conf, nth):
    """A rewriting element (IPOutputCombo, IPFragmenter, DecIPTTL) whose
    flush fails at the n-th checked HIP call -- the completion wait
    included, after the rewritten arena was copied back -- retries from the
    bytes as staged: the packets are rewritten ONCE, exactly as the oracle
    (the copy back went into the staging arena itself)."""
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    n = 200
    arena, L, stride = udp_600(n)
    ref = arena.copy()
    if cls == "IPOutputCombo":
        rc, _, _ = oracle_lib.ip_out_batch("ip_output_combo", ref, n, stride=stride, fixed_len=L, my_ip=0x18041A12,
                                           mtu=1500)
    elif cls == "DecIPTTL":
        rc, _ = oracle_lib.batch("dec_ttl", ref, n, stride=stride, fixed_len=L)
    else:
        fr = oracle_lib.ip_fragment(ref, n, 576, True, stride=stride, fixed_len=L)
        rc = fr["port"]
    e = Element(ctx, cls, conf, noutputs=5 if cls == "IPOutputCombo" else 2)
    ptrs = np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(stride)
    e.push_burst(ptrs, np.full(n, L, np.uint32), np.zeros(n, np.int32))
    hook = ctx.lib.clk_glue_inject_fault_internal
    hook.argtypes, hook.restype = [ctypes.c_int], None
    hook(nth)
    try:
        with pytest.raises(ClickAmdError):
            e.flush()
    finally:
        hook(0)
    assert len(e.results()[0]) == 0
    e.flush()
    tok, port, ln, aux = e.results(aux=True)
    prim = aux == 0 if cls == "IPFragmenter" else np.ones(len(tok), bool)
    assert (tok[prim] == np.arange(n)).all()
    if cls == "IPFragmenter":
        assert (np.where(port[prim] == 0, np.where(ln[prim] < L, 2, 0), 1) == rc).all()
        # first fragments written back in place, byte for byte
        for i in range(n):
            o = i * stride
            assert np.array_equal(arena[o:o + int(fr["first_len"][i])], ref[o:o + int(fr["first_len"][i])]), i
        extra = [e.take_packet(int(a)) for a in aux[~prim]]
        assert extra == fr["frags"]
    else:
        assert (port == rc.astype(np.int32)).all()
        assert np.array_equal(arena, ref)
    e.close()


def test_zerocopy_rewriting_batch_is_abandoned(ctx):
    """ZEROCOPY DecIPTTL: the kernel decrements TTL in host memory itself,
    so a batch whose completion wait fails is not retried (that would
    decrement twice) but abandoned: every packet routed as killed, counted
    by the "lost" handler, and no TTL decremented twice."""
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    n, L, stride = 300, 600, 640
    raw = np.zeros(n * stride + 8192, np.uint8)
    arena = raw[(-raw.ctypes.data) % 4096:][:n * stride]
    a2, _, _ = udp_600(n)
    arena[:] = a2
    ttl0 = arena.reshape(n, stride)[:, 8].copy()
    ctx.host_register(arena)
    try:
        e = Element(ctx, "DecIPTTL", "ZEROCOPY true", noutputs=2)
        ptrs = np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(stride)
        e.push_burst(ptrs, np.full(n, L, np.uint32), np.zeros(n, np.int32))
        hook = ctx.lib.clk_glue_inject_fault_internal
        hook.argtypes, hook.restype = [ctypes.c_int], None
        hook(-1)                                   # the completion wait of the zero-copy flush
        try:
            with pytest.raises(ClickAmdError) as ei:
                e.flush()
        finally:
            hook(0)
        assert "not retried" in str(ei.value)
        tok, port, _ = e.results()
        assert (tok == np.arange(n)).all() and (port == -1).all()
        assert e.read_handler("lost") == str(n)
        e.flush()                                  # nothing left to retry
        assert len(e.results()[0]) == 0
        assert (arena.reshape(n, stride)[:, 8] >= ttl0 - 1).all()
        e.close()
    finally:
        ctx.host_unregister(arena)


@pytest.mark.parametrize("nth", list(range(1, 13)))
def test_zerocopy_rewriting_batch_any_failed_step(ctx, nth):
    """ZEROCOPY DecIPTTL with the nth checked HIP call of its flush failing
    (event creation, descriptor copies, the records around the kernel, the
    verdict / checksum / aux copies back): whatever step fails, no TTL is
    decremented twice.  A failure before the kernel leaves the batch staged
    and the retry forwards every packet decremented once; a failure after it
    abandons the batch (every packet killed, counted as lost) -- the
    kernel already rewrote the host packets, so a retry would decrement
    again."""
    from click_amd import ClickAmdError
    from click_amd.elements import Element
    n, L, stride = 300, 600, 640
    raw = np.zeros(n * stride + 8192, np.uint8)
    arena = raw[(-raw.ctypes.data) % 4096:][:n * stride]
    a2, _, _ = udp_600(n)
    arena[:] = a2
    ttl0 = arena.reshape(n, stride)[:, 8].copy()
    ctx.host_register(arena)
    try:
        e = Element(ctx, "DecIPTTL", "ZEROCOPY true", noutputs=2)
        ptrs = np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(stride)
        e.push_burst(ptrs, np.full(n, L, np.uint32), np.zeros(n, np.int32))
        hook = ctx.lib.clk_glue_inject_fault_internal
        hook.argtypes, hook.restype = [ctypes.c_int], None
        hook(nth)
        failed = None
        try:
            e.flush()
        except ClickAmdError as ex:
            failed = str(ex)
        finally:
            hook(0)
        e.flush()                                  # the retry, if the batch is still staged
        tok, port, _ = e.results()
        assert (np.sort(tok) == np.arange(n)).all()
        ttl = arena.reshape(n, stride)[:, 8]
        assert (ttl >= ttl0 - 1).all(), "a TTL was decremented twice"
        if failed and "not retried" in failed:
            assert (port == -1).all() and e.read_handler("lost") == str(n)
        else:                                      # no failure reached, or one before the kernel: retried
            assert (port == 0).all() and (ttl == ttl0 - 1).all() and e.read_handler("lost") == "0"
        e.close()
    finally:
        ctx.host_unregister(arena)
