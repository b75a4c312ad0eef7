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
