"""Click's -j N: several RouterThreads push packets at once.  The boundary's
rule (include/click_amd_cksum.h) is one context per thread -- calls on one
context are not re-entrant, distinct contexts are independent -- and the
adapter keeps one glue element per (element, thread) (INTEGRATION.md,
"Threads").  These tests run that layout from concurrent host threads
(ctypes releases the GIL around every library call) and check every
thread's packets and routing against the oracle."""
import threading

import numpy as np
import pytest

from tests import oracle_lib
from tests.test_gpu_elements import frames

pytestmark = pytest.mark.gpu

NTHREADS = 4


def _run_threads(fn, n=NTHREADS):
    errors, results = [], [None] * n

    def body(k):
        try:
            results[k] = fn(k)
        except Exception as exc:            # reported in the main thread
            errors.append((k, repr(exc)))

    ts = [threading.Thread(target=body, args=(k,)) for k in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errors, errors
    return results


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("cls", ["SetUDPChecksum", "CheckUDPHeader"])
def test_element_per_thread(gpu, cls):
    """Each thread: its own context, its own element, its own packets,
    pushed in bursts and flushed double-buffered while the others do the same."""
    import click_amd
    from click_amd.elements import Element
    data = [frames(np.random.default_rng(700 + k), 1500, 17) for k in range(NTHREADS)]
    refs = [a.copy() for a, _, _ in data]

    def work(k):
        arena, foff, flen = data[k]
        ctx = click_amd.Context(0, stream="own")
        try:
            e = Element(ctx, cls, "BATCH 256", name="t%d" % k, noutputs=2)
            base = arena.ctypes.data
            for s in range(0, len(foff), 100):
                ptrs = [base + int(o) for o in foff[s:s + 100]]
                e.push_burst(ptrs, [int(x) for x in flen[s:s + 100]], [14] * len(ptrs), first_token=s)
                if s % 500 == 400:
                    e.flush_async()
            e.flush()
            tok, port, _ = e.results(cap=1 << 14)
            e.close()
            return tok, port
        finally:
            ctx.close()

    out = _run_threads(work)
    op = "set_udp" if cls == "SetUDPChecksum" else "check_udp"
    for k in range(NTHREADS):
        arena, foff, flen = data[k]
        codes, _ = oracle_lib.batch(op, refs[k], len(foff), off=foff + 14, length=flen - 14)
        tok, port = out[k]
        assert np.array_equal(tok, np.arange(len(foff))), k
        assert np.array_equal(port, np.where(codes == 0, 0, 1)), k
        assert np.array_equal(arena, refs[k]), k


def test_abi_context_per_thread(gpu):
    """The device ABI directly: threads share nothing but the device; each
    runs Set then Check over its own HBM batch many times."""
    import torch
    import click_amd
    n, L, stride = 20000, 1500, 1536

    def work(k):
        ctx = click_amd.Context(0, stream="own")       # each thread its own HIP stream
        try:
            dev = torch.zeros(n * stride, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            b = click_amd.Batch(dev, n, stride=stride, fixed_len=L)
            ctx.gen_packets(b, proto=17, seed=0x5EED + k)
            for _ in range(20):
                ctx.set_ip_checksum(b, want_sums=False)
                ctx.set_udp_checksum(b, want_sums=False)
                v = ctx.check_udp_header(b)
            ctx.sync()
            return dev.cpu().numpy(), v.cpu().numpy()
        finally:
            ctx.close()

    out = _run_threads(work)
    for k in range(NTHREADS):
        host = np.zeros(n * stride, np.uint8)
        oracle_lib.gen(host, n, stride=stride, fixed_len=L, proto=17, seed=0x5EED + k)
        oracle_lib.batch("set_ip", host, n, stride=stride, fixed_len=L)
        oracle_lib.batch("set_udp", host, n, stride=stride, fixed_len=L)
        arena, v = out[k]
        assert np.array_equal(arena, host), k
        assert not v.any(), k
