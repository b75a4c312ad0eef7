"""Zero-copy host packet memory (clk_host_register): kernels read and write
packets in registered host memory over PCIe.  The C ABI on a registered
arena and the element glue with ZEROCOPY true must give the same bytes and
results as the staged (gather + copy) path and as the oracle."""
import numpy as np
import pytest

from tests import fuzz, oracle_lib

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


def aligned_copy(a):
    """A page-aligned host copy (hipHostRegister wants whole pages)."""
    buf = np.zeros(a.size + 2 * 4096, np.uint8)
    o = (-buf.ctypes.data) % 4096
    out = buf[o:o + ((a.size + 4095) // 4096) * 4096]
    out[:a.size] = a
    return out


@pytest.mark.parametrize("op", ["check_udp", "set_udp", "check_tcp", "set_tcp", "check_ip", "set_ip", "dec_ttl"])
def test_abi_on_registered_host_memory(ctx, op):
    import torch
    import click_amd
    rng = np.random.default_rng(hash(op) % 1000)
    proto = 6 if "tcp" in op else 17
    arena, off, caplen, ml = fuzz.make_batch(rng, 3000, proto, max_total=1600)
    host = aligned_copy(arena)
    dev = ctx.host_register(host)
    try:
        b = click_amd.Batch(dev, len(off), off=torch.from_numpy(off.view(np.int64)).cuda(),
                            length=torch.from_numpy(caplen.view(np.int32)).cuda(), max_len=ml)
        fn = {"check_udp": lambda: (ctx.check_udp_header(b), None), "set_udp": lambda: ctx.set_udp_checksum(b),
              "check_tcp": lambda: (ctx.check_tcp_header(b), None),
              "set_tcp": lambda: ctx.set_tcp_checksum(b, fixoff=True),
              "check_ip": lambda: (ctx.check_ip_header(b), None), "set_ip": lambda: ctx.set_ip_checksum(b),
              "dec_ttl": lambda: ctx.dec_ip_ttl(b)}[op]
        codes, sums = fn()
        ctx.sync()
        ref = arena.copy()
        rc, rs = oracle_lib.batch(op, ref, len(off), off=off, length=caplen, arg=1)
        assert np.array_equal(codes.cpu().numpy(), rc)
        if sums is not None:
            assert np.array_equal(sums.cpu().numpy(), rs)
        assert np.array_equal(host[:arena.size], ref)
    finally:
        ctx.host_unregister(host)


@pytest.mark.parametrize("cls,conf,nout,proto", [
    ("CheckUDPHeader", "DETAILS true", 2, 17), ("SetUDPChecksum", "", 2, 17),
    ("SetTCPChecksum", "FIXOFF true", 1, 6), ("DecIPTTL", "", 2, 17),
    ("CheckIPHeader", "OFFSET 0", 2, 17), ("IPOutputCombo", "1, 18.26.4.24, 600", 5, 17),
    ("IPFragmenter", "576, true", 2, 17)])   # HONOR_DF false draws random ip_ids
def test_glue_zerocopy_matches_staged(ctx, cls, conf, nout, proto):
    from click_amd.elements import Element
    rng = np.random.default_rng(len(cls) * 31 + nout)
    arena, off, caplen, _ = fuzz.make_batch(rng, 2000, proto, max_total=1500)
    if cls == "DecIPTTL":
        fuzz.vary_ttl(rng, arena, off, caplen)
    host = aligned_copy(arena)
    staged = arena.copy()
    ctx.host_register(host)
    try:
        res = []
        for buf, zc in ((staged, False), (host, True)):
            cf = ", ".join(x for x in (conf, "BATCH 700", "ZEROCOPY true" if zc else "") if x)
            e = Element(ctx, cls, cf, noutputs=nout)
            base = buf.ctypes.data
            for i in range(len(off)):
                rc = e.lib.clk_element_push_anno(e.h, base + int(off[i]), int(caplen[i]), 0, 0, i)
                assert rc >= 0, e.lib.clk_last_error(ctx.h)
                if rc == 1:
                    e.flush()
            e.flush()
            tok, port, ln, aux = e.results(aux=True)
            frags = [e.take_packet(int(a)) for t, p, a in zip(tok, port, aux)
                     if cls == "IPFragmenter" and a and p == 0]
            res.append((tok, port, ln, frags))
            e.close()
        for k in range(3):
            assert np.array_equal(res[0][k], res[1][k]), (cls, k)
        assert res[0][3] == res[1][3]
        assert np.array_equal(staged, host[:arena.size])
    finally:
        ctx.host_unregister(host)


@pytest.mark.parametrize("zc", [False, True])
def test_push_burst_double_buffered(ctx, zc):
    """push_burst flushes with flush_async (batch k on the GPU while batch
    k+1 is staged): results come back in push order and equal the
    synchronous path's, bytes included, across many small batches."""
    from click_amd.elements import Element
    rng = np.random.default_rng(77 + zc)
    arena, off, caplen, _ = fuzz.make_batch(rng, 5000, 17, max_total=1500)
    bufs = [aligned_copy(arena), aligned_copy(arena)]
    if zc:
        for b in bufs:
            ctx.host_register(b)
    try:
        res = []
        for cls, conf in [("SetUDPChecksum", ""), ("CheckUDPHeader", "DETAILS true")]:
            for mode, buf in (("sync", bufs[0]), ("burst", bufs[1])):
                cf = ", ".join(x for x in (conf, "BATCH 333", "ZEROCOPY true" if zc else "") if x)
                e = Element(ctx, cls, cf, noutputs=2)
                ptrs = off.astype(np.uint64) + np.uint64(buf.ctypes.data)
                if mode == "burst":
                    for s in range(0, len(off), 1000):          # bursts, as an rx loop delivers them
                        m = min(1000, len(off) - s)
                        e.push_burst(ptrs[s:s + m], caplen[s:s + m], np.zeros(m, np.int32), first_token=s)
                else:
                    for i in range(len(off)):
                        if e.push_ptr(int(ptrs[i]), int(caplen[i]), 0, token=i):
                            e.flush()
                e.flush()
                tok, port, ln = e.results()
                assert np.array_equal(tok, np.arange(len(off))), (cls, mode)
                res.append((port, ln, e.read_handler("drops") if cls.startswith("Check") else ""))
                e.close()
            assert all(np.array_equal(a, b) for a, b in zip(res[-2][:2], res[-1][:2])), cls
            assert res[-2][2] == res[-1][2]
        assert np.array_equal(bufs[0], bufs[1])
    finally:
        if zc:
            for b in bufs:
                ctx.host_unregister(b)
