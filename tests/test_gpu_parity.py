"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle.

Bit-exact on every output: per-packet verdict/status codes, returned 16-bit
checksums, and every byte of the arena after a Set element (no stray
writes).  Inputs: the golden vectors from the reference's files, seeded
fuzzed batches covering every branch and alignment, and full-size batches
checked through size-independent properties.
"""
import json
import os

import numpy as np
import pytest

from tests import oracle_lib, fuzz

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")
OPS_L4 = {17: ("check_udp", "set_udp"), 6: ("check_tcp", "set_tcp"), 1: ("check_icmp",)}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def ctx(torch):
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def dev_batch(torch, arena, n, off=None, length=None, stride=0, fixed_len=0, max_len=0, place=None):
    """A device batch over a copy of `arena`; `place(arena)` may put that copy
    at a chosen device address (a view into a larger buffer)."""
    import click_amd
    base = torch.from_numpy(arena).to("cuda:0") if place is None else place(arena)
    o = torch.from_numpy(off.astype(np.uint64).view(np.int64)).to("cuda:0") if off is not None else None
    ln = torch.from_numpy(length.astype(np.uint32).view(np.int32)).to("cuda:0") if length is not None else None
    return click_amd.Batch(base, n, stride=stride, fixed_len=fixed_len, off=o, length=ln, max_len=max_len)


def run_gpu(ctx, op, b, arg=1):
    if op == "in_cksum":
        return None, ctx.in_cksum(b)
    if op == "check_ip":
        return ctx.check_ip_header(b, checksum=bool(arg)), None
    if op == "set_ip":
        return ctx.set_ip_checksum(b)
    if op == "check_udp":
        return ctx.check_udp_header(b), None
    if op == "set_udp":
        return ctx.set_udp_checksum(b)
    if op == "check_tcp":
        return ctx.check_tcp_header(b), None
    if op == "set_tcp":
        return ctx.set_tcp_checksum(b, fixoff=bool(arg))
    if op == "check_icmp":
        return ctx.check_icmp_header(b), None
    if op == "dec_ttl":
        return ctx.dec_ip_ttl(b, multicast=bool(arg))
    raise ValueError(op)


def compare(torch, ctx, op, arena, n, off=None, length=None, stride=0, fixed_len=0, max_len=0, arg=1, place=None):
    """Run op on GPU and oracle over identical inputs; assert bit-exactness."""
    b = dev_batch(torch, arena, n, off, length, stride, fixed_len, max_len, place)
    codes, sums = run_gpu(ctx, op, b, arg)
    ctx.sync()
    ref = arena.copy()
    rc, rs = oracle_lib.batch(op, ref, n, stride=stride, fixed_len=fixed_len, off=off, length=length, arg=arg)
    if codes is not None:
        g = codes.cpu().numpy()
        bad = np.nonzero(g != rc)[0]
        assert bad.size == 0, (op, bad[:10], g[bad[:10]], rc[bad[:10]])
    if sums is not None:
        g = sums.cpu().numpy()
        bad = np.nonzero(g != rs)[0]
        assert bad.size == 0, (op, bad[:10], g[bad[:10]], rs[bad[:10]])
    after = b.base.cpu().numpy()
    diff = np.nonzero(after != ref)[0]
    assert diff.size == 0, (op, "arena differs at", diff[:10])
    return rc, rs


# ---------------------------------------------------------------------------
def test_golden_vectors_on_gpu(torch, ctx):
    vecs = json.load(open(GOLDEN))["vectors"]
    for v in vecs:
        data = bytes([v["fill"]]) * v["caplen"] if "fill" in v else bytes.fromhex(v["l3"])
        op = "set_tcp" if v["op"] == "set_tcp_then_rfc1071" else v["op"]
        for shift in (0, 1, 2, 3, 14):          # the vector at several alignments
            arena = np.zeros(shift + len(data) + 32, np.uint8)
            arena[shift:shift + len(data)] = np.frombuffer(data, np.uint8)
            off = np.array([shift], np.uint64)
            ln = np.array([v["caplen"]], np.uint32)
            b = dev_batch(torch, arena, 1, off, ln, max_len=v["caplen"])
            codes, sums = run_gpu(ctx, op, b, v.get("arg", 1 if op != "set_tcp" else 0))
            ctx.sync()
            if v["op"] == "set_tcp_then_rfc1071":
                assert int(codes.cpu()[0]) == 0, v["name"]
                from tests.test_oracle import rfc1071_tcp_ok
                out = b.base.cpu().numpy()[shift:shift + len(data)].tobytes()
                assert rfc1071_tcp_ok(out, v["final_dst"]), v["name"]
                continue
            got = int(sums.cpu()[0]) if (op == "in_cksum" or op.startswith("set_")) else int(codes.cpu()[0])
            assert got == v["expect"], (v["name"], shift, got)


@pytest.mark.parametrize("proto", [17, 6, 1])
@pytest.mark.parametrize("max_total,align", [(96, "any"), (400, "any"), (1600, "even"), (1600, "any"),
                                             (5000, "any"), (20000, "even")])
def test_fuzz_parity(torch, ctx, proto, max_total, align):
    rng = np.random.default_rng(proto * 1000 + max_total + (align == "any"))
    n = 3000 if max_total <= 1600 else 400
    arena, off, caplen, ml = fuzz.make_batch(rng, n, proto, max_total=max_total, align=align)
    for op in ("check_ip", "set_ip") + OPS_L4[proto]:
        compare(torch, ctx, op, arena, n, off=off, length=caplen, max_len=ml, arg=1)
    if proto != 1:
        compare(torch, ctx, OPS_L4[proto][1], arena, n, off=off, length=caplen, max_len=ml, arg=0)
    compare(torch, ctx, "check_ip", arena, n, off=off, length=caplen, max_len=ml, arg=0)   # CheckIPHeader2
    fuzz.vary_ttl(rng, arena, off, caplen)
    for multicast in (1, 0):                                                            # DecIPTTL
        compare(torch, ctx, "dec_ttl", arena, n, off=off, length=caplen, max_len=ml, arg=multicast)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 130, 257])
@pytest.mark.parametrize("proto,max_total", [(17, 1600), (6, 1600), (17, 20000), (6, 20000)])
@pytest.mark.parametrize("set_mode", [-1, 0])
def test_run_tails(torch, n, proto, max_total, set_mode):
    """The fixed-geometry kernels store their outputs per run of 64 packets
    (CLK_L4_RUNS): batch sizes around a run boundary, 16 and 64 lanes per
    packet, Check and Set (two-phase by default; set_mode 0: fused, the
    field's 64 B block stored whole from the pass-0 registers where it lies
    in the packet), FIXOFF on and off, 64 B-aligned and any alignment."""
    import click_amd
    c = click_amd.Context(0).tune(set_mode=set_mode)
    rng = np.random.default_rng(n * 31 + proto + max_total)
    for align in ("any", 64):
        arena, off, caplen, ml = fuzz.make_batch(rng, n, proto, max_total=max_total, align=align)
        for op in OPS_L4[proto]:
            compare(torch, c, op, arena, n, off=off, length=caplen, max_len=ml, arg=1)
        compare(torch, c, OPS_L4[proto][1], arena, n, off=off, length=caplen, max_len=ml, arg=0)
    c.close()


def test_run_outputs_at_odd_address(torch, ctx):
    """Verdict bytes written into an output view at an odd address."""
    rng = np.random.default_rng(3)
    n = 200
    arena, off, caplen, ml = fuzz.make_batch(rng, n, 17, max_total=1600, align="any")
    b = dev_batch(torch, arena, n, off, caplen, max_len=ml)
    big = torch.full((n + 2,), 0xEE, dtype=torch.uint8, device="cuda:0")
    ctx.check_udp_header(b, out=big[1:n + 1])
    ctx.sync()
    rc, _ = oracle_lib.batch("check_udp", arena.copy(), n, off=off, length=caplen)
    g = big.cpu().numpy()
    assert g[0] == 0xEE and g[n + 1] == 0xEE
    assert np.array_equal(g[1:n + 1], rc)


@pytest.mark.parametrize("max_len_hint", [0, 64, 500, 2000, 100000])
def test_geometry_hint_does_not_change_results(torch, ctx, max_len_hint):
    """Lanes per packet (1/4/16/64, multi-pass) is a speed choice only; a
    hint smaller than the real maximum must stay exact (multi-pass)."""
    rng = np.random.default_rng(77)
    arena, off, caplen, _ = fuzz.make_batch(rng, 800, 17, max_total=3000)
    for op in ("check_udp", "set_udp", "in_cksum"):
        compare(torch, ctx, op, arena, 800, off=off, length=caplen, max_len=max_len_hint)


def test_in_cksum_ranges(torch, ctx):
    rng = np.random.default_rng(5)
    n = 1500
    lens = np.concatenate([np.arange(0, 300), rng.integers(0, 70000, n - 310),
                           np.array([131072, 131074, 131076, 200000, 262147, 0, 1, 2, 3, 5])]).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 16))
        off[i] = pos
        pos += int(lens[i])
    arena = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    for i in range(n - 10, n - 5):              # the wrap cases are all 0xFF
        arena[int(off[i]):int(off[i]) + int(lens[i])] = 0xFF
    compare(torch, ctx, "in_cksum", arena, n, off=off, length=lens, max_len=int(lens.max()))
    compare(torch, ctx, "in_cksum", arena, n, off=off, length=lens, max_len=0)
    # negative int lengths sum nothing (click_in_cksum's `int len`)
    neg = np.array([0xFFFFFFF0, 0x80000000], np.uint32)
    compare(torch, ctx, "in_cksum", arena, 2, off=off[:2], length=neg, max_len=64)


def test_fixed_stride_and_generator(torch, ctx):
    import click_amd
    for proto, L, stride in ((17, 1500, 1536), (6, 9000, 9024), (17, 46, 64), (6, 64, 64), (17, 577, 640)):
        n = 1000
        arena = np.zeros(n * stride, np.uint8)
        oracle_lib.gen(arena, n, stride=stride, fixed_len=L, proto=proto, seed=0x5EED, first_idx=7)
        dev = torch.zeros(n * stride, dtype=torch.uint8, device="cuda:0")
        b = click_amd.Batch(dev, n, stride=stride, fixed_len=L)
        ctx.gen_packets(b, proto=proto, seed=0x5EED, first_idx=7)
        ctx.sync()
        g = dev.cpu().numpy()
        assert np.array_equal(g, arena), (proto, L, np.nonzero(g != arena)[0][:8])
        for op in ("set_ip", "check_ip") + OPS_L4[proto]:
            compare(torch, ctx, op, arena, n, stride=stride, fixed_len=L)
            oracle_lib.batch(op, arena, n, stride=stride, fixed_len=L)


def test_check_ip_offset_badsrc(torch, ctx):
    rng = np.random.default_rng(9)
    n, L, stride = 2000, 60, 80
    arena = np.zeros(n * stride + 64, np.uint8)
    oracle_lib.gen(arena[14:], n, stride=stride, fixed_len=L, proto=17)
    oracle_lib.batch("set_ip", arena[14:], n, stride=stride, fixed_len=L)
    # BADSRC: a handful of the packets' own sources; GOODDST: some dsts
    words = arena[14:].view(np.uint8)
    src_words = np.array([int.from_bytes(words[i * stride + 12:i * stride + 16].tobytes(), "little")
                          for i in range(n)], np.uint32)
    dst_words = np.array([int.from_bytes(words[i * stride + 16:i * stride + 20].tobytes(), "little")
                          for i in range(n)], np.uint32)
    bad = src_words[rng.choice(n, 50, replace=False)]
    good = dst_words[rng.choice(n, 700, replace=False)]
    b = dev_batch(torch, arena, n, stride=stride, fixed_len=L + 14)
    bt = torch.from_numpy(bad.view(np.int32)).to("cuda:0")
    gt = torch.from_numpy(good.view(np.int32)).to("cuda:0")
    codes = ctx.check_ip_header(b, offset=14, checksum=True, badsrc=bt, gooddst=gt).cpu().numpy()
    L_ = oracle_lib.load_oracle()
    exp = np.array([L_.oracle_check_ip_header(arena[i * stride:].ctypes.data, L + 14, 14, 1,
                                              bad.ctypes.data, len(bad), good.ctypes.data, len(good))
                    for i in range(n)], np.uint8)
    assert np.array_equal(codes, exp)
    assert (exp == 6).sum() > 0 and (exp == 0).sum() > 0


def test_count_codes(torch, ctx):
    rng = np.random.default_rng(11)
    c = rng.integers(0, 7, 1_000_003, dtype=np.uint8)
    counts = ctx.count_codes(torch.from_numpy(c).to("cuda:0"), ncounts=8).cpu().numpy()
    assert np.array_equal(counts, np.bincount(c, minlength=8))


# ---------------------------------------------------------------------------
# Full-size properties (BASELINE configs 2 and 3 shapes).
# ---------------------------------------------------------------------------
def splitmix64_np(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


@pytest.mark.parametrize("proto,L,stride,n", [(17, 1500, 1536, 16 << 20), (17, 46, 64, 16 << 20),
                                              (6, 9000, 9024, 1 << 20)])
def test_full_size_properties(torch, ctx, proto, L, stride, n):
    """Set then Check passes everywhere; the whole batch's SetIPChecksum and
    Set L4 checksums, and the corrupted L4 Check's verdicts, match the host
    oracle's digest (as bench.py's verify); one flipped bit in 1/1024
    packets is caught exactly on those packets; a random sample of packets
    matches the oracle byte for byte."""
    import bench
    import click_amd
    from click_amd import shard
    check_el, set_el = ("CheckUDPHeader", "SetUDPChecksum") if proto == 17 else ("CheckTCPHeader", "SetTCPChecksum")
    els = ["SetIPChecksum"] + ([check_el, set_el] if L >= 28 else [])
    od = oracle_lib.digest(els, proto, 0, n, fixed_len=L, threads=bench.verify_threads(1))

    def same(codes, sums, e):
        gd = shard.digest(torch, codes, sums, 0)
        assert {f: gd[f] for f in shard.DIGEST_FIELDS} == od[e], (e, gd, od[e])
    with np.errstate(over="ignore"):
        arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda:0")
        b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
        ctx.gen_packets(b, proto=proto)
        st, sums = ctx.set_ip_checksum(b)
        assert int(ctx.count_codes(st)[0]) == n
        same(st, sums, "SetIPChecksum")
        if L >= 28:
            st, sums = (ctx.set_udp_checksum(b) if proto == 17 else ctx.set_tcp_checksum(b))
            assert int(ctx.count_codes(st)[0]) == n
            same(st, sums, set_el)
            v = ctx.check_udp_header(b) if proto == 17 else ctx.check_tcp_header(b)
            assert int(ctx.count_codes(v)[0]) == n
        v = ctx.check_ip_header(b)
        assert int(ctx.count_codes(v)[0]) == n
        # sample vs oracle
        rng = np.random.default_rng(12)
        idx = np.sort(rng.choice(n, 512, replace=False))
        host = arena.view(n, stride)[torch.from_numpy(idx).to("cuda:0")].cpu().numpy().reshape(-1)
        ref = np.zeros_like(host)
        for k, i in enumerate(idx):
            oracle_lib.gen(ref[k * stride:], 1, stride=stride, fixed_len=L, proto=proto, first_idx=int(i))
        oracle_lib.batch("set_ip", ref, len(idx), stride=stride, fixed_len=L)
        if L >= 28:
            oracle_lib.batch("set_udp" if proto == 17 else "set_tcp", ref, len(idx), stride=stride,
                             fixed_len=L, arg=0)
        # slot bytes past L are not part of the packet (torch.empty garbage)
        assert np.array_equal(host.reshape(-1, stride)[:, :L], ref.reshape(-1, stride)[:, :L])
        # corruption is caught exactly where it was injected
        if L >= 28:
            ctx.gen_corrupt(b, seed=0xBAD, rate_log2=10)
            vt = ctx.check_udp_header(b) if proto == 17 else ctx.check_tcp_header(b)
            same(vt, None, check_el)
            v = vt.cpu().numpy()
            i64 = np.arange(n, dtype=np.uint64)
            h = splitmix64_np(np.uint64(0xBAD) ^ (i64 * np.uint64(0xD1B54A32D192ED03)))
            sel = (h & np.uint64(1023)) == 0
            assert sel.sum() > 0
            assert np.array_equal(v == 3, sel)
            assert np.array_equal(v == 0, ~sel)
        del arena
        torch.cuda.empty_cache()


def test_dec_ttl_full_size(torch, ctx):
    """DecIPTTL over a C2-sized batch (16M x 64 B slots): every TTL drops by
    one and the RFC 1624 update equals a full recomputation (CheckIPHeader
    passes; SetIPChecksum rewrites the same values)."""
    import click_amd
    n, L, stride = 16 << 20, 46, 64
    arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda:0")
    b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
    ctx.gen_packets(b, proto=17)
    ctx.set_ip_checksum(b, want_sums=False)
    st, sums = ctx.dec_ip_ttl(b)
    assert int((st != 0).sum()) == 0
    assert int(ctx.check_ip_header(b).ne(0).sum()) == 0
    ttl = arena.view(n, stride)[:, 8]
    assert int((ttl != 63).sum()) == 0
    st2, sums2 = ctx.set_ip_checksum(b)
    assert torch.equal(sums, sums2)
    del arena
    torch.cuda.empty_cache()


@pytest.mark.parametrize("chunks", [2, 5, 64])
def test_chunked_two_phase_set_bit_exact(torch, chunks):
    """The two-phase Set in packet ranges (set_chunks: each range's scatter
    on a side stream, overlapping the next range's compute pass) equals the
    oracle on fuzzed off/len batches, on fixed-stride batches, and on
    batches smaller than one range."""
    import click_amd
    c = click_amd.Context(0).tune(set_mode=1, set_chunks=chunks)
    rng = np.random.default_rng(chunks)
    for proto in (17, 6):
        arena, off, caplen, ml = fuzz.make_batch(rng, 3000, proto, max_total=1600)
        compare(torch, c, OPS_L4[proto][1], arena, len(off), off=off, length=caplen, max_len=ml, arg=1)
    for n in (4096 + 77, 100):
        L, stride = 1500, 1536
        arena = np.zeros(n * stride, np.uint8)
        oracle_lib.gen(arena, n, stride=stride, fixed_len=L)
        compare(torch, c, "set_udp", arena, n, stride=stride, fixed_len=L)
    c.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_set_modes_bit_exact(torch, mode):
    """Fused (mode 0) and two-phase (mode 1, compute then scatter) Set
    kernels give identical results on fuzzed batches."""
    import click_amd
    c = click_amd.Context(0).tune(set_mode=mode)
    rng = np.random.default_rng(31)
    for proto in (17, 6):
        arena, off, caplen, ml = fuzz.make_batch(rng, 1500, proto, max_total=1600)
        for op in ("set_ip", OPS_L4[proto][1]):
            compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1)
    n, L, stride = 4096, 1500, 1536
    arena = np.zeros(n * stride, np.uint8)
    oracle_lib.gen(arena, n, stride=stride, fixed_len=L)
    for op in ("set_ip", "set_udp"):
        compare(torch, c, op, arena, n, stride=stride, fixed_len=L)
    c.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_stream_set_modes_bit_exact(torch, mode):
    """The packet-stream kernel's Sets: fused (mode 0: the patched 64 B
    blocks stored coalesced from the LDS stash, or the field alone when its
    block is not the packet's) and two-phase (mode 1: the compute pass
    stashes fewer chunks, then the nontemporal scatter), any alignment,
    FIXOFF on and off."""
    import click_amd
    c = click_amd.Context(0).tune(set_mode=mode, stream_min=1)
    rng = np.random.default_rng(57 + int(mode))
    for proto, mt in ((17, 1600), (6, 1600), (17, 200), (6, 9000)):
        for align in ("any", 64):
            arena, off, caplen, ml = fuzz.make_batch(rng, 1500, proto, max_total=mt, align=align)
            op = OPS_L4[proto][1]
            compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1)
            if proto == 6:
                compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=0)
    c.close()


@pytest.mark.parametrize("stream_min,group", [(1, 0), (100000000, 0), (100000000, 4), (100000000, 64)])
def test_variable_length_paths_bit_exact(torch, stream_min, group):
    """Variable-length batches run by the packet-stream kernel (stream_min
    1) or in one lanes-per-packet geometry (by max_len, or forced): all
    identical and oracle-exact."""
    import click_amd
    c = click_amd.Context(0).tune(stream_min=stream_min, group=group)
    rng = np.random.default_rng(41)
    for proto, mt in ((17, 1600), (6, 9000), (17, 200), (1, 1600)):
        arena, off, caplen, ml = fuzz.make_batch(rng, 2000, proto, max_total=mt)
        for op in ("in_cksum",) + OPS_L4[proto]:
            compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1)
            compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=0, arg=1)
    # IMIX-like sizes, packed at 64 B-aligned offsets
    n = 20000
    L = rng.choice(np.array([64, 576, 1500], np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12]).astype(np.uint32)
    slot = (L + 63) // 64 * 64
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(slot[:-1])
    arena = np.zeros(int(off[-1] + slot[-1]), np.uint8)
    for i in range(n):
        oracle_lib.gen(arena[int(off[i]):], 1, stride=0, fixed_len=int(L[i]), proto=17, first_idx=i)
    oracle_lib.batch("set_ip", arena, n, off=off, length=L)
    for op in ("set_udp", "check_udp", "in_cksum"):
        compare(torch, c, op, arena, n, off=off, length=L, max_len=1500)
        oracle_lib.batch(op, arena, n, off=off, length=L)
    c.close()


class HighPlacer:
    """Places an arena copy at a device address whose low 32 bits are just
    below `low` (2^31 or 2^32), inside one buffer a little over 4 GiB, so the
    batch's chunk spans cross bit 31 of the address's low word or a 4 GiB
    boundary.  Round 3's readfirstlane variant of the packet-stream kernel
    widened the span base's low word as a signed int and faulted on exactly
    these addresses (DESIGN.md "Stream-kernel fault")."""

    def __init__(self, torch, room=1 << 24):
        self.torch = torch
        self.room = room
        self.buf = torch.empty((1 << 32) + 2 * room, dtype=torch.uint8, device="cuda:0")
        self.p = self.buf.data_ptr()

    def at(self, low, back):
        def place(arena):
            assert arena.size <= self.room
            o = ((low - back - self.p) % (1 << 32)) & ~15   # (p + o) mod 2^32 = low - back, 16 B-aligned
            v = self.buf[o:o + arena.size]
            v.copy_(self.torch.from_numpy(arena))
            return v
        return place


@pytest.mark.parametrize("low", [1 << 31, 1 << 32])
def test_stream_high_address_bits(torch, low):
    """Packet-stream batches (seed 41, as test_variable_length_paths_bit_exact,
    and the dense / generic layouts) placed so that their runs straddle bit
    31 of the address's low word (low = 2^31) or a 4 GiB boundary (low =
    2^32): every chunk address is formed in 64 bits, oracle-exact."""
    import click_amd
    hp = HighPlacer(torch)
    c = click_amd.Context(0).tune(stream_min=1)
    rng = np.random.default_rng(41)
    for proto, mt in ((17, 1600), (6, 9000), (1, 1600)):
        arena, off, caplen, ml = fuzz.make_batch(rng, 2000, proto, max_total=mt)
        for back in (4096, arena.size // 2):
            for op in ("in_cksum",) + OPS_L4[proto]:
                compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1,
                        place=hp.at(low, back))
    for kind in ("packed", "odd", "shared"):
        arena, off, caplen, ml = dense_layout(rng, 700, 17, kind)
        for back in (4096, arena.size // 2):
            for op in OPS_L4[17]:
                compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1,
                        place=hp.at(low, back))
    c.close()
    del hp


def test_stream_descriptor_past_max_len(torch):
    """A len[] entry longer than the batch's max_len (a caller's contract
    slip) and longer than the packet stream's 16 MiB chunk-index bound: the
    run holding it sums each packet from memory (no chunk index wraps), and
    every result still equals the oracle's over the true lengths."""
    import click_amd
    c = click_amd.Context(0).tune(stream_min=1)
    rng = np.random.default_rng(17)
    for proto in (17, 6):
        arena, off, caplen, ml = fuzz.make_batch(rng, 300, proto, max_total=1600)
        big = (1 << 24) + 4096 + 3
        tail = int(off.max()) + int(caplen.max()) + 64
        big_pkt = np.frombuffer(fuzz.build(rng, proto, 1400), np.uint8)
        arena = np.concatenate([arena[:tail], np.zeros(tail + big + 64 - arena[:tail].size, np.uint8)])
        arena[tail:tail + big_pkt.size] = big_pkt
        off = off.copy()
        caplen = caplen.copy()
        off[150], caplen[150] = tail, big       # 1400 B of IP packet, then zeros to 16 MiB + 4 KiB
        oracle_lib.batch("set_ip", arena, len(off), off=off, length=caplen)
        for op in ("in_cksum",) + OPS_L4[proto]:
            compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1)
    c.close()


def test_tune_rejects_bad_values(torch):
    import click_amd
    c = click_amd.Context(0)
    for k, v in (("group", 3), ("set_mode", 2), ("max_blocks", 0), ("stream_min", 0)):
        with pytest.raises(click_amd.ClickAmdError):
            c.tune(**{k: v})
    c.close()


def dense_layout(rng, n, proto, kind):
    """Packets of random sizes laid out for the packet-stream kernel's dense
    (span) and generic runs: 'packed' (64 B-aligned, disjoint: dense),
    'odd' (odd starts, >= 16 B gaps: disjoint chunk ranges, dense with byte
    swaps), 'empty' (every 7th packet caplen 0), 'gaps' (a 4 KB hole every
    50 packets: those runs exceed the span slack -> generic), 'shared' (no
    gap: neighbours share a chunk -> generic), 'reversed' (every other run
    in reverse address order -> generic), 'padded' / 'padded_odd' (as
    packed / odd, 60 % of the packets with 1-39 bytes past ip_len)."""
    pkts = []
    for k in range(n):
        L = int(rng.choice([40, 64, 300, 576, 1500, 1501]))
        if kind == "empty" and k % 7 == 3:
            pkts.append(b"")
            continue
        ow = int(rng.integers(1, 6)) if rng.random() < 0.15 else 0
        p = fuzz.build(rng, proto, max(L, 28 + 4 * ow + 20), ow)
        if kind.startswith("padded") and rng.random() < 0.6:
            # bytes past ip_len / the transport length (link-layer padding):
            # the kernel re-reads the last chunk to take them out
            p = p + bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))
        pkts.append(p)
    off = np.zeros(n, np.uint64)
    pos = 0
    for k, p in enumerate(pkts):
        if kind in ("packed", "empty", "reversed", "padded"):
            pos = (pos + 63) // 64 * 64
        elif kind in ("odd", "padded_odd"):
            pos = (pos + 15) // 16 * 16 + 16 + 2 * int(rng.integers(0, 4)) + 1
        elif kind == "gaps" and k % 50 == 0:
            pos += 4096
        off[k] = pos
        pos += len(p)
    size = int(max(off[k] + len(p) for k, p in enumerate(pkts))) + 64
    arena = np.zeros(size, np.uint8)
    for k, p in enumerate(pkts):
        arena[int(off[k]):int(off[k]) + len(p)] = np.frombuffer(p, np.uint8)
    caplen = np.array([len(p) for p in pkts], np.uint32)
    if kind == "reversed":                         # every other 64-packet run in reverse address order
        for r0 in range(0, n, 128):
            off[r0:r0 + 64] = off[r0:r0 + 64][::-1].copy()
            caplen[r0:r0 + 64] = caplen[r0:r0 + 64][::-1].copy()
    oracle_lib.batch("set_ip", arena, n, off=off, length=caplen)
    if proto == 1:
        fuzz.set_icmp_checksums(arena, off, caplen)
    else:
        oracle_lib.batch("set_udp" if proto == 17 else "set_tcp", arena, n, off=off, length=caplen, arg=0)
    bad = rng.random(n) < 0.1                      # some corrupted payload bytes
    for k in np.nonzero(bad & (caplen > 60))[0]:
        arena[int(off[k]) + 50] ^= 0x40
    return arena, off, caplen, int(caplen.max())


@pytest.mark.parametrize("kind", ["packed", "odd", "empty", "gaps", "shared", "reversed", "padded", "padded_odd"])
@pytest.mark.parametrize("mode", [-1, 1])
def test_stream_dense_and_generic_runs(torch, kind, mode):
    """The packet-stream kernel's two per-run paths -- the dense span loaded
    coalesced through LDS (CLK_DENSE) and the per-packet chunk list -- on
    layouts that pick each (and mixes within one batch), with and without
    bytes past the transport length, Check and Set (fused and two-phase),
    every protocol: oracle-exact."""
    import click_amd
    c = click_amd.Context(0).tune(stream_min=1, set_mode=mode)
    rng = np.random.default_rng(hash(kind) % 1000 + mode)
    for proto in (17, 6, 1):
        arena, off, caplen, ml = dense_layout(rng, 700, proto, kind)
        for op in OPS_L4[proto]:
            compare(torch, c, op, arena, len(off), off=off, length=caplen, max_len=ml, arg=1)
        if proto == 6:
            compare(torch, c, "set_tcp", arena, len(off), off=off, length=caplen, max_len=ml, arg=0)
    c.close()


def test_empty_batches(torch, ctx):
    """n = 0 through every entry point (fixed stride, descriptors, packet
    stream): success, empty outputs, nothing written."""
    import click_amd
    arena = np.full(256, 0xA5, np.uint8)
    for kw in (dict(stride=64, fixed_len=46), dict(off=np.zeros(0, np.uint64), length=np.zeros(0, np.uint32),
                                                    max_len=1500)):
        for stream_min in (1, 100000000):
            c = click_amd.Context(0).tune(stream_min=stream_min)
            for op in ("in_cksum", "check_ip", "set_ip", "check_udp", "set_udp", "check_tcp", "set_tcp",
                       "check_icmp", "dec_ttl"):
                b = dev_batch(torch, arena, 0, **kw)
                codes, sums = run_gpu(c, op, b)
                c.sync()
                for t in (codes, sums):
                    assert t is None or t.numel() == 0, op
                assert np.array_equal(b.base.cpu().numpy(), arena), op
            c.close()


@pytest.mark.parametrize("stream_min,group", [(1, 0), (100000000, 0)])
def test_maximum_ip_length(torch, stream_min, group):
    """Packets at the largest IP total length (65535 B: a 65515 B UDP
    datagram / TCP segment) mixed with small ones, through the packet
    stream and the fixed 64-lane geometry: Check and Set (FIXOFF on and off)
    bit-exact against the oracle, every arena byte compared."""
    import click_amd
    c = click_amd.Context(0).tune(stream_min=stream_min, group=group)
    rng = np.random.default_rng(65535 + stream_min % 7)
    for proto in (17, 6):
        sizes = [65535, 65535, 64, 1500, 65535, 40000, 576] * 10
        pkts = [fuzz.build(rng, proto, t) for t in sizes]
        n = len(pkts)
        caplen = np.array([len(p) for p in pkts], np.uint32)
        off = np.zeros(n, np.uint64)
        pos = 0
        for i, p in enumerate(pkts):
            pos += int(rng.integers(0, 4)) * 16 + (i & 1)       # 16 B-aligned and odd starts
            off[i] = pos
            pos += len(p)
        arena = np.zeros(pos + 64, np.uint8)
        for i, p in enumerate(pkts):
            arena[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
        oracle_lib.batch("set_ip", arena, n, off=off, length=caplen)
        oracle_lib.batch(OPS_L4[proto][1], arena, n, off=off, length=caplen, arg=0)
        for i in range(0, n, 3):                                  # a third corrupted: Check must drop them
            arena[int(off[i]) + int(caplen[i]) - 1] ^= 0x10
        for op in OPS_L4[proto]:
            compare(torch, c, op, arena, n, off=off, length=caplen, max_len=int(caplen.max()), arg=1)
        compare(torch, c, OPS_L4[proto][1], arena, n, off=off, length=caplen, max_len=int(caplen.max()), arg=0)
    c.close()
