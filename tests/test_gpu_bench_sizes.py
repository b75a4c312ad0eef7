"""GPU tests at the bench's own sizes (BASELINE configs 4 and 5) and of the
bench's multi-rank path.

* C4: the full 64M-packet IMIX batch of bench.py (64/576/1500 B, 7:4:1,
  packed at 64 B-aligned offsets) through the packet-stream kernels: Set
  then Check pass everywhere, the Set's checksums and the corrupted
  Check's verdicts of the WHOLE batch match the host oracle's digest, a
  random sample matches the oracle byte for byte, and one flipped bit in
  1/1024 packets is caught exactly on those
  packets (except where SetUDPChecksum stored uh_sum = 0, which
  CheckUDPHeader does not verify: checkudpheader.cc:100).
* C5: one GPU's 16M x 9000 B TCP shard (128M over 8 GPUs), same checks.
* bench.py --gpus 2 (two gloo ranks on GPU 0) reports n_gpus 2 and the
  same digest as one rank over both shards.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def oracle_packet(L, proto, idx):
    ref = np.zeros(L, np.uint8)
    oracle_lib.gen(ref, 1, fixed_len=L, proto=proto, first_idx=idx)
    oracle_lib.batch("set_ip", ref, 1, fixed_len=L)
    oracle_lib.batch("set_udp" if proto == 17 else "set_tcp", ref, 1, fixed_len=L, arg=0)
    return ref


def check_full_batch(torch, ctx, b, n, proto, off_np, len_np, sample=384, fixed_len=0, imix=False):
    import bench
    from click_amd import shard
    check_el, set_el = ("CheckUDPHeader", "SetUDPChecksum") if proto == 17 else ("CheckTCPHeader", "SetTCPChecksum")
    # the host oracle's digest of the whole batch (as bench.py's verify), Set and corrupted Check
    od = oracle_lib.digest([check_el, set_el], proto, 0, n, fixed_len=fixed_len, imix=imix,
                           threads=bench.verify_threads(1))
    st, _ = ctx.set_ip_checksum(b, want_sums=False)
    assert int(ctx.count_codes(st)[0]) == n
    st, sums = ctx.set_udp_checksum(b) if proto == 17 else ctx.set_tcp_checksum(b)
    assert int(ctx.count_codes(st)[0]) == n
    gd = shard.digest(torch, st, sums, 0)
    assert {f: gd[f] for f in shard.DIGEST_FIELDS} == od[set_el], (gd, od[set_el])
    v = ctx.check_udp_header(b) if proto == 17 else ctx.check_tcp_header(b)
    assert int(ctx.count_codes(v)[0]) == n
    assert int(ctx.count_codes(ctx.check_ip_header(b))[0]) == n
    # a sample of packets, byte for byte against the oracle
    rng = np.random.default_rng(proto * 1000 + n % 997)
    idx = np.sort(rng.choice(n, sample, replace=False))
    for i in idx:
        o, L = int(off_np[i]), int(len_np[i])
        got = b.base[o:o + L].cpu().numpy()
        assert np.array_equal(got, oracle_packet(L, proto, int(i))), "packet %d" % i
    # corruption caught exactly (the bench's timed Check batches)
    picks = bench.corrupt_picks(0, n)
    ctx.gen_corrupt(b, seed=bench.CORRUPT_SEED, rate_log2=bench.CORRUPT_LOG2, first_idx=0)
    vt = ctx.check_udp_header(b) if proto == 17 else ctx.check_tcp_header(b)
    gd = shard.digest(torch, vt, None, 0)
    assert {f: gd[f] for f in shard.DIGEST_FIELDS} == od[check_el], (gd, od[check_el])
    v = vt.cpu().numpy()
    detect = picks & (sums.cpu().numpy() != 0) if proto == 17 else picks
    assert detect.sum() > 0
    assert np.array_equal(v == 3, detect)
    assert np.array_equal(v == 0, ~detect)
    ctx.gen_corrupt(b, seed=bench.CORRUPT_SEED, rate_log2=bench.CORRUPT_LOG2, first_idx=0)   # restore
    v = ctx.check_udp_header(b) if proto == 17 else ctx.check_tcp_header(b)
    assert int(ctx.count_codes(v)[0]) == n


def test_c4_full_imix_batch(torch, ctx):
    import bench
    import click_amd
    n = bench.WORKLOADS["c4"]["n"]
    off, ln, total, _ = bench.imix_layout(torch, n, 0x5EED, 0)
    arena = torch.empty(total, dtype=torch.uint8, device="cuda")
    b = click_amd.Batch(arena, n, off=off, length=ln, max_len=1500)
    ctx.gen_packets(b, proto=17)
    try:
        check_full_batch(torch, ctx, b, n, 17, off.cpu().numpy(), ln.cpu().numpy(), imix=True)
    finally:
        del arena, b
        torch.cuda.empty_cache()


def test_c5_full_jumbo_shard(torch, ctx):
    import bench
    import click_amd
    w = bench.WORKLOADS["c5"]
    n, L, stride = w["n"], w["L"], w["stride"]
    arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
    ctx.gen_packets(b, proto=6)
    try:
        check_full_batch(torch, ctx, b, n, 6, np.arange(n, dtype=np.uint64) * np.uint64(stride),
                         np.full(n, L, np.uint32), sample=128, fixed_len=L)
    finally:
        del arena, b
        torch.cuda.empty_cache()


def run_bench(gpus, packets, skip="c4,c5", extra_env=None):
    env = dict(os.environ, CLK_BENCH_SAME_DEVICE="1", CLK_BENCH_BACKEND="gloo", **(extra_env or {}))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--packets", str(packets),
           "--steps", "2", "--warmup", "1", "--no-c2", "--no-c1", "--no-cpu", "--no-peak", "--no-frag",
           "--skip", skip, "--scatter-bytes", str(1 << 20)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def without_timing(v):
    v = dict(v)
    o = dict(v.pop("oracle"))
    o.pop("oracle_s_rank0", None)
    return v, o


def test_bench_two_ranks_match_one(torch):
    """bench.py --gpus 2 launches two ranks itself (no WORLD_SIZE), reports
    n_gpus 2, per-rank times and shards, the reduced digests equal one
    rank's over both shards and the host oracle's (full batch), the Set's
    checksums reach rank 0 only, and the C4 shards are byte-balanced."""
    n = 1 << 17
    two = run_bench(2, n, skip="c5")
    one = run_bench(1, 2 * n, skip="c5")
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["packets_per_gpu"] == n
    # the root-scatter sample (an input starting on one GPU), N > 1 only
    rs = two["root_scatter"]
    assert rs["sample_bytes_per_rank"] == 1 << 20 and rs["seconds"] > 0 and "root_scatter" not in one
    for sect, elements in ((None, ("CheckUDPHeader", "SetUDPChecksum")),
                           ("c4_imix", ("CheckUDPHeader", "SetUDPChecksum"))):
        t_el = two["elements"] if sect is None else two[sect]["elements"]
        o_el = one["elements"] if sect is None else one[sect]["elements"]
        for e in elements:
            tv, to = without_timing(t_el[e]["verify"])
            ov, oo = without_timing(o_el[e]["verify"])
            assert tv == ov, (sect, e)
            assert to == oo and to["oracle_match"] is True and to["full_batch"] is True, (sect, e, to)
            assert tv["packets"] == 2 * n
            pr = t_el[e]["per_rank"]
            assert len(pr) == 2 and "per_rank" not in o_el[e]
            assert max(p["kernel_ms"] for p in pr) == t_el[e]["roofline"]["kernel_ms"]
        chk = t_el["CheckUDPHeader"]["verify"]
        assert chk["drops_exact"] and chk["drops"] > 0
        # the Set's checksums gathered to rank 0 only, agreeing with the reduced digest
        g = t_el["SetUDPChecksum"]["gather_to_rank0"]
        assert g.get("matches_digest") is True and g.get("on_root_only") is True, g
        assert "gather_to_rank0" not in o_el["SetUDPChecksum"]
    # C4: byte-balanced shards of the 2n-packet IMIX batch
    pr = two["c4_imix"]["elements"]["CheckUDPHeader"]["per_rank"]
    assert pr[0]["first"] == 0 and pr[1]["first"] == pr[0]["packets"] and pr[0]["packets"] + pr[1]["packets"] == 2 * n
    mean = (pr[0]["bytes"] + pr[1]["bytes"]) / 2
    assert all(abs(p["bytes"] - mean) <= 1500 for p in pr), pr


def test_bench_rccl_one_rank(torch):
    """The RCCL (nccl backend) code path of bench.py on one GPU: the
    communicator with one rank (device-bound init, barriers, all-reduce and
    all-gather of device tensors, C4's byte-balanced cuts, the grouped
    send/recv of the gather to rank 0) gives the same digests as the run
    without a communicator, and the oracle matches."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    n = 1 << 17
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CLK_BENCH_DIST_WORLD1="1")
    env.pop("CLK_BENCH_BACKEND", None)
    env.pop("CLK_BENCH_SAME_DEVICE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--packets", str(n),
           "--steps", "2", "--warmup", "1", "--no-c2", "--no-c1", "--no-cpu", "--no-peak", "--no-frag",
           "--skip", "c5"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rccl = json.loads(lines[0])
    plain = run_bench(1, n, skip="c5")
    assert rccl["n_gpus"] == 1 and rccl["clk_env"].get("CLK_BENCH_DIST_WORLD1") == "1"
    for sect in (None, "c4_imix"):
        r_el = rccl["elements"] if sect is None else rccl[sect]["elements"]
        p_el = plain["elements"] if sect is None else plain[sect]["elements"]
        for e in ("CheckUDPHeader", "SetUDPChecksum"):
            rv, ro = without_timing(r_el[e]["verify"])
            pv, po = without_timing(p_el[e]["verify"])
            assert rv == pv and ro == po and ro["oracle_match"] is True, (sect, e)
        g = r_el["SetUDPChecksum"]["gather_to_rank0"]
        assert g.get("matches_digest") is True and g.get("on_root_only") is True, g
