"""Multi-process (gloo, CPU) tests of the sharded path.

Each rank processes its contiguous shard of global packet indices with the
oracle (the GPU path runs the same shard logic over RCCL in bench.py); the
reduced digest must equal the single-process digest over all packets, i.e.
sharding changes nothing bit for bit, the time reduction takes the max and
keeps every rank's times, the Set checksums reach rank 0 only, and C4-style
variable-length shards are byte-balanced without any rank holding the whole
length array.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from click_amd import shard
from tests import oracle_lib

N_TOTAL, L, STRIDE = 3000, 1500, 1536


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_shard(lo, hi):
    n = hi - lo
    arena = np.zeros(n * STRIDE, np.uint8)
    oracle_lib.gen(arena, n, stride=STRIDE, fixed_len=L, proto=17, first_idx=lo)
    oracle_lib.batch("set_ip", arena, n, stride=STRIDE, fixed_len=L)
    codes, sums = oracle_lib.batch("set_udp", arena, n, stride=STRIDE, fixed_len=L)
    return torch.from_numpy(codes.copy()), torch.from_numpy(sums.astype(np.int64))


def imix_block(first, n):
    import bench
    return bench.imix_lengths(n, 0x5EED, first)


def worker(rank, world, port, q, n_imix):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.shard_range(rank, world, N_TOTAL)
    codes, sums = run_shard(lo, hi)
    dig = shard.digest(torch, codes, sums, lo)
    wall, kms, total, extra, per_rank = shard.reduce_results(torch, dist, "cpu", 1.0 + rank, 2.0 * (rank + 1), dig,
                                                             [rank + 1])
    allsums = shard.gather_results(torch, dist, "cpu", sums.to(torch.uint16))
    # byte-balanced shards of world * n_imix IMIX packets from per-rank blocks
    clo, chi = shard.balanced_cuts(torch, dist, "cpu", rank * n_imix, imix_block(rank * n_imix, n_imix))
    # unequal shard sizes gather too (the C4 shards)
    g2 = shard.gather_results(torch, dist, "cpu", torch.arange(clo, chi, dtype=torch.int64).to(torch.int16))
    rs = shard.root_scatter(torch, dist, "cpu", 1 << 16, reps=2)
    q.put((rank, lo, hi, wall, kms, total, None if allsums is None else allsums.numpy(), extra, per_rank,
           (clo, chi), None if g2 is None else g2.numpy(), rs))
    dist.barrier()
    dist.destroy_process_group()


def run_world(world, n_imix=5000):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q, n_imix)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda o: o[0])
    return out


@pytest.mark.parametrize("world", [2, 3, 8])        # 8: the driver's largest node, as gloo ranks
def test_sharded_digest_matches_single_process(world):
    n_imix = 5000
    out = run_world(world, n_imix)
    # shards are disjoint and cover every packet
    assert out[0][1] == 0 and out[-1][2] == N_TOTAL
    assert all(out[r][2] == out[r + 1][1] for r in range(world - 1))
    # max over ranks, and every rank's times in rank order
    assert all(o[3] == float(world) and o[4] == 2.0 * world for o in out)
    assert all(o[8] == [[1.0 + r, 2.0 * (r + 1)] for r in range(world)] for o in out)
    assert all(o[7] == [world * (world + 1) // 2] for o in out)
    codes, sums = run_shard(0, N_TOTAL)
    single = shard.digest(torch, codes, sums, 0)
    assert all(o[5] == single for o in out)
    assert single["ok"] == N_TOTAL
    # the gathered checksums are on rank 0 only: the whole batch's, in packet order
    assert all(o[6] is None for o in out[1:])
    assert out[0][6].dtype == np.uint16 and np.array_equal(out[0][6].astype(np.int64), sums.numpy())
    # byte-balanced IMIX shards: contiguous, covering, within one packet of the mean
    cuts = [o[9] for o in out]
    assert cuts[0][0] == 0 and cuts[-1][1] == world * n_imix
    assert all(cuts[r][1] == cuts[r + 1][0] for r in range(world - 1))
    lens = imix_block(0, world * n_imix)
    sizes = [int(lens[a:b].sum()) for a, b in cuts]
    assert max(abs(s - lens.sum() / world) for s in sizes) <= 1500
    assert out[0][10] is not None and np.array_equal(out[0][10], np.arange(world * n_imix).astype(np.int16))
    # root scatter: the same (max-over-ranks) time everywhere, root's bytes
    rs = [o[11] for o in out]
    assert all(r is not None and r == rs[0] for r in rs) and rs[0][1] == (1 << 16) * (world - 1) and rs[0][0] > 0


def test_shard_by_bytes_balances_imix():
    rng = np.random.default_rng(3)
    lens = rng.choice([64, 576, 1500], 100000, p=[7 / 12, 4 / 12, 1 / 12])
    parts = [shard.shard_by_bytes(r, 8, lens) for r in range(8)]
    assert parts[0][0] == 0 and parts[-1][1] == len(lens)
    assert all(parts[i][1] == parts[i + 1][0] for i in range(7))
    sizes = [int(lens[a:b].sum()) for a, b in parts]
    # each cut is the packet boundary nearest its byte target (within 750 B),
    # so a shard is within one packet (1500 B) of the mean
    assert max(abs(s - lens.sum() / 8) for s in sizes) <= 1500


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partition(world):
    parts = [shard.shard_range(r, world, 1001) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == 1001
    assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("wname,elements,proto,L", [
    ("c3", ("CheckUDPHeader", "SetUDPChecksum"), 17, 1500),
    ("c5", ("CheckTCPHeader", "SetTCPChecksum"), 6, 9000),
    ("c2", ("CheckIPHeader", "SetIPChecksum", "DecIPTTL", "IPOutputCombo"), 17, 46)])
def test_oracle_digest_matches_batch_digest(wname, elements, proto, L):
    """oracle_digest (what bench.py verifies the GPU against) equals
    shard.digest over the oracle's own per-packet batch results for the
    same work: the bench's preparation, corruption and element passes."""
    import bench
    first, n, runs = 12345, 700, 5
    stride = (L + 63) // 64 * 64
    host = oracle_lib.digest(elements, proto, first, n, fixed_len=L, ttl_runs=runs, threads=3)
    arena = np.zeros(n * stride, np.uint8)
    oracle_lib.gen(arena, n, stride=stride, fixed_len=L, proto=proto, first_idx=first)
    ip_c, ip_s = oracle_lib.batch("set_ip", arena, n, stride=stride, fixed_len=L)
    l4_c, l4_s = oracle_lib.batch("set_tcp" if proto == 6 else "set_udp", arena, n, stride=stride, fixed_len=L,
                                  arg=0)
    picks = bench.corrupt_picks(first, n)
    for e in elements:
        sums = None
        if e in ("SetUDPChecksum", "SetTCPChecksum"):
            codes, sums = l4_c, l4_s
        elif e == "SetIPChecksum":
            codes, sums = ip_c, ip_s
        elif e.startswith("Check"):
            a = arena.copy()
            for i in np.nonzero(picks)[0]:          # corrupt_kernel, restated
                g = first + int(i)
                h = int(oracle_lib.load_oracle().oracle_splitmix64(0xBAD ^ ((g * 0xD1B54A32D192ED03) & (2**64 - 1))))
                lo, hi = (12, 20) if e == "CheckIPHeader" else ((40 if L > 40 else 20), L)
                a[int(i) * stride + lo + (h >> 20) % (hi - lo)] ^= 1 << ((h >> 8) & 7)
            op = {"CheckIPHeader": "check_ip", "CheckUDPHeader": "check_udp", "CheckTCPHeader": "check_tcp"}[e]
            codes, _ = oracle_lib.batch(op, a, n, stride=stride, fixed_len=L)
            assert (codes != 0).sum() > 0
        else:
            a = arena.copy()
            a.reshape(n, stride)[:, 8] = 255
            oracle_lib.batch("set_ip", a, n, stride=stride, fixed_len=L)
            for _ in range(runs):
                if e == "DecIPTTL":
                    codes, _ = oracle_lib.batch("dec_ttl", a, n, stride=stride, fixed_len=L)
                else:
                    codes, _, _ = oracle_lib.ip_out_batch("ip_output_combo", a, n, stride=stride, fixed_len=L,
                                                          my_ip=0x18041A12, mtu=1500)
        d = shard.digest(torch, torch.from_numpy(codes.copy()),
                         None if sums is None else torch.from_numpy(sums.astype(np.int64)), first)
        assert d == host[e], e
