"""Multi-process (gloo, world_size 2, CPU) tests of the sharded path.

Each rank processes its contiguous shard of global packet indices with the
oracle (the GPU path runs the same shard logic over RCCL in bench.py); the
reduced digest must equal the single-process digest over all packets, i.e.
sharding changes nothing bit for bit, and the time reduction takes the max.
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


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.shard_range(rank, world, N_TOTAL)
    codes, sums = run_shard(lo, hi)
    dig = shard.digest(torch, codes, sums)
    wall, kms, total = shard.reduce_results(torch, dist, "cpu", 1.0 + rank, 2.0 * (rank + 1), dig)
    allsums = shard.gather_results(torch, dist, "cpu", sums.to(torch.uint16))
    q.put((rank, lo, hi, wall, kms, total, None if allsums is None else allsums.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_digest_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    # shards are disjoint and cover every packet
    assert out[0][1] == 0 and out[0][2] == out[1][1] and out[1][2] == N_TOTAL
    # max over ranks
    assert all(o[3] == 2.0 and o[4] == 4.0 for o in out)
    codes, sums = run_shard(0, N_TOTAL)
    single = shard.digest(torch, codes, sums)
    assert out[0][5] == single and out[1][5] == single
    assert single[0] == N_TOTAL
    # the gathered checksums on rank 0 are the whole batch's, in packet order
    assert out[1][6] is None
    assert out[0][6].dtype == np.uint16 and np.array_equal(out[0][6].astype(np.int64), sums.numpy())


def test_shard_by_bytes_balances_imix():
    rng = np.random.default_rng(3)
    lens = rng.choice([64, 576, 1500], 100000, p=[7 / 12, 4 / 12, 1 / 12])
    parts = [shard.shard_by_bytes(r, 8, lens) for r in range(8)]
    assert parts[0][0] == 0 and parts[-1][1] == len(lens)
    assert all(parts[i][1] == parts[i + 1][0] for i in range(7))
    sizes = [int(lens[a:b].sum()) for a, b in parts]
    assert max(sizes) - min(sizes) <= 1500


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partition(world):
    parts = [shard.shard_range(r, world, 1001) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == 1001
    assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
