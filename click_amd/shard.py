"""Multi-GPU sharding of packet batches.

Packets are independent, so N ranks (one process per GPU) each take a
contiguous range of global packet indices and run the same kernels on their
own HBM shard: no collective in the data path.  After the timed region one
all-reduce of (max time) and one of a result digest verify the job.  The
helpers here are device-agnostic so the same code runs over RCCL (backend
"nccl", GPU tensors) in bench.py and over gloo (CPU tensors) in tests.
"""


def shard_range(rank, world, n_total):
    """[lo, hi) of global packet indices for `rank` (contiguous, balanced)."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


def shard_by_bytes(rank, world, lengths):
    """For variable-length batches: split so every rank gets about the same
    number of BYTES (prefix sum of lengths), not packets."""
    import numpy as np
    csum = np.cumsum(np.asarray(lengths, dtype=np.int64))
    total = int(csum[-1]) if len(csum) else 0
    cut = lambda r: int(np.searchsorted(csum, total * r // world, side="right")) if r < world else len(csum)
    lo = 0 if rank == 0 else cut(rank)
    return lo, cut(rank + 1)


def digest(torch, codes, sums=None):
    """Order-independent digest of a shard's results: (#ok, #packets,
    sum of u16 checksums, xor-fold of checksums) as int64."""
    ok = int((codes == 0).sum())
    n = int(codes.numel())
    if sums is not None:
        s = sums.to(torch.int64)
        total = int(s.sum())
        x = 0
        xv = s.cpu().numpy()
        import numpy as np
        x = int(np.bitwise_xor.reduce(xv)) if len(xv) else 0
    else:
        total, x = 0, 0
    return [ok, n, total, x]


def reduce_results(torch, dist, device, wall_s, kernel_ms, dig):
    """All-reduce the timing (MAX) and the digest (SUM / XOR) over ranks.
    dig = [ok, packets, sum16, xor16, extra counts...]: entry 3 is
    xor-folded, every other entry summed.  Returns (wall_s, kernel_ms,
    digest) as seen by every rank."""
    if dist is None:
        return wall_s, kernel_ms, list(dig)
    t = torch.tensor([wall_s, kernel_ms], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    summed = list(dig[:3]) + list(dig[4:])           # entries past the xor-fold are counts too
    d = torch.tensor(summed, dtype=torch.int64, device=device)
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    x = torch.tensor([dig[3]], dtype=torch.int64, device=device)
    gathered = [torch.zeros_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(gathered, x)
    xr = 0
    for g in gathered:
        xr ^= int(g.item())
    d = [int(v) for v in d.tolist()]
    return float(t[0]), float(t[1]), d[:3] + [xr] + d[3:]


def gather_results(torch, dist, device, values, root=0):
    """SURVEY §8(e) collective (2): every rank's per-packet results (the u16
    checksums a Set wrote) to `root`, in rank order -- the shards are
    contiguous global index ranges, so the concatenation is the whole
    batch's result array.  One all_gather over the communicator (RCCL over
    xGMI for the nccl backend; gloo on the CPU); equal shard sizes.
    Returns the concatenated tensor on `root`, None elsewhere."""
    if dist is None:
        return values
    # as bytes: neither RCCL nor gloo carries uint16
    src = values.to(device).contiguous().view(torch.uint8)
    parts = [torch.empty_like(src) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, src)
    return torch.cat(parts).view(values.dtype) if dist.get_rank() == root else None

