"""Multi-GPU sharding of packet batches.

Packets are independent, so N ranks (one process per GPU) each take a
contiguous range of global packet indices and run the same kernels on their
own HBM shard: no collective in the data path.  After the timed region one
all-reduce of (max time) and one of a result digest verify the job, and the
Set elements' checksums can be gathered to rank 0 (grouped send/recv).  The
helpers here are device-agnostic so the same code runs over RCCL (backend
"nccl", GPU tensors) in bench.py and over gloo (CPU tensors) in tests.
"""

# digest fields, in the order of the int64 vector the collectives carry;
# "xor16" is xor-folded over ranks, every other field summed
DIGEST_FIELDS = ("ok", "packets", "sum16", "xor16", "wsum16", "wcode")
W_MUL = 40503      # w(g) = (g * W_MUL) mod 2^16: the position weight (oracle_digest)


def shard_range(rank, world, n_total):
    """[lo, hi) of global packet indices for `rank` (contiguous, balanced)."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


def shard_by_bytes(rank, world, lengths):
    """For variable-length batches held in one array: split so every rank
    gets about the same number of BYTES (prefix sum of lengths), not packets
    (SURVEY §8e).  Each cut is the packet boundary nearest its byte target,
    so a shard's bytes differ from total / world by at most max(length)."""
    import numpy as np
    csum = np.cumsum(np.asarray(lengths, dtype=np.int64))
    total = int(csum[-1]) if len(csum) else 0

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return len(csum)
        return _nearest_cut(csum, total * r / world)
    return cut(rank), cut(rank + 1)


def _nearest_cut(csum, target):
    """Packet count c (0..len) whose byte prefix (csum[c-1], 0 for c = 0) is
    nearest `target`."""
    import numpy as np
    c = int(np.searchsorted(csum, target, side="right"))     # prefix(c) <= target < prefix(c + 1)
    lo = int(csum[c - 1]) if c > 0 else 0
    if c < len(csum) and int(csum[c]) - target < target - lo:
        c += 1
    return c


def balanced_cuts(torch, dist, device, block_first, block_lengths):
    """Byte-balanced contiguous shards of a batch held as per-rank blocks.

    Rank r holds the lengths of its count-based block of global packets
    [block_first, block_first + len(block_lengths)) (blocks are contiguous and
    in rank order).  One all_gather of the block byte totals gives every
    rank the global prefix at block boundaries; the rank whose block holds a
    cut's byte target finds the nearest packet boundary by a search of its
    own prefix sums, and one all_reduce shares the cuts.  Returns (lo, hi):
    this rank's global packet range; its bytes differ from total / world by
    at most the largest packet.  No rank holds the whole length array."""
    import numpy as np
    rank, world = dist.get_rank(), dist.get_world_size()
    csum = np.cumsum(np.asarray(block_lengths, dtype=np.int64))
    mine = torch.tensor([int(csum[-1]) if len(csum) else 0, block_first, len(csum)], dtype=torch.int64,
                        device=device)
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    tot = [int(p[0]) for p in parts]
    firsts = [int(p[1]) for p in parts]
    prefix = [0]
    for t in tot:
        prefix.append(prefix[-1] + t)
    total = prefix[-1]
    cuts = torch.zeros(world + 1, dtype=torch.int64, device=device)
    if rank == 0:
        cuts[0] = firsts[0]
    if rank == world - 1:
        cuts[world] = firsts[-1] + int(parts[-1][2])
    for k in range(1, world):
        target = total * k / world
        # the block holding the target: prefix[b] <= target < prefix[b + 1]
        b = max(i for i in range(world) if prefix[i] <= target) if target < total else world - 1
        if b == rank:
            cuts[k] = block_first + _nearest_cut(csum, target - prefix[b])
    dist.all_reduce(cuts, op=dist.ReduceOp.SUM)
    c = [int(x) for x in cuts.tolist()]
    return c[rank], c[rank + 1]


def digest(torch, codes, sums=None, first_idx=0):
    """Order-sensitive digest of a shard's results (the fields of
    DIGEST_FIELDS, as a dict of ints): #ok, #packets, sum and xor-fold of
    the u16 checksums, and the position-weighted sums of checksums and codes
    with w(g) = (g * 40503) mod 2^16 over global indices g -- the same
    digest oracle_digest computes on the host (tests/oracle_lib.digest)."""
    n = int(codes.numel())
    g = torch.arange(first_idx, first_idx + n, dtype=torch.int64, device=codes.device)
    w = (g * W_MUL) & 0xFFFF
    c = codes.to(torch.int64)
    d = {"ok": int((codes == 0).sum()), "packets": n, "wcode": int((c * w).sum())}
    if sums is not None:
        s = sums.to(torch.int64) & 0xFFFF
        d["sum16"] = int(s.sum())
        d["wsum16"] = int((s * w).sum())
        x = s.cpu().numpy()
        import numpy as np
        d["xor16"] = int(np.bitwise_xor.reduce(x)) if len(x) else 0
    else:
        d["sum16"] = d["wsum16"] = d["xor16"] = 0
    return d


def reduce_results(torch, dist, device, wall_s, kernel_ms, dig, extra=()):
    """Reduce over ranks: the timing to its MAX (and every rank's times, in
    rank order), the digest dict summed (xor16 xor-folded), and `extra`
    counts summed.  Returns (wall_s, kernel_ms, digest, extra, per_rank) as
    seen by every rank; per_rank = [[wall_s, kernel_ms], ...]."""
    if dist is None:
        return wall_s, kernel_ms, dict(dig), list(extra), [[wall_s, kernel_ms]]
    world = dist.get_world_size()
    t = torch.tensor([wall_s, kernel_ms], dtype=torch.float64, device=device)
    times = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(times, t)
    per_rank = [[float(x) for x in v.tolist()] for v in times]
    fields = [f for f in DIGEST_FIELDS if f != "xor16"]
    d = torch.tensor([dig[f] for f in fields] + list(extra), dtype=torch.int64, device=device)
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    x = torch.tensor([dig["xor16"]], dtype=torch.int64, device=device)
    xs = [torch.zeros_like(x) for _ in range(world)]
    dist.all_gather(xs, x)
    xr = 0
    for v in xs:
        xr ^= int(v.item())
    vals = [int(v) for v in d.tolist()]
    out = dict(zip(fields, vals[:len(fields)]))
    out["xor16"] = xr
    return (max(p[0] for p in per_rank), max(p[1] for p in per_rank), out, vals[len(fields):], per_rank)


def all_gather_ints(torch, dist, device, values):
    """Every rank's list of ints, in rank order (e.g. each shard's first
    packet, packets and bytes for the record)."""
    if dist is None:
        return [list(values)]
    t = torch.tensor(list(values), dtype=torch.int64, device=device)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [[int(x) for x in p.tolist()] for p in parts]


def gather_results(torch, dist, device, values, root=0):
    """SURVEY §8(e) collective (2): every rank's per-packet results (the u16
    checksums a Set wrote) to `root` only, in rank order -- the shards are
    contiguous global index ranges, so the concatenation is the whole
    batch's result array.  Shards may differ in length (byte-balanced C4):
    the sizes are all-gathered first, then one grouped send/recv
    (batch_isend_irecv: RCCL over xGMI for the nccl backend, gloo on the
    CPU) moves each shard once, into root.  Returns the concatenated tensor
    on `root`, None elsewhere."""
    if dist is None:
        return values
    rank, world = dist.get_rank(), dist.get_world_size()
    # as bytes: neither RCCL nor gloo carries uint16
    src = values.to(device).contiguous().view(torch.uint8)
    n = torch.tensor([src.numel()], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank == root:
        parts = [src if r == root else torch.empty(sizes[r], dtype=torch.uint8, device=device) for r in range(world)]
        ops = [dist.P2POp(dist.irecv, parts[r], r) for r in range(world) if r != root]
    else:
        parts = None
        ops = [dist.P2POp(dist.isend, src, root)]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return torch.cat(parts).view(values.dtype) if rank == root else None


def root_scatter(torch, dist, device, sample_bytes, reps=3, root=0):
    """an input that originates on one GPU (a single NIC) must
    first reach the other ranks.  `root` sends `sample_bytes` to every other
    rank in one grouped send/recv (RCCL point-to-point over xGMI: one piece
    per link), timed between barriers, `reps` times after one untimed round;
    returns (seconds of the slowest rank's median round, bytes root sent per
    round), the same on every rank, or None without a process group of two
    or more.  Kept out of the device-resident metric: the caller reports it
    beside the time the whole shards would take at that rate."""
    if dist is None or dist.get_world_size() < 2:
        return None
    import time
    rank, world = dist.get_rank(), dist.get_world_size()
    sync = (lambda: torch.cuda.synchronize()) if str(device).startswith("cuda") else (lambda: None)
    if rank == root:
        buf = torch.empty(sample_bytes * (world - 1), dtype=torch.uint8, device=device)
        peers = [r for r in range(world) if r != root]
        ops = [dist.P2POp(dist.isend, buf[k * sample_bytes:(k + 1) * sample_bytes], r) for k, r in enumerate(peers)]
    else:
        buf = torch.empty(sample_bytes, dtype=torch.uint8, device=device)
        ops = [dist.P2POp(dist.irecv, buf, root)]
    times = []
    for it in range(reps + 1):
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        sync()
        dt = time.perf_counter() - t0
        if it:
            times.append(dt)
    times.sort()
    t = torch.tensor([times[len(times) // 2]], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), sample_bytes * (world - 1)
