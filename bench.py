#!/usr/bin/env python3
"""Benchmark of the MI355X checksum path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]

One step = one pass of one element over one device-resident batch (inputs
generated in HBM before timing).  Default workload C3: 16M x 1500 B
UDP/IPv4 packets in 1536 B slots per GPU; the headline element is
CheckUDPHeader (full-payload checksum + verdict, read-bound), and
SetUDPChecksum (checksum written in place) is timed beside it under
"elements".  The 64 B min-size batch (C2: CheckIPHeader and SetIPChecksum
over 16M packets in 64 B slots) is measured in the same run under "c2_64b"
because the metric names both sizes; the IMIX (C4, "c4_imix") and 9000 B
(C5, "c5_jumbo": 16M per GPU, 128M at 8 GPUs) configurations and the
IPFragmenter (C3 to MTU 576, "fragmenter") follow.
Multi-GPU (torchrun, one process per GPU): every rank generates and
processes its own shard of global packet indices -- packets are independent,
so there is no collective in the data path (weak scaling); one RCCL
all-reduce after the timed region takes the max time and a result digest.

Rank 0 prints ONE JSON line.  roofline.achieved = algorithmic bytes per
launch / mean kernel time from HIP events recorded on the stream the kernel
runs on; roofline.traffic = HBM bytes per launch from the committed
rocprofv3 PMC summary (profiles/pmc_<workload>.json) when present.
cpu_baseline: the oracle restatement of lib/in_cksum.c + the element (-O2 -g)
on the host cores, on a bounded sample of the same workload.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s checksummed (device-resident) + Mpps, 64B and 1500B packet batches"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
GIB = float(1 << 30)

# workload: protocol, packet bytes L, slot stride, packets per GPU, bytes
# "checksummed" per packet (the metric's numerator), and the elements timed:
# the first is the headline, the others are reported beside it.  Algorithmic
# HBM bytes per packet per element: Check = L read + 1 verdict byte;
# Set = L read + 2 field bytes + 1 status byte (CheckIPHeader/SetIPChecksum
# read the 20 B header, not the slot).
WORKLOADS = {
    "c3": dict(proto=17, L=1500, stride=1536, n=16 << 20, ck=1500,
               elements=("CheckUDPHeader", "SetUDPChecksum"),
               desc="C3: 1500 B UDP/IPv4 full-payload checksum, 16M-packet batch per GPU, 1536 B slots"),
    "c2": dict(proto=17, L=46, stride=64, n=16 << 20, ck=20,
               elements=("CheckIPHeader", "SetIPChecksum", "DecIPTTL", "IPOutputCombo"),
               desc="C2: 64 B min-size packets (IP length 46, 64 B slots), IP-header checksum, 16M-packet batch per GPU"),
    "c5": dict(proto=6, L=9000, stride=9024, n=16 << 20, ck=9000,
               elements=("CheckTCPHeader", "SetTCPChecksum"),
               desc="C5: 9000 B jumbo TCP/IPv4 checksum, 16M packets per GPU (128M over 8 GPUs)"),
    "c4": dict(proto=17, L=0, stride=0, n=64 << 20, ck=None,
               elements=("CheckUDPHeader", "SetUDPChecksum"),
               desc="C4: IMIX 64/576/1500 (7:4:1) UDP/IPv4 checksum, 64M packets, 64 B-aligned packing"),
}
ALG = {"CheckUDPHeader": lambda L: L + 1, "CheckTCPHeader": lambda L: L + 1, "CheckIPHeader": lambda L: 20 + 1,
       "SetUDPChecksum": lambda L: L + 3, "SetTCPChecksum": lambda L: L + 3, "SetIPChecksum": lambda L: 20 + 3,
       "DecIPTTL": lambda L: 3 + 3 + 1,   # ip_ttl + ip_sum read and written, status (MULTICAST true)
       "IPOutputCombo": lambda L: 1 + 3 + 3 + 1}   # + ip_hl byte; no options, no FIX_IP_SRC
# element-glue configuration for elements with mandatory arguments
ELEMENT_CONF = {"IPOutputCombo": "1, 18.26.4.24, 1500"}
# C2 slot traffic per packet beyond the 64 B slot read: status + written field bytes
SLOT_EXTRA = {"CheckIPHeader": 1, "SetIPChecksum": 3, "DecIPTTL": 4, "IPOutputCombo": 4}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def imix_lengths(n, seed, first_idx):
    """C4 packet lengths 64/576/1500 with P = 7/12, 4/12, 1/12, by a hash of
    the global packet index (the same hash as oracle/cksum_oracle.c
    imix_len)."""
    import numpy as np
    i = np.arange(first_idx, first_idx + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = i * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    r = (x % np.uint64(12)).astype(np.int64)
    return np.where(r < 7, 64, np.where(r < 11, 576, 1500)).astype(np.int64)


def imix_layout(torch, n, seed, first_idx):
    """C4 packets [first_idx, first_idx + n) packed at 64 B-aligned offsets.
    Returns (off int64, len int32, arena bytes, sum L)."""
    import numpy as np
    L = imix_lengths(n, seed, first_idx)
    slot = (L + 63) // 64 * 64
    off = np.zeros(n, np.int64)
    np.cumsum(slot[:-1], out=off[1:])
    total = int(off[-1] + slot[-1])
    return (torch.from_numpy(off).cuda(), torch.from_numpy(L.astype(np.int32)).cuda(), total, int(L.sum()))


# Host-oracle verification of every timed element:
# nanoseconds of one host thread per packet byte for oracle_digest (gen +
# the Set and Check passes), used to size the verified range to the budget
ORACLE_NS_PER_BYTE = 1.3
VERIFY_BUDGET_S = float(os.environ.get("CLK_VERIFY_BUDGET_S", 20))     # bench-side: per workload and rank


class OracleVerify:
    """The oracle's digest (tests/oracle_lib.digest over oracle/cksum_oracle.c
    oracle_digest) of exactly this rank's work -- global packets
    [first, first + m), m = n or the prefix that fits VERIFY_BUDGET_S on
    `threads` host threads -- run after the workload's timed regions (start()
    then join()), never beside them: with the oracle's threads using the
    box's whole CPU quota, the cgroup throttled the launching thread and the
    GPU idled inside a timed region (C4 Check: 4.22 ms per step around
    3.79 ms kernels, profiles/r03/bench_overlap_note.txt)."""

    def __init__(self, wname, elements, first, n, ttl_runs, threads):
        import threading
        w = WORKLOADS[wname]
        mean_len = 354.33 if wname == "c4" else w["L"]
        fit = int(VERIFY_BUDGET_S * 1e9 * threads / (ORACLE_NS_PER_BYTE * (mean_len + 64)))
        self.m = min(n, max(fit, 1 << 16))
        self.first, self.elements, self.result, self.error = first, elements, None, None
        self.secs = None
        kw = dict(elements=list(elements), proto=w["proto"], first_idx=first, n=self.m, fixed_len=w["L"],
                  imix=wname == "c4", corrupt_seed=CORRUPT_SEED, corrupt_log2=CORRUPT_LOG2, ip_span=(12, 20),
                  ttl_runs=ttl_runs, my_ip=0x18041A12, mtu=1500, threads=threads)

        def run():
            try:
                from tests import oracle_lib
                t0 = time.perf_counter()
                self.result = oracle_lib.digest(**kw)
                self.secs = time.perf_counter() - t0
            except Exception as e:            # reported in the record
                self.error = repr(e)
        self.t = threading.Thread(target=run, daemon=True)

    def start(self):
        self.t.start()

    def join(self):
        self.t.join()
        return self.result


def verify_threads(world):
    """Host threads for the oracle digest of one rank: the CPUs this process
    may use (cgroup quota), shared by the node's ranks, one left for the
    rank's launching thread."""
    topo = host_topology()
    ncpu = len(topo["cpus"])
    if topo["quota"]:
        ncpu = min(ncpu, max(1, int(topo["quota"])))
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return max(1, ncpu // max(1, local) - 1)


def run_element(ctx, name, b, status):
    if name == "SetUDPChecksum":
        ctx.set_udp_checksum(b, status=status, want_sums=False)
    elif name == "SetTCPChecksum":
        ctx.set_tcp_checksum(b, status=status, want_sums=False)
    elif name == "SetIPChecksum":
        ctx.set_ip_checksum(b, status=status, want_sums=False)
    elif name == "CheckUDPHeader":
        ctx.check_udp_header(b, out=status)
    elif name == "CheckTCPHeader":
        ctx.check_tcp_header(b, out=status)
    elif name == "CheckIPHeader":
        ctx.check_ip_header(b, out=status)
    elif name == "DecIPTTL":
        ctx.dec_ip_ttl(b, status=status, want_sums=False)
    elif name == "IPOutputCombo":          # IPOutputCombo(1, 18.26.4.24, 1500)
        ctx.ip_output_combo(b, 0x18041A12, 1500, port=status, want_problem=False, want_sums=False)
    else:
        raise ValueError(name)


def load_torch_kernels(torch):
    """Run once, on tiny tensors, the torch operations measure() issues
    between a workload's GPU preparation and its warm-ups (a strided byte
    fill, a clone): the first use of a torch kernel in a process loads its
    code object, tens of milliseconds in which the GPU idles and drops its
    clocks right before a warm-up."""
    x = torch.zeros(64 * 64, dtype=torch.uint8, device="cuda")
    x.view(64, 64)[:, 8] = 255
    y = x.clone()
    z = torch.zeros(64, dtype=torch.uint16, device="cuda")
    int((y[:64].bool() & (z.view(torch.int16) != 0)).sum())
    torch.cuda.synchronize()


def measure(torch, ctx, dist, rank, world, wname, steps, warmup, seed=0x5EED, packets=None, coll_dev="cuda",
            verify=True):
    """Generate the shard in HBM, make every checksum valid (untimed), then
    time each of the workload's elements: warmup + `steps` launches between
    barriers + synchronize; HIP events on the launch stream give the kernel
    time.  Check elements run over a batch with 1 in 1024 packets corrupted
    (one flipped bit), so the drop path is inside the timed
    region; the corruption is undone before the next element.
    Shards: contiguous global packet ranges; C4's are byte-balanced
    (shard.balanced_cuts).  verify: the host oracle's digest of this rank's
    packets (OracleVerify) is compared with the GPU's after the reduction.
    Returns {element: result}."""
    import click_amd
    from click_amd import shard
    w = dict(WORKLOADS[wname])
    n = packets or w["n"]
    if wname == "c4":
        first = 0
        if dist is not None:       # byte-balanced shards of the world * n packet batch
            first, hi = shard.balanced_cuts(torch, dist, coll_dev, rank * n, imix_lengths(n, seed, rank * n))
            n = hi - first
        off, ln, total, sum_l = imix_layout(torch, n, seed, first)
        arena = torch.empty(total, dtype=torch.uint8, device="cuda")
        b = click_amd.Batch(arena, n, off=off, length=ln, max_len=1500)
        ck_bytes = sum_l
        alg = {e: (sum_l + (ALG[e](0)) * n + 12 * n) for e in w["elements"]}   # + descriptor (off u64, len u32)
    else:
        first, _ = shard.shard_range(rank, world, n * world)   # this rank's global packet indices
        arena = torch.empty(n * w["stride"], dtype=torch.uint8, device="cuda")
        b = click_amd.Batch(arena, n, stride=w["stride"], fixed_len=w["L"])
        ck_bytes = w["ck"] * n
        alg = {e: ALG[e](w["L"]) * n for e in w["elements"]}
    shards = shard.all_gather_ints(torch, dist, coll_dev, [first, n, ck_bytes])   # [first, packets, bytes] per rank
    ver = OracleVerify(wname, w["elements"], first, n, warmup + steps, verify_threads(world)) if verify else None
    # host-side preparation first: the GPU work from generation through the
    # last timed element then runs back to back, so the GPU does not idle
    # (and drop its clocks) between the preparation and a warm-up
    picks = corrupt_picks(first, n)
    n_picks = int(picks.sum())
    picks_t = torch.from_numpy(picks).to("cuda")
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.reserve(n)
    ctx.gen_packets(b, proto=w["proto"], seed=seed, first_idx=first)
    ctx.set_ip_checksum(b, status=status, want_sums=False)
    l4sums = torch.empty(n, dtype=torch.uint16, device="cuda")
    (ctx.set_tcp_checksum if w["proto"] == 6 else ctx.set_udp_checksum)(b, status=status, sums=l4sums)
    stream = torch.cuda.current_stream()
    timed = []
    for e in w["elements"]:
        if e in ("DecIPTTL", "IPOutputCombo"):
            # untimed: TTL 255 so that every timed pass decrements (<= 254 passes)
            arena.view(n, w["stride"])[:, 8] = 255
            ctx.set_ip_checksum(b, status=status, want_sums=False)
        corrupt = None
        expect = 0
        if e.startswith("Check"):
            # IP: a bit of ip_src/ip_dst (only the checksum can see it);
            # L4: a payload bit (CheckUDPHeader skips uh_sum == 0,
            # checkudpheader.cc:100, so those picks pass)
            corrupt = dict(seed=CORRUPT_SEED, rate_log2=CORRUPT_LOG2, first_idx=first,
                           lo=12 if e == "CheckIPHeader" else None, hi=20 if e == "CheckIPHeader" else 0)
            ctx.gen_corrupt(b, **corrupt)
            expect = "picks with uh_sum != 0" if e == "CheckUDPHeader" else n_picks    # counted after the timing
        for _ in range(warmup):
            run_element(ctx, e, b, status)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            ev[k][0].record(stream)
            run_element(ctx, e, b, status)
            ev[k][1].record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if dist:
            dist.barrier()
        # untimed, on the GPU only (the host work waits until every element
        # of the workload is timed): the Set's checksums as it wrote them,
        # this element's outputs kept, the corruption undone
        sums = None
        if e.startswith("Set"):
            sums = torch.empty(n, dtype=torch.uint16, device="cuda")
            {"SetUDPChecksum": ctx.set_udp_checksum, "SetTCPChecksum": ctx.set_tcp_checksum,
             "SetIPChecksum": ctx.set_ip_checksum}[e](b, status=status, sums=sums)
        codes = status.clone()
        if corrupt:
            ctx.gen_corrupt(b, **corrupt)             # flip the same bits back (untimed)
        timed.append((e, wall, ev, codes, sums, expect))
    torch.cuda.synchronize()
    out = {}
    for e, wall, ev, codes, sums, expect in timed:
        kms = [a.elapsed_time(z) for a, z in ev]
        kernel_ms = sum(kms) / len(kms)
        expect_drops = int((picks_t & (l4sums.view(torch.int16) != 0)).sum()) if isinstance(expect, str) else expect
        dig = shard.digest(torch, codes, sums, first)
        # the same digest over the oracle-verified prefix of the shard
        m = ver.m if ver else 0
        sub = shard.digest(torch, codes[:m], None if sums is None else sums[:m], first) if ver else None
        wall, kernel_ms, dig, (expect_drops,), per_rank = shard.reduce_results(
            torch, dist, coll_dev, wall, kernel_ms, dig, [expect_drops])
        if sub is not None:
            _, _, sub, _, _ = shard.reduce_results(torch, dist, coll_dev, 0.0, 0.0, sub)
        gather = None
        if dist is not None and sums is not None:
            # SURVEY §8(e) (2), untimed for the metric: every rank's checksums
            # to rank 0 only (grouped send/recv), checked against the digest
            try:
                dist.barrier()
                torch.cuda.synchronize()
                tg = time.perf_counter()
                allsums = shard.gather_results(torch, dist, coll_dev, sums)
                torch.cuda.synchronize()
                g_ms = (time.perf_counter() - tg) * 1e3
                gather = {"bytes_into_root": 2 * (dig["packets"] - n), "ms": round(g_ms, 3),
                          "GBs_into_root": round(2 * (dig["packets"] - n) / (g_ms * 1e-3) / 1e9, 1),
                          "on_root_only": (allsums is not None) == (rank == 0)}
                if allsums is not None:
                    gather["matches_digest"] = (int(allsums.to(torch.int64).sum()) == dig["sum16"]
                                                and int(allsums.numel()) == dig["packets"])
            except Exception as ex:             # reported, not fatal
                gather = {"error": repr(ex)}
        out[e] = dict(wall=wall, kernel_ms=kernel_ms, kernel_ms_min=min(kms), n=n, ck_bytes=ck_bytes,
                      alg_bytes=alg[e], w=w, element=e, ok_total=dig["ok"], n_total=dig["packets"],
                      per_rank=per_rank, sub=sub, shards=shards,
                      digest=dict(dig, drops=dig["packets"] - dig["ok"], expected_drops=expect_drops,
                                  drops_exact=dig["packets"] - dig["ok"] == expect_drops),
                      gather=gather)
    del timed, picks_t
    del arena, status, b, l4sums
    torch.cuda.empty_cache()
    if ver:
        ver.start()
        res = ver.join()
        for e, r in out.items():
            o = oracle_check(torch, dist, coll_dev, ver, res, e, r["sub"])
            if "verified_packets" in o:
                o["full_batch"] = o["verified_packets"] == r["digest"]["packets"]
            r["digest"]["oracle"] = o
    return out


def oracle_check(torch, dist, coll_dev, ver, res, e, sub):
    """Reduce this rank's oracle digest of element e over ranks (every rank
    joins the same collectives, with an error flag) and compare it field by
    field with the GPU's digest of the same packets."""
    from click_amd import shard
    err = 1 if res is None else 0
    od = {f: 0 if err else res[e][f] for f in shard.DIGEST_FIELDS}
    _, _, od, (m_all, errs), _ = shard.reduce_results(torch, dist, coll_dev, 0.0, 0.0, od, [ver.m, err])
    if errs:
        return {"error": ver.error or "oracle digest failed on %d rank(s)" % errs}
    return {"oracle_match": od == sub, "verified_packets": m_all, "host_digest": od,
            "oracle_s_rank0": round(ver.secs or 0, 2)}


CORRUPT_SEED, CORRUPT_LOG2 = 0xBAD, 10


def corrupt_picks(first, n, seed=CORRUPT_SEED, rate_log2=CORRUPT_LOG2):
    """The packets clk_gen_corrupt_span picks (cksum_kernels.hh corrupt_kernel):
    the low rate_log2 bits of splitmix64(seed ^ (first + i) * C) are zero."""
    import numpy as np
    i = np.arange(first, first + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) ^ (i * np.uint64(0xD1B54A32D192ED03))) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z & np.uint64((1 << rate_log2) - 1)) == 0


def measure_fragmenter(torch, ctx, dist, rank, world, steps, warmup, mtu=576, seed=0x5EED, packets=None,
                       coll_dev="cuda"):
    """IPFragmenter(MTU 576, HONOR_DF true) over the C3 batch (16M x 1500 B
    per GPU): every packet becomes a 572 B first fragment rewritten in place
    plus 572 B and 396 B fragments appended to an HBM arena (16 B-aligned
    slots).  The first-fragment header fields are restored between steps
    (outside the HIP events); the numbers are kernel-time based.
    Algorithmic bytes per packet: the 20 B header and the 928 payload bytes
    the appended fragments carry are read (the first fragment's payload
    stays in place); 968 B of fragments are appended and 8 header bytes
    rewritten in place: 1924 B."""
    import click_amd
    from click_amd import shard
    w = WORKLOADS["c3"]
    n, L, stride = packets or w["n"], w["L"], w["stride"]
    first, _ = shard.shard_range(rank, world, n * world)
    arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
    ctx.gen_packets(b, proto=17, seed=seed, first_idx=first)
    ctx.set_ip_checksum(b, want_sums=False)
    hdr = arena.view(n, stride)[:, :12]
    saved = hdr.clone()
    out = torch.empty(n * (576 + 400), dtype=torch.uint8, device="cuda")
    port = torch.empty(n, dtype=torch.uint8, device="cuda")
    first_len = torch.empty(n, dtype=torch.int32, device="cuda")
    frag_first = torch.empty(n, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    r = None
    for _ in range(warmup):
        hdr.copy_(saved)
        r = ctx.ip_fragment(b, mtu, True, arena=out, max_frags=2 * n, port=port, first_len=first_len,
                            frag_first=frag_first)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    for k in range(steps):
        hdr.copy_(saved)
        ev[k][0].record(stream)
        r = ctx.ip_fragment(b, mtu, True, arena=out, max_frags=2 * n, port=port, first_len=first_len,
                            frag_first=frag_first)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    kms = [a.elapsed_time(z) for a, z in ev]
    kernel_ms = sum(kms) / len(kms)
    totals = [int(x) for x in r["totals"].cpu()]
    ok = int((port == 2).sum()) if totals == [2 * n, 976 * n] else 0
    dig = dict.fromkeys(shard.DIGEST_FIELDS, 0)
    dig.update(ok=ok, packets=n)
    _, kernel_ms, dig, (nfrag,), _ = shard.reduce_results(torch, dist, coll_dev, 0.0, kernel_ms, dig, [totals[0]])
    dig = [dig["ok"], dig["packets"], nfrag]
    del arena, out, saved, port, first_len, frag_first
    torch.cuda.empty_cache()
    alg = (20 + 928 + 968 + 8) * n
    ach = alg / (kernel_ms * 1e-3) / 1e9
    traffic, tsrc = load_traffic("c3", "IPFragmenter")
    return {"element": "IPFragmenter(576, HONOR_DF true)", "workload": w["desc"],
            "kernel_ms": round(kernel_ms, 4), "kernel_ms_min": round(min(kms), 4),
            "mpps": round(dig[1] / (kernel_ms * 1e-3) / 1e6, 1),
            "fragments_per_s_M": round((dig[1] + dig[2]) / (kernel_ms * 1e-3) / 1e6, 1),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "alg_bytes_per_launch": alg,
                         "traffic_source": tsrc},
            "verify": {"fragmented": dig[0], "packets": dig[1], "appended_fragments": dig[2]},
            "note": "kernel time (one plan + look-back + write launch, after a small memset); first-fragment headers restored between steps"}


COPY_SHAPES = {0: "gs4_ntst_8k", 1: "gs8_ntst_8k", 2: "gs4_st_8k", 3: "gs8_st_16k", 5: "gs16_st_4k",
               6: "wave8_st_4k", 7: "flat4_st"}


def copy_stream_peak(torch, ctx, nbytes=4 << 30, reps=3, launches=5, rounds=2):
    """Measured HBM copy ceiling (clk_copy_stream): `nbytes` copied between
    two device buffers, 16 B nontemporal loads, 4 or 8 in flight per lane,
    nontemporal or plain stores, capped grids -- the traffic of equal read
    and write streams (the fragmenter's); and shape 4, the IMIX Set's own
    pattern without its arithmetic (the stream read once, one 64 B block in
    six written back in place).  GB/s of read + written bytes, best of
    `reps` x `launches`, the shapes in turn for `rounds` rounds.  Returns
    ({shape: GB/s}, the best copy shape's GB/s, the Set pattern's GB/s)."""
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    src.fill_(3)
    dst.fill_(0)
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    names = {**COPY_SHAPES, 4: "set_blocks_1in6"}
    best = {name: 1e30 for name in names.values()}
    for _ in range(rounds):
        for shape, name in names.items():
            ctx.copy_stream(dst, src, shape=shape, out=out)
            torch.cuda.synchronize()
            for _ in range(reps):
                s.record()
                for _ in range(launches):
                    ctx.copy_stream(dst, src, shape=shape, out=out)
                e.record()
                torch.cuda.synchronize()
                best[name] = min(best[name], s.elapsed_time(e) / launches)
    moved = {name: (2 * nbytes if shape != 4 else nbytes + (nbytes // 64 + 5) // 6 * 64) for shape, name in names.items()}
    rates = {name: round(moved[name] / (ms * 1e-3) / 1e9, 1) for name, ms in best.items()}
    del src, dst
    torch.cuda.empty_cache()
    return rates, max(rates[n] for n in COPY_SHAPES.values()), rates["set_blocks_1in6"]


READ_SHAPES = {0: "gs8_nt_8k", 1: "gs4_nt_8k", 2: "gs16_nt_2k", 3: "wave8_nt_4k", 4: "rows1536_nt",
               5: "rows1536_nt_8k"}


def read_stream_peak(torch, ctx, nbytes=8 << 30, reps=5, launches=10, rounds=3, detail=None):
    """Measured HBM read-stream ceiling: clk_read_stream in the four best
    shapes of tools/probes/read_probe.hip (CLK_TUNE_READ_SHAPE: nontemporal
    16 B loads, grid-stride with 4 / 8 / 16 in flight per lane on a capped
    grid, or wave-contiguous runs) and the fixed-geometry Check kernels' own
    pattern without their arithmetic (16-lane groups on 1536 B rows, 6 loads
    per lane), each `launches` back to back, best of
    `reps`, the shapes taken in turn for `rounds` rounds (one slow moment of
    the box does not set a shape's figure); the best shape's GB/s (`detail`:
    every shape's)."""
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    buf.fill_(1)
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = {name: 1e30 for name in READ_SHAPES.values()}
    for _ in range(rounds):
        for shape, name in READ_SHAPES.items():
            ctx.tune(read_shape=shape)
            ctx.read_stream(buf, out=out)
            torch.cuda.synchronize()
            for _ in range(reps):
                s.record()
                for _ in range(launches):
                    ctx.read_stream(buf, out=out)
                e.record()
                torch.cuda.synchronize()
                best[name] = min(best[name], s.elapsed_time(e) / launches)
    rates = {name: round(nbytes / (ms * 1e-3) / 1e9, 1) for name, ms in best.items()}
    ctx.tune(read_shape=0)
    del buf
    torch.cuda.empty_cache()
    if detail is not None:
        detail.update(rates)
    return max(rates.values())


def host_topology():
    """Logical CPUs this process may run on, one per physical core (the first
    sibling), ordered round-robin over sockets so a leg with fewer threads
    than cores still uses every socket's memory; plus the cgroup CPU quota
    (cpu.max; None: unlimited), the L3 bytes of the whole machine and the
    CPU model."""
    allowed = sorted(os.sched_getaffinity(0))
    cores = {}
    for c in allowed:
        base = "/sys/devices/system/cpu/cpu%d/topology/" % c
        try:
            pkg = int(open(base + "physical_package_id").read())
            core = int(open(base + "core_id").read())
        except (OSError, ValueError):
            pkg, core = 0, c
        cores.setdefault((pkg, core), c)
    by_pkg = {}
    for (pkg, core), c in sorted(cores.items()):
        by_pkg.setdefault(pkg, []).append(c)
    order = []
    for k in range(max(len(v) for v in by_pkg.values())):
        for pkg in sorted(by_pkg):
            if k < len(by_pkg[pkg]):
                order.append(by_pkg[pkg][k])
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    l3 = 0
    seen = set()
    for c in allowed:
        d = "/sys/devices/system/cpu/cpu%d/cache/index3/" % c
        try:
            ids = open(d + "shared_cpu_list").read().strip()
            if ids in seen:
                continue
            seen.add(ids)
            sz = open(d + "size").read().strip()
            l3 += int(sz[:-1]) * {"K": 1 << 10, "M": 1 << 20}.get(sz[-1], 1) if sz[-1] in "KM" else int(sz)
        except (OSError, ValueError):
            pass
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return dict(cpus=order, sockets=len(by_pkg), physical_cores=len(cores), logical_cpus=len(allowed),
                quota=quota, l3_bytes=l3, model=model)


# CPU legs: workload -> (element, oracle op, metric bytes/pkt)
CPU_LEGS = {"c2": ("CheckIPHeader", 20), "c3": ("CheckUDPHeader", 1500), "c4": ("CheckUDPHeader", None),
            "c5": ("CheckTCPHeader", 9000)}


def cpu_baseline(legs=("c2", "c3", "c4", "c5"), reps=5, single_only=False):
    """The oracle restatement of lib/in_cksum.c + the element (-O2 -g) on the
    host cores, per BASELINE.md §2: one thread, then one thread pinned per
    physical core (capped by the cgroup CPU quota; CLK_CPU_THREADS
    overrides), each pinned BEFORE it first-touches its own DRAM-resident
    shard (>= 4 GiB in all and >= 4x the machine's L3; C5: a 1M-packet
    subset); warm-up, then the median of `reps` passes."""
    import ctypes
    from tests import oracle_lib
    L_ = oracle_lib.load_oracle()

    class Cfg(ctypes.Structure):
        _fields_ = [("op", ctypes.c_int), ("arg", ctypes.c_int), ("proto", ctypes.c_int), ("imix", ctypes.c_int),
                    ("fixed_len", ctypes.c_uint32), ("stride", ctypes.c_uint64),
                    ("bytes_per_thread", ctypes.c_uint64), ("seed", ctypes.c_uint64), ("reps", ctypes.c_int)]

    class Res(ctypes.Structure):
        _fields_ = [("median_s", ctypes.c_double), ("min_s", ctypes.c_double), ("max_s", ctypes.c_double),
                    ("gen_s", ctypes.c_double), ("packets", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                    ("ok", ctypes.c_uint64), ("pinned", ctypes.c_int)]

    L_.oracle_cpu_baseline.restype = ctypes.c_int
    L_.oracle_cpu_baseline.argtypes = [ctypes.POINTER(Cfg), ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Res)]
    topo = host_topology()
    nthr = len(topo["cpus"])
    if topo["quota"]:
        nthr = min(nthr, max(1, int(topo["quota"])))
    nthr = int(os.environ.get("CLK_CPU_THREADS", nthr))
    total = int(os.environ.get("CLK_CPU_SAMPLE_BYTES", max(4 << 30, 4 * topo["l3_bytes"])))   # env: tests only
    ops = {"CheckIPHeader": oracle_lib.OP_CHECK_IP, "CheckUDPHeader": oracle_lib.OP_CHECK_UDP,
           "CheckTCPHeader": oracle_lib.OP_CHECK_TCP}
    out = {}
    for wl in legs:
        element, ck = CPU_LEGS[wl]
        w = WORKLOADS[wl]
        res = {}
        for label, t in (("single_thread", 1),) + ((("all_cores", nthr),) if not single_only else ()):
            cfg = Cfg()
            cfg.op, cfg.arg, cfg.proto, cfg.imix = ops[element], 1, w["proto"], 1 if wl == "c4" else 0
            cfg.fixed_len, cfg.stride = w["L"], w["stride"]
            sample = min(1 << 30, total) if t == 1 else total
            if wl == "c5" and t > 1 and "CLK_CPU_SAMPLE_BYTES" not in os.environ:
                sample = (1 << 20) * w["stride"]                # the 1M-packet subset
            cfg.bytes_per_thread = max(sample // t, 64 << 10)
            cfg.seed, cfg.reps = 0x5EED, reps
            cpus = (ctypes.c_int * t)(*topo["cpus"][:t])
            r = Res()
            rc = L_.oracle_cpu_baseline(ctypes.byref(cfg), cpus, t, ctypes.byref(r))
            if rc != 0:
                res[label] = {"error": "oracle_cpu_baseline rc %d" % rc}
                continue
            pps = r.packets / r.median_s
            ckb = r.bytes if ck is None else r.packets * ck
            res[label] = {"value": round(ckb / r.median_s / GIB, 3), "unit": "GiB/s", "mpps": round(pps / 1e6, 3),
                          "threads": t, "pinned": r.pinned, "packets": r.packets,
                          "sample_bytes": r.packets * w["stride"] if wl != "c4" else cfg.bytes_per_thread * t,
                          "median_s": round(r.median_s, 5), "min_s": round(r.min_s, 5), "max_s": round(r.max_s, 5),
                          "ok": r.ok}
        out[wl] = {"element": element, "workload": w["desc"], **res}
    return {"legs": out, "threads": nthr, "host": topo | {"cpus": None},
            "method": "oracle/cksum_oracle.c (-O2 -g restatement of lib/in_cksum.c + the element), one thread "
                      "pinned per physical core (round-robin over sockets, capped by the cgroup CPU quota), "
                      "NUMA-local first touch of a DRAM-resident shard per thread, warm-up + median of %d" % reps}


def load_traffic(wname, element):
    """HBM bytes per launch of `element` from the committed PMC summary."""
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % wname)
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get("elements", {}).get(element, {})
        return e.get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)
    except (OSError, ValueError):
        return None, None


def summarize(r, steps, wname):
    """Per-element numbers: rate from the wall clock over the timed steps,
    roofline from the HIP-event kernel time."""
    step_s = r["wall"] / steps
    pps = r["n_total"] / step_s
    achieved = r["alg_bytes"] / (r["kernel_ms"] * 1e-3) / 1e9
    traffic, tsrc = load_traffic(wname, r["element"])
    return {
        "element": r["element"],
        "value": round(pps * (r["ck_bytes"] / r["n"]) / GIB, 2), "unit": "GiB/s",
        "mpps": round(pps / 1e6, 1), "ms_per_step": round(step_s * 1e3, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel_ms": round(r["kernel_ms"], 4), "kernel_ms_min": round(r["kernel_ms_min"], 4),
                     "alg_bytes_per_launch": r["alg_bytes"], "traffic_source": tsrc},
        "verify": r["digest"],
        **({"per_rank": [{"wall_ms": round(w_ * 1e3, 3), "kernel_ms": round(k_, 4), "first": sh[0], "packets": sh[1],
                          "bytes": sh[2]} for (w_, k_), sh in zip(r["per_rank"], r["shards"])]}
           if len(r["per_rank"]) > 1 else {}),
        **({"gather_to_rank0": r["gather"]} if r.get("gather") else {}),
    }


def e2e(torch, ctx, wname, element, chunk_pkts=1 << 18, nchunks=24,
        glue_pkts=int(os.environ.get("CLK_E2E_GLUE_PKTS", 1 << 21))):
    """End-to-end rates with the packets in HOST memory (DESIGN.md "E2E").

    (a) device C ABI over pinned SoA chunks: per chunk, hipMemcpyAsync H2D of
        the packet slots, the element kernel, D2H of the 1 B verdicts (and
        2 B checksums for Set), double-buffered on two streams so chunk k+1's
        H2D overlaps chunk k's kernel and D2H;
    (b) the host element glue (click_amd/host/elements.cc) fed one packet
        at a time, as a Click element would be: gather into pinned staging,
        H2D, kernel, D2H, route -- single host thread."""
    import click_amd
    from click_amd.elements import Element
    w = WORKLOADS[wname]
    L, stride = w["L"], w["stride"]
    host = torch.empty(chunk_pkts * stride * 2, dtype=torch.uint8, pin_memory=True)
    dev = [torch.empty(chunk_pkts * stride, dtype=torch.uint8, device="cuda") for _ in range(2)]
    status = [torch.empty(chunk_pkts, dtype=torch.uint8, device="cuda") for _ in range(2)]
    sums = [torch.empty(chunk_pkts, dtype=torch.uint16, device="cuda") for _ in range(2)]
    # host packets: generate on the GPU, copy down once
    g = click_amd.Batch(dev[0], chunk_pkts, stride=stride, fixed_len=L)
    ctx.gen_packets(g, proto=w["proto"])
    ctx.set_ip_checksum(g, want_sums=False)
    run_element(ctx, "SetTCPChecksum" if w["proto"] == 6 else "SetUDPChecksum", g, status[0])
    torch.cuda.synchronize()
    host[:chunk_pkts * stride].copy_(dev[0])
    host[chunk_pkts * stride:].copy_(dev[0])
    streams = [torch.cuda.Stream() for _ in range(2)]
    # one context per stream: a context's scratch is not shared across streams
    ctxs = [click_amd.Context(ctx.device, stream=st) for st in streams]
    for c in ctxs:
        c.reserve(chunk_pkts)
    is_set = element.startswith("Set")

    def chunk(k):
        j = k % 2
        st = streams[j]
        c = ctxs[j]
        with torch.cuda.stream(st):
            src = host[(k % 2) * chunk_pkts * stride:(k % 2 + 1) * chunk_pkts * stride]
            dev[j].copy_(src, non_blocking=True)
            b = click_amd.Batch(dev[j], chunk_pkts, stride=stride, fixed_len=L)
            if is_set:
                {"SetUDPChecksum": c.set_udp_checksum, "SetTCPChecksum": c.set_tcp_checksum,
                 "SetIPChecksum": c.set_ip_checksum}[element](b, status=status[j], sums=sums[j])
                out_h[j * chunk_pkts * 3:(j * 3 + 2) * chunk_pkts].view(torch.uint16).copy_(sums[j], non_blocking=True)
            else:
                run_element(c, element, b, status[j])
            out_h[(j * 3 + 2) * chunk_pkts:(j * 3 + 3) * chunk_pkts].copy_(status[j], non_blocking=True)

    out_h = torch.empty(chunk_pkts * 6, dtype=torch.uint8, pin_memory=True)
    chunk(0)
    chunk(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(nchunks):
        chunk(k)
    torch.cuda.synchronize()
    dt_a = time.perf_counter() - t0
    for c in ctxs:
        c.close()
    pk_a = chunk_pkts * nchunks
    ok_a = int((out_h[2 * chunk_pkts:3 * chunk_pkts] == 0).sum())
    # (b) element glue, one packet at a time from C++ (bursts of 32 packet
    # pointers, as FromDPDKDevice receives them), batches of 64K packets
    import numpy as np
    e = Element(ctx, element, ", ".join(x for x in (ELEMENT_CONF.get(element, ""), "BATCH 65536") if x), noutputs=2)
    base = host.data_ptr()
    slots = np.arange(glue_pkts, dtype=np.uint64) % np.uint64(2 * chunk_pkts)    # the host buffer's packets, reused
    ptrs = slots * np.uint64(stride) + np.uint64(base)
    lens = np.full(glue_pkts, L, np.uint32)
    nhs = np.zeros(glue_pkts, np.int32)
    e.push_burst(ptrs, lens, nhs, first_token=0)     # warm-up: both staging buffers allocated
    e.flush()
    e.results()
    t0 = time.perf_counter()
    e.push_burst(ptrs, lens, nhs, first_token=0)     # C++ loop: push() per packet, flush_async per 64K
    e.flush()
    dt_b = time.perf_counter() - t0
    _, ports, _ = e.results()
    ok_b = int((ports == 0).sum())
    gpu_ns = int(e.read_handler("gpu_ns"))
    e.close()
    # (c) zero-copy: the host arena registered (clk_host_register), the
    # kernel reads the packets over PCIe where they lie; D2H of verdicts only
    raw = np.zeros(host.numel() + 8192, np.uint8)            # pageable memory, registered below
    hostnp = raw[(-raw.ctypes.data) % 4096:][:host.numel()]
    hostnp[:] = host.numpy()
    dbase = ctx.host_register(hostnp)
    zptrs = slots * np.uint64(stride) + np.uint64(hostnp.ctypes.data)
    try:
        zb = click_amd.Batch(dbase, chunk_pkts * 2, stride=stride, fixed_len=L)
        st = torch.empty(chunk_pkts * 2, dtype=torch.uint8, device="cuda")
        run_element(ctx, element, zb, st)
        torch.cuda.synchronize()
        reps_c = max(2, nchunks // 2)
        t0 = time.perf_counter()
        for _ in range(reps_c):
            run_element(ctx, element, zb, st)
            out_h[:chunk_pkts * 2].copy_(st, non_blocking=True)
        torch.cuda.synchronize()
        dt_c = time.perf_counter() - t0
        pk_c = reps_c * chunk_pkts * 2
        ok_c = int((st == 0).sum())
        # (d) the element glue with ZEROCOPY true: push() records offsets only
        e = Element(ctx, element, ", ".join(x for x in (ELEMENT_CONF.get(element, ""), "BATCH 65536, ZEROCOPY true")
                                            if x), noutputs=2)
        e.push_burst(zptrs, lens, nhs, first_token=0)    # warm-up
        e.flush()
        e.results()
        t0 = time.perf_counter()
        e.push_burst(zptrs, lens, nhs, first_token=0)
        e.flush()
        dt_d = time.perf_counter() - t0
        _, ports, _ = e.results()
        ok_d = int((ports == 0).sum())
        e.close()
    finally:
        ctx.host_unregister(hostnp)
    return {
        "metric": "end-to-end (host-resident packets) GiB/s checksummed", "element": element,
        "workload": w["desc"],
        "pinned_soa": {"value": round(pk_a * L / dt_a / GIB, 2), "unit": "GiB/s", "mpps": round(pk_a / dt_a / 1e6, 1),
                       "pcie_GBs": round(pk_a * (stride + (3 if is_set else 1)) / dt_a / 1e9, 1),
                       "packets": pk_a, "chunk_packets": chunk_pkts, "ok": ok_a,
                       "note": "H2D of slots + kernel + D2H of verdicts/checksums, 2 streams"},
        "zero_copy_abi": {"value": round(pk_c * L / dt_c / GIB, 2), "unit": "GiB/s", "mpps": round(pk_c / dt_c / 1e6, 1),
                          "packets": pk_c, "ok": ok_c,
                          "note": "kernel reads the registered pinned host arena over PCIe (clk_host_register); D2H of verdicts"},
        "element_glue_zero_copy": {"value": round(glue_pkts * L / dt_d / GIB, 3), "unit": "GiB/s",
                                   "mpps": round(glue_pkts / dt_d / 1e6, 3), "packets": glue_pkts, "ok": ok_d,
                                   "note": "C++ push() per packet records the packet's offset in the registered region (no gather), 64K-packet batches double-buffered, 1 host thread"},
        "element_glue": {"value": round(glue_pkts * L / dt_b / GIB, 3), "unit": "GiB/s",
                         "mpps": round(glue_pkts / dt_b / 1e6, 3), "packets": glue_pkts, "ok": ok_b,
                         "gpu_ms": round(gpu_ns / 1e6, 3), "wall_ms": round(dt_b * 1e3, 3),
                         "note": "C++ push() per packet (gather memcpy into pinned staging), 64K-packet batches double-buffered (flush_async: batch k on the GPU while k+1 is staged), 1 host thread"},
    }


# BASELINE config 1: conf/fake-iprouter.click's forwarding path
# (fake-iprouter.click:38-100) on the 86 B frame of its InfiniteSource,
# 600000 packets (test/userlevel/iprouter-01.clicktest:243), run through the
# element glue as the separate elements and as iprouter-01's click-xform
# combos (IPInputCombo / IPOutputCombo; OUTA == OUTB, iprouter-01:57).
C1_PACKETS = 600000
C1_CHAINS = {
    "elements": [("CheckIPHeader", "INTERFACES 18.26.4.1/24 18.26.7.1/24, OFFSET 14", 2),
                 ("IPGWOptions", "18.26.4.24", 2), ("FixIPSrc", "18.26.4.24", 1),
                 ("DecIPTTL", "", 2), ("IPFragmenter", "300", 2)],
    "combos": [("IPInputCombo", "2, INTERFACES 18.26.4.1/24 18.26.7.1/24", 1),
               ("IPOutputCombo", "1, 18.26.4.24, 300", 5)],
}


def glue_thread_legs(timeout=300):
    """The element glue from 1, 2 and 4 host threads on one GPU
    (tests/native/mt_glue: click -j N's RouterThreads, each pinned to its own
    physical core with its own glue element and context; C2 64 B packets,
    ZEROCOPY, BATCH 65536).  A native program, as Click's threads are: from
    Python threads the legs met the process's other (torch) threads in the
    cgroup's CPU quota.  None if the program was not built."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "native", "bin", "mt_glue")
    if not os.path.exists(exe):
        return None
    r = subprocess.run([exe], capture_output=True, text=True, timeout=timeout)
    if r.returncode:
        return {"error": (r.stderr or r.stdout)[-400:]}
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def pull_legs(scale=1, timeout=300):
    """Pull mode through the Click adapter's core (tests/native/pull_bench,
    built by build()): Queue -> CheckIPHeader -> SetIPChecksum (C2, 64 B) and
    Queue -> CheckUDPHeader -> SetUDPChecksum (C3, 1500 B) pulled on one
    thread; Mpps and the per-pull() latency distribution.  None if the
    program was not built."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "native", "bin", "pull_bench")
    if not os.path.exists(exe):
        return None
    r = subprocess.run([exe, str(scale)], capture_output=True, text=True, timeout=timeout)
    if r.returncode:
        return {"error": (r.stderr or r.stdout)[-400:]}
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def c1_frame():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_vectors.json")))["vectors"]
    l3 = bytes.fromhex([v for v in g if v["name"] == "fake-iprouter-ip-check"][0]["l3"])
    return bytes.fromhex("0000c0ae67ef0000000000000800") + l3          # fake-iprouter.click:42-44


CHAIN_BATCH = 16384     # a chain's host passes over a batch that stays in L2
C1_RUNS = 5             # timed runs per leg (after one warm-up); the median is reported


def c1_median(walls):
    """The median of a config-1 leg's timed runs (wall seconds)."""
    return sorted(walls)[len(walls) // 2]


def config1(ctx, n=C1_PACKETS, batch=65536):
    """Config 1 through the element glue on the GPU: every element of the
    chain takes all n frames by push_burst (C++ push() per packet, batches of
    `batch` double-buffered), flushes and routes them; the next element takes
    the survivors.  One untimed warm-up run on a copy allocates the staging
    buffers; then C1_RUNS timed runs, each on fresh frames, and the median
    run is reported (`mpps`; every run in `runs_mpps`).  Asserts all n
    forwarded on port 0 and identical bytes both ways (OUTA == OUTB)."""
    import numpy as np
    from click_amd.elements import Element, ResultBuffers
    frame = c1_frame()
    out, arenas = {}, {}
    rbufs = ResultBuffers(n + 1)              # the harness pops results into reused arrays
    runs = [(name, chain, False) for name, chain in C1_CHAINS.items()] + \
           [(name + "_zerocopy", chain, True) for name, chain in C1_CHAINS.items()]
    for name, chain, zc in runs:
        extra = "BATCH %d" % batch + (", ZEROCOPY true" if zc else "")
        els = [Element(ctx, cls, ", ".join(x for x in (conf, extra) if x), noutputs=nout) for cls, conf, nout in chain]
        walls, runs = [], []
        for run in range(1 + C1_RUNS):
            raw = np.empty(n * len(frame) + 8192, np.uint8)          # page-aligned, registrable
            arena = raw[(-raw.ctypes.data) % 4096:][:n * len(frame)]
            arena[:] = np.tile(np.frombuffer(frame, np.uint8), n)
            if zc:
                ctx.host_register(arena)
            ptrs = np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(len(frame))
            lens = np.full(n, len(frame), np.uint32)
            nhs = np.full(n, 14, np.int32)
            t0 = time.perf_counter()
            fwd = n
            parts = []
            for e in els:
                ta = time.perf_counter()
                e.push_burst(ptrs, lens, nhs, first_token=0)
                tb = time.perf_counter()
                e.flush()
                tc = time.perf_counter()
                tok, port, _ = e.results(bufs=rbufs)
                keep = port == 0
                fwd = int(keep.sum())
                if fwd != len(ptrs):
                    ptrs, lens, nhs = ptrs[tok[keep].astype(np.int64)], lens[keep], nhs[keep]
                parts.append((tb - ta, tc - tb, time.perf_counter() - tc))
            dt = time.perf_counter() - t0
            if zc:
                ctx.host_unregister(arena)
            if run:
                walls.append(dt)
                runs.append(parts)
        for e in els:
            e.close()
        dt = c1_median(walls)
        parts = runs[walls.index(dt)]
        arenas[name] = arena
        out[name] = {"chain": [c[0] for c in chain], "forwarded": fwd, "wall_s": round(dt, 4),
                     "mpps": round(n / dt / 1e6, 2), "runs_mpps": [round(n / w / 1e6, 2) for w in walls],
                     "per_element_ms": {c[0]: {"push": round(a * 1e3, 2), "flush": round(b * 1e3, 2),
                                               "results": round(r * 1e3, 2)} for c, (a, b, r) in zip(chain, parts)}}
    # the same chains on one device-resident batch (clk_chain_*: one gather,
    # one H2D, each member's kernel over what the members before it passed,
    # one D2H, one routing pass per packet)
    from click_amd.elements import Chain
    cbufs = [np.empty(n + 1, t) for t in (np.uint64, np.int32, np.int32, np.uint32, np.uint32)]
    cptrs = [b.ctypes.data_as(ctypes.c_void_p) for b in cbufs]
    for name, chain, cb, zc in [(nm, ch_, b_, z_) for nm, ch_ in C1_CHAINS.items()
                                for b_, z_ in ((batch, False), (CHAIN_BATCH, False), (batch, True))]:
        name = name + ("_zerocopy" if zc else "") + ("" if cb == batch else "_%dk" % (cb >> 10))
        extra = "BATCH %d" % cb + (", ZEROCOPY true" if zc else "")
        els = [Element(ctx, cls, ", ".join(x for x in (conf, extra) if x), noutputs=nout)
               for cls, conf, nout in chain]
        ch = Chain(els)
        walls, phases = [], []
        for run in range(1 + C1_RUNS):
            raw = np.empty(n * len(frame) + 8192, np.uint8)
            arena = raw[(-raw.ctypes.data) % 4096:][:n * len(frame)]
            arena[:] = np.tile(np.frombuffer(frame, np.uint8), n)
            if zc:
                ctx.host_register(arena)
            ptrs = np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(len(frame))
            lens = np.full(n, len(frame), np.uint32)
            t0 = time.perf_counter()
            ch.push_burst(ptrs, lens, None, first_token=0)
            tb = time.perf_counter()
            ch.flush()
            tc = time.perf_counter()
            k = int(ch.lib.clk_chain_results(ch.h, *cptrs, n + 1))
            dt = time.perf_counter() - t0
            fwd = int(((cbufs[1][:k] == len(chain) - 1) & (cbufs[2][:k] == 0)).sum())
            if zc:
                ctx.host_unregister(arena)
            if run:
                walls.append(dt)
                phases.append((tb - t0, tc - tb, t0 + dt - tc))
        dt = c1_median(walls)
        ph = phases[walls.index(dt)]
        st = (ctypes.c_double * 8)()
        ch.lib.clk_chain_stats(ch.h, ctypes.cast(st, ctypes.c_void_p), 8)
        ch.close()
        for e in els:
            e.close()
        arenas[name + "_chain"] = arena
        out[name + "_chain"] = {"chain": [c[0] for c in chain], "forwarded": fwd, "wall_s": round(dt, 4),
                                "mpps": round(n / dt / 1e6, 2), "runs_mpps": [round(n / w / 1e6, 2) for w in walls],
                                "ms": {"push": round(ph[0] * 1e3, 2), "flush": round(ph[1] * 1e3, 2),
                                       "results": round(ph[2] * 1e3, 2)},
                                # host ns per packet by phase, over all runs (warm-up + timed)
                                "ns_per_packet": {k: round(v * 1e9 / ((1 + C1_RUNS) * n), 1) for k, v in zip(
                                    ("push", "rebuild", "gpu_round_trips", "unused", "h2d", "d2h_back",
                                     "route", "copy_back"), list(st)) if k != "unused"}}
    # as the Click adapter forms fake-iprouter.click's graph (lines 91-106):
    # CheckIPHeader alone (StaticIPLookup follows it), then gio -> FixIPSrc ->
    # dt -> fr on one chain (each fed only by the one before, output 0)
    spec = C1_CHAINS["elements"]
    head = Element(ctx, spec[0][0], spec[0][1] + ", BATCH %d" % batch, noutputs=spec[0][2])
    tail = [Element(ctx, cls, ", ".join(x for x in (conf, "BATCH %d" % batch) if x), noutputs=nout)
            for cls, conf, nout in spec[1:]]
    ch = Chain(tail)
    walls = []
    for run in range(1 + C1_RUNS):
        raw = np.empty(n * len(frame) + 8192, np.uint8)
        arena = raw[(-raw.ctypes.data) % 4096:][:n * len(frame)]
        arena[:] = np.tile(np.frombuffer(frame, np.uint8), n)
        ptrs = np.uint64(arena.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(len(frame))
        lens = np.full(n, len(frame), np.uint32)
        nhs = np.full(n, 14, np.int32)
        t0 = time.perf_counter()
        head.push_burst(ptrs, lens, nhs, first_token=0)
        head.flush()
        tok, port, ln = head.results(bufs=rbufs)
        keep = port == 0
        if keep.all() and len(tok) == n:         # every frame on (in push order): no re-indexing
            ch.push_burst(ptrs, ln if ln.dtype == np.uint32 else ln.astype(np.uint32), nhs, first_token=0)
        else:
            sel = tok[keep].astype(np.int64)
            ch.push_burst(ptrs[sel], ln[keep].astype(np.uint32), nhs[sel], first_token=0)
        ch.flush()
        k = int(ch.lib.clk_chain_results(ch.h, *cptrs, n + 1))
        dt = time.perf_counter() - t0
        fwd = int(((cbufs[1][:k] == len(tail) - 1) & (cbufs[2][:k] == 0)).sum())
        if run:
            walls.append(dt)
    dt = c1_median(walls)
    ch.close()
    for e in [head] + tail:
        e.close()
    arenas["elements_as_click_forms"] = arena
    out["elements_as_click_forms"] = {"chain": [spec[0][0], "[" + ", ".join(c[0] for c in spec[1:]) + "]"],
                                      "forwarded": fwd, "wall_s": round(dt, 4), "mpps": round(n / dt / 1e6, 2),
                                      "runs_mpps": [round(n / w / 1e6, 2) for w in walls]}
    same = all(np.array_equal(arenas["elements"], arenas[k]) for k in arenas)
    return {"workload": "C1: conf/fake-iprouter.click forwarding path, %d x %d B frames, element glue on the GPU "
                        "(staged: push() gathers into pinned staging; _zerocopy: registered host arena); "
                        "median of %d timed runs" % (n, len(frame), C1_RUNS),
            "packets": n, "expect_forwarded": n, "outa_eq_outb": same,
            "ok": same and all(v["forwarded"] == n for v in out.values()), **out}


def config1_cpu(n=C1_PACKETS):
    """The same chains on one host thread through the oracle restatement
    (the byte-touching elements only; Click's scheduler, Classifier and
    queues are not part of it): CheckIPHeader + IPGWOptions + FixIPSrc +
    DecIPTTL + IPFragmenter(300), and IPInputCombo + IPOutputCombo.  The
    thread is pinned to one core; the frames' arena and every output array
    are allocated and first-touched there once, outside the clock (oracle_lib's
    helpers allocate per call, and the fragmenter helper copies the whole
    arena for a sizing pass: BENCH_r05's 22-or-40 Mpps runs), and the
    pristine frames are copied back before each run; one warm-up, then
    C1_RUNS timed runs: min / median / max."""
    import numpy as np
    from tests import oracle_lib
    L = oracle_lib.load_oracle()
    P = oracle_lib._np_ptr
    frame = c1_frame()
    fl = len(frame)
    prev = os.sched_getaffinity(0)
    core = min(prev)
    os.sched_setaffinity(0, {core})
    try:
        pristine = np.tile(np.frombuffer(frame, np.uint8), n)
        arena = np.empty_like(pristine)
        arena[:] = pristine                        # first touch on the pinned core
        l3 = arena[14:]
        flags = np.zeros(n, np.uint8)
        codes, c2, port, prob = (np.zeros(n, np.uint8) for _ in range(4))
        sums = np.zeros(n, np.uint16)
        first = np.zeros(n, np.uint32)
        ffirst = np.zeros(n, np.uint64)
        totals = np.zeros(2, np.uint64)
        fcap = 4 * n                               # room for the fragments (fake-iprouter's frames make none)
        fout = np.zeros(fcap * 64, np.uint8)
        foff, flen, fsrc = np.zeros(fcap, np.uint64), np.zeros(fcap, np.uint32), np.zeros(fcap, np.uint32)
        ops, iops = oracle_lib.OPS, oracle_lib.IP_OUT_OPS
        stride, flen3, my_ip = fl, fl - 14, 0x18041A12

        def out_op(op, fl_=None, mtu=0xFFFFFFFF, dst=codes):
            assert L.oracle_ip_out_batch(iops[op], P(l3), None, stride, None, flen3, n, P(fl_), my_ip, None, 0, 0,
                                         mtu, P(dst), P(prob), P(sums)) == 0

        res = {}
        for name in ("elements", "combos"):
            walls = []
            for run in range(1 + C1_RUNS):
                np.copyto(arena, pristine)
                t0 = time.perf_counter()
                assert L.oracle_batch(ops["check_ip"], P(l3), None, stride, None, flen3, n, 1, P(codes), P(sums)) == 0
                if name == "elements":
                    ok = codes == 0
                    out_op("ip_gw_options", dst=port)
                    out_op("fix_ip_src", fl_=flags, dst=port)
                    assert L.oracle_batch(ops["dec_ttl"], P(l3), None, stride, None, flen3, n, 1, P(c2), P(sums)) == 0
                    L.oracle_ip_fragment_batch(P(l3), None, stride, None, flen3, n, 300, 0, None, P(port), P(first),
                                               P(ffirst), P(fout), P(foff), P(flen), P(fsrc), P(totals))
                    fwd = int((ok & (c2 == 0) & (port == 0)).sum())
                else:
                    ok = codes == 0
                    out_op("ip_output_combo", mtu=300, dst=port)
                    fwd = int((ok & (port == 0)).sum())
                if run:
                    walls.append(time.perf_counter() - t0)
            dt = c1_median(walls)
            rates = [round(n / w / 1e6, 2) for w in walls]
            res[name] = {"forwarded": fwd, "wall_s": round(dt, 4), "mpps": round(n / dt / 1e6, 2),
                         "min_med_max_mpps": [min(rates), round(n / dt / 1e6, 2), max(rates)], "runs_mpps": rates}
    finally:
        os.sched_setaffinity(0, prev)
    return {"threads": 1, "kind": "port", "runs": C1_RUNS, "pinned_cpu": core, **res,
            "note": "oracle restatement of the byte-touching elements, one pinned host thread, every buffer allocated "
                    "and first-touched once; Click's own runtime on the same graph: drop_in.c1 (click-cpu)"}


CLICK_LEGS = (("c1", 3000000, 1), ("c1", 3000000, 32), ("c3chk", 1000000, 32), ("c3set", 1000000, 32))


def click_drop_in(reps=3, timeout=180):
    """The GPU elements inside Click: the userlevel driver built with the GPU
    group under the reference class names (click-dropin) against the stock
    driver (click-cpu, the reference's CPU elements) on the same graph and
    host, both built by tools/click_scratch_build.sh (tools/click_perf.py):
    c1 = config 1's forwarding path (click_integration/conf/c1-forward.click,
    InfiniteSource BURST 1 and 32), c3chk = 1500 B UDP frames through
    CheckIPHeader -> CheckUDPHeader, c3set = SetUDPChecksum.  Mpps by the
    graph's AverageCounter, median of `reps` processes; x_cpu = drop-in /
    stock.  Both run with glibc's tcache deepened (click_perf.TCACHE: the
    packets a GPU element holds outrun Click's 1000-packet pool, and freed
    chunks then stay per-thread; the stock build's rate does not change).  Also the adapter core's C3 push legs (tests/native/pull_bench c3:
    staged and ZEROCOPY).  None if the binaries were not built."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import click_perf
        from tests import click_run
    except Exception as e:                       # reported, not fatal
        return {"error": repr(e)}
    if not (click_run.binary("cpu") and click_run.binary("dropin")):
        return None
    out = {}
    for graph, limit, burst in CLICK_LEGS:
        rec = {"packets": limit, "burst": burst}
        for mode in ("cpu", "dropin"):
            runs = [click_perf.run_one(mode, graph, "", limit, burst, timeout=timeout, extra_env=click_perf.TCACHE)
                    for _ in range(reps)]
            ok = sorted(r["mpps_counter"] for r in runs if "count" in r and r["count"] == limit)
            rec[mode] = round(ok[len(ok) // 2], 2) if len(ok) == reps else None
            rec[mode + "_runs"] = [round(r["mpps_counter"], 2) if "count" in r else r for r in runs]
        rec["x_cpu"] = round(rec["dropin"] / rec["cpu"], 2) if rec["cpu"] and rec["dropin"] else None
        out["%s_burst%d" % (graph, burst)] = rec
    exe = os.path.join(ROOT, "tests", "native", "bin", "pull_bench")
    if os.path.exists(exe):
        try:
            r = subprocess.run([exe, "2", "c3"], capture_output=True, text=True, timeout=timeout)
            core = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
            out["core_c3_push"] = {x["leg"]: x.get("mpps") for x in core if "leg" in x} or core
        except Exception as e:
            out["core_c3_push"] = {"error": repr(e)}
    return {"workload": "GPU elements in Click's userlevel driver (click-dropin) vs the stock elements (click-cpu), "
                        "same graph and host; Mpps", **out}


def comm_info(torch, dist, dev):
    """Which communicator the run had: backend, world size as the process
    group reports it, and every rank's (rank, device index, device name,
    PCI bus id), gathered over the group -- an N-rank run shows N ranks."""
    name = torch.cuda.get_device_name(dev)
    try:
        bus = torch.cuda.get_device_properties(dev).pci_bus_id
    except Exception:                       # older torch: no pci_bus_id
        bus = None
    mine = [int(os.environ.get("RANK", "0")), dev, name, bus]
    if dist is None:
        return {"backend": None, "world_size": 1, "devices": [mine]}
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, mine)
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "devices": allr}


def compact_legs(legs):
    """cpu_baseline legs for the line: [GiB/s, Mpps] for one thread and
    [GiB/s, Mpps, threads] for all cores per workload; config 1 in Mpps."""
    out = {}
    for wl, leg in legs.items():
        if wl == "c1":
            out[wl] = {k: leg[k]["mpps"] for k in ("elements", "combos") if k in leg}
            continue
        one, al = leg.get("single_thread", {}), leg.get("all_cores", {})
        out[wl] = {"element": leg.get("element"), "1t": [one.get("value"), one.get("mpps")],
                   "all": [al.get("value"), al.get("mpps"), al.get("threads")]}
    return out


def bench_summary(line):
    """{workload/element: [kernel_ms, roofline frac, oracle_match, drops_exact]}
    over every timed element of the line (fragmenter: [kernel_ms, frac,
    all fragmented, null])."""
    out = {}
    wl0 = line["config"]["workload"].split(":")[0]
    sects = [(wl0, line.get("elements", {}))] + [(line[k]["workload"].split(":")[0], line[k]["elements"])
                                                 for k in ("c2_64b", "c4_imix", "c5_jumbo") if k in line]
    for wl, els in sects:
        for e, r in els.items():
            v = r.get("verify", {})
            out["%s %s" % (wl, e)] = [r["roofline"]["kernel_ms"], r["roofline"]["frac"],
                                      v.get("oracle", {}).get("oracle_match"), v.get("drops_exact")]
    f = line.get("fragmenter")
    if f:
        vf = f.get("verify", {})
        out["C3 IPFragmenter"] = [f["kernel_ms"], f["roofline"]["frac"],
                                  vf.get("fragmented") == vf.get("packets") and vf.get("packets", 0) > 0, None]
    c1 = line.get("c1_fake_iprouter")
    if c1:
        out["C1 mpps"] = {k: c1[k]["mpps"] for k in c1 if isinstance(c1[k], dict) and "mpps" in c1[k]}
        out["C1 ok"] = c1.get("ok")
    di = line.get("drop_in")
    if isinstance(di, dict):
        out["drop_in x_cpu"] = {k: [v.get("dropin"), v.get("cpu"), v.get("x_cpu")] for k, v in di.items()
                                if isinstance(v, dict) and "x_cpu" in v}
    rs = line.get("root_scatter")
    if rs:
        out["root scatter GB/s"] = rs["GBps_out_of_rank0"]
    comm = line.get("comm")
    if comm:
        out["ranks"] = [comm.get("backend"), comm.get("world_size")]
    return out


def spawn_ranks(args):
    """--gpus N > 1 without a torchrun environment: launch N ranks (one per
    GPU) under torch.distributed.run as a child process before anything
    touches the GPU, and exit with its status."""
    import socket
    import subprocess
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("bench: --gpus %d without WORLD_SIZE: launching %s" % (args.gpus, " ".join(cmd)))
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # the first ~8 launches of a 25 GB stream in a process run up to 25 %
    # slower (profiles/r02: C3 Check 4.92 -> 3.84 ms over launches 1-9)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: the workload's)")
    ap.add_argument("--no-c2", action="store_true", help="skip the extra 64 B (C2) measurement")
    ap.add_argument("--no-c1", action="store_true", help="skip the config-1 (fake-iprouter) measurement")
    ap.add_argument("--no-click", action="store_true", help="skip the GPU-elements-in-Click legs (drop_in)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-peak", action="store_true", help="skip the read-stream ceiling")
    ap.add_argument("--no-frag", action="store_true", help="skip the IPFragmenter measurement (C3)")
    ap.add_argument("--skip", default="", help="comma list of side configurations to skip: c4,c5")
    ap.add_argument("--e2e", action="store_true", help="measure the host-resident end-to-end rates instead")
    ap.add_argument("--scatter-bytes", type=int, default=1 << 30,
                    help="N > 1: bytes rank 0 sends each rank for the root-scatter measurement (0: skip)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the host-oracle digest of each element's results (SURVEY §8(e)(1))")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        log("bench: WORLD_SIZE=%d but --gpus %d: refusing to report a mislabelled run" % (world, args.gpus))
        sys.exit(2)
    same_dev = os.environ.get("CLK_BENCH_SAME_DEVICE") == "1"

    import torch
    if world > 1 and not same_dev and torch.cuda.device_count() < world:
        log("bench: --gpus %d but %d GPUs visible" % (world, torch.cuda.device_count()))
        sys.exit(2)
    import click_amd

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CLK_BENCH_SAME_DEVICE=1 + CLK_BENCH_BACKEND=gloo rehearse the
    # multi-rank code path with every rank on GPU 0 (RCCL refuses duplicate
    # GPUs); the driver's N>1 runs use RCCL, one rank per GPU.
    dev = 0 if same_dev else local
    torch.cuda.set_device(dev)
    dist = None
    coll_dev = "cuda"
    # CLK_BENCH_DIST_WORLD1=1 (tests): one rank through the communicator
    # anyway (WORLD_SIZE=1 and the MASTER_* variables set), so the RCCL code
    # path -- init, barriers, all-reduce / all-gather of device tensors,
    # grouped send/recv -- runs on a one-GPU box
    if world > 1 or os.environ.get("CLK_BENCH_DIST_WORLD1") == "1":
        import torch.distributed as dist
        backend = os.environ.get("CLK_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
            coll_dev = "cpu"
    ctx = click_amd.Context(dev)
    load_torch_kernels(torch)
    if args.e2e:
        w = WORKLOADS[args.workload]
        res = [e2e(torch, ctx, args.workload, el) for el in w["elements"]]
        pull = pull_legs() if rank == 0 else None
        threads = glue_thread_legs() if rank == 0 else None
        if rank == 0:
            out = {"e2e": res, "pull": pull, "glue_threads": threads}
            # the push legs through the adapter core beside the same run's
            # one-thread CPU CheckUDPHeader (oracle, 1500 B, DRAM-resident)
            try:
                cpu1 = cpu_baseline(legs=("c3",), single_only=True)["legs"]["c3"]["single_thread"]
                legs = {x["leg"]: x for x in pull if isinstance(x, dict) and "leg" in x} if isinstance(pull, list) else {}
                out["core_vs_cpu_c3"] = {"cpu_one_thread_mpps": cpu1.get("mpps"),
                                         **{k: {"mpps": legs[k]["mpps"], "x_cpu": round(legs[k]["mpps"] / cpu1["mpps"], 2)}
                                            for k in ("push_c3_staged", "push_c3_zerocopy") if k in legs}}
            except Exception as e:        # reported, not fatal
                out["core_vs_cpu_c3"] = {"error": repr(e)}
            print(json.dumps(out), flush=True)
        ctx.close()
        return
    pk = args.packets or None
    meas = lambda wl: measure(torch, ctx, dist, rank, world, wl, args.steps, args.warmup, packets=pk,
                              coll_dev=coll_dev, verify=not args.no_verify)
    main_res = meas(args.workload)
    c2 = None
    if args.workload != "c2" and not args.no_c2:
        c2 = meas("c2")
    # the other configurations of BASELINE.json, reported beside the
    # headline (C4: IMIX 64M; C5: 9000 B, 16M per GPU = 128M at N = 8)
    extra = {}
    for sect, wl in (("c4_imix", "c4"), ("c5_jumbo", "c5")):
        if args.workload != wl and wl not in args.skip.split(","):
            extra[sect] = (wl, meas(wl))
    frag = None
    if args.workload == "c3" and not args.no_frag:
        frag = measure_fragmenter(torch, ctx, dist, rank, world, args.steps, args.warmup, packets=pk,
                                  coll_dev=coll_dev)
    peak_shapes = {}
    peak_meas = None if args.no_peak else read_stream_peak(torch, ctx, detail=peak_shapes)
    copy_meas = None if args.no_peak else copy_stream_peak(torch, ctx)
    c1 = None
    if rank == 0 and world == 1 and not args.no_c1:
        c1 = config1(ctx)
    drop_in = None
    if rank == 0 and world == 1 and not args.no_click:
        drop_in = click_drop_in()

    # an input that starts on one GPU would first be scattered;
    # measured on a sample after the timed regions, never part of `value`
    rsc = None
    if dist is not None and world > 1 and args.scatter_bytes > 0:
        from click_amd import shard
        r_ = shard.root_scatter(torch, dist, coll_dev, args.scatter_bytes)
        if r_:
            t_, b_ = r_
            w_ = WORKLOADS[args.workload]
            per_rank = (pk or w_["n"]) * (w_["stride"] or 354)       # C4: the IMIX mean
            rsc = {"sample_bytes_per_rank": args.scatter_bytes, "seconds": round(t_, 5),
                   "GBps_out_of_rank0": round(b_ / t_ / 1e9, 1),
                   "whole_shards_s": {args.workload: round(per_rank * (world - 1) * t_ / b_, 3),
                                      "c5": round((16 << 20) * 9024 * (world - 1) * t_ / b_, 3)},
                   "note": "rank 0 sends each other rank its piece (grouped send/recv over RCCL); "
                           "an input that starts on one GPU, not the device-resident value"}
    comm = comm_info(torch, dist, dev)         # a collective: every rank joins
    if rank == 0:
        w = WORKLOADS[args.workload]
        head = main_res[w["elements"][0]]
        hs = summarize(head, args.steps, args.workload)
        hs["roofline"]["read_stream_measured_GBs"] = round(peak_meas, 1) if peak_meas else None
        hs["roofline"]["read_stream_shapes_GBs"] = peak_shapes or None
        # frac is against the 8 TB/s spec; this one against the read ceiling
        # measured in the same run (read_stream_kernel: the best probe shape)
        hs["roofline"]["frac_of_measured_read"] = round(hs["roofline"]["achieved"] / peak_meas, 4) if peak_meas else None
        if copy_meas:
            # the ceilings of the read+write kernels (IPFragmenter, the IMIX
            # Set): a copy of equal streams, and the Set's own block pattern
            hs["roofline"]["copy_stream_measured_GBs"] = copy_meas[1]
            hs["roofline"]["copy_stream_shapes_GBs"] = copy_meas[0]
        line = {
            "metric": METRIC, "value": hs["value"], "unit": "GiB/s", "mpps": hs["mpps"],
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": hs["ms_per_step"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic (splitmix64 IPv4 packets generated in HBM)",
            "config": {"workload": w["desc"], "element": head["element"], "packets_per_gpu": head["n"],
                       "packet_bytes": w["L"] or "imix", "slot_bytes": w["stride"] or "64B-aligned",
                       "parallelism": "dp%d (disjoint packet shards, no data-path collective)" % world},
            "roofline": hs["roofline"],
            "verify": hs["verify"],
            # the library reads no environment variable; bench-side CLK_* test
            # switches present in this run are recorded here
            "clk_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("CLK_")},
            "elements": {e: summarize(r, args.steps, args.workload) for e, r in main_res.items()},
            "comm": comm,
        }
        if rsc:
            line["root_scatter"] = rsc
        if c2:
            line["c2_64b"] = {"workload": WORKLOADS["c2"]["desc"],
                              "elements": {e: summarize(r, args.steps, "c2") for e, r in c2.items()}}
            for e, r in c2.items():
                line["c2_64b"]["elements"][e]["slot_GBs"] = round(
                    (64 + SLOT_EXTRA[e]) * r["n"] / (r["kernel_ms"] * 1e-3) / 1e9, 1)
        for sect, (wl, res) in extra.items():
            line[sect] = {"workload": WORKLOADS[wl]["desc"],
                          "elements": {e: summarize(r, args.steps, wl) for e, r in res.items()}}
            if copy_meas and wl == "c4":
                for e, r in line[sect]["elements"].items():
                    if e.startswith("Set"):            # against the measured read + one-block-in-six pattern
                        r["roofline"]["frac_of_set_pattern"] = round(r["roofline"]["achieved"] / copy_meas[2], 4)
        if frag:
            if copy_meas:
                frag["roofline"]["frac_of_measured_copy"] = round(frag["roofline"]["achieved"] / copy_meas[1], 4)
            line["fragmenter"] = frag
        if c1:
            line["c1_fake_iprouter"] = c1
        if drop_in:
            line["drop_in"] = drop_in
        if world == 1 and not args.no_cpu:
            try:
                cb = cpu_baseline()
                if c1:
                    cb["legs"]["c1"] = config1_cpu()
                log("bench: cpu_baseline detail " + json.dumps(cb))     # the full legs, on stderr
                head_leg = cb["legs"].get(args.workload, {}).get("all_cores", {})
                line["cpu_baseline"] = {
                    "value": head_leg.get("value"), "unit": "GiB/s", "cores": cb["threads"], "kind": "port",
                    "mpps": head_leg.get("mpps"),
                    "sample": "%s over %s packets (%s B, DRAM-resident, NUMA-local shards), median of 5"
                              % (cb["legs"][args.workload]["element"], head_leg.get("packets"),
                                 head_leg.get("sample_bytes")),
                    "cpu": cb["host"]["model"], "quota": cb["host"]["quota"], "method": cb["method"],
                    "legs": compact_legs(cb["legs"])}
            except Exception as e:        # reported, not fatal
                line["cpu_baseline"] = {"error": repr(e)}
        # last key: one entry per timed element, so that the tail of the line
        # alone (the driver keeps the last few KB of stdout) carries them all
        line["summary"] = bench_summary(line)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
