#!/usr/bin/env python3
"""Where the two-phase Set's time goes (C3 or C5 batch, one process).

Times every launch by HIP events on the launch stream, in sequences:
  check            Check element alone, back to back
  set              two-phase Set (compute pass + field_scatter_kernel)
  compute          the Set's compute pass alone (CLK_DIAG_SET_PHASE=1)
  scatter          the scatter alone over the last work words (=2)
  alt_compute / alt_scatter   compute and scatter alternating, each timed
  after_scatter_check         a Check launched right after a scatter
and the same for variant libraries built by tools/tune.py --build
(--variants).  Diagnostics only; results of the phase-split runs are not
checked.
  python tools/probes/set_phases.py --workload c3 --variants base,setruns16
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--reps", type=int, default=12)
    args = ap.parse_args()
    import torch
    import click_amd
    import bench
    import tune
    w = bench.WORKLOADS[args.workload]
    n = w["n"]
    if args.workload == "c4":
        off, ln, total, _ = bench.imix_layout(torch, n, 0x5EED, 0)
        arena = torch.empty(total, dtype=torch.uint8, device="cuda")
        b = click_amd.Batch(arena, n, off=off, length=ln, max_len=1500)
    else:
        arena = torch.empty(n * w["stride"], dtype=torch.uint8, device="cuda")
        b = click_amd.Batch(arena, n, stride=w["stride"], fixed_len=w["L"])
    c0 = click_amd.Context(0)
    c0.gen_packets(b, proto=w["proto"])
    c0.set_ip_checksum(b, want_sums=False)
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    udp = w["proto"] == 17
    set_name, check_name = ("SetUDPChecksum", "CheckUDPHeader") if udp else ("SetTCPChecksum", "CheckTCPHeader")

    def ctx(variant, phase):
        env = dict(tune.VARIANTS[variant][1], CLK_DIAG_SET_PHASE=str(phase))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return click_amd.Context(0, lib_path=tune.lib_for(variant))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v

    def setf(c):
        return (c.set_udp_checksum if udp else c.set_tcp_checksum)(b, status=status, want_sums=False)

    def checkf(c):
        return (c.check_udp_header if udp else c.check_tcp_header)(b, out=status)

    def timed(seq, reps):
        """seq: list of (label, fn); returns {label: [ms, ...]} over reps passes."""
        out = {lab: [] for lab, _ in seq}
        evs = []
        for _ in range(reps):
            for lab, fn in seq:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                evs.append((lab, s, e))
        torch.cuda.synchronize()
        for lab, s, e in evs[len(seq):]:          # the first pass is warm-up
            out[lab].append(s.elapsed_time(e))
        return out

    res = {}
    for v in args.variants.split(","):
        full, comp, scat = ctx(v, 0), ctx(v, 1), ctx(v, 2)
        setf(full)           # work words in the scratch of each context
        setf(comp)
        setf(scat)
        torch.cuda.synchronize()
        # the scatter-only context needs work words: run its compute once by a full call on it
        seqs = {
            "check": [("check", lambda: checkf(full))],
            "set": [("set", lambda: setf(full))],
            "compute": [("compute", lambda: setf(comp))],
            "alt": [("alt_compute", lambda: setf(comp)), ("alt_scatter", lambda: setf(scat))],
            "after_scatter": [("scatter", lambda: setf(scat)), ("after_scatter_check", lambda: checkf(full))],
            # ~1 ms of an idle spin between the scatter and the Check: does the write-back drain by itself?
            "gap": [("gap_scatter", lambda: setf(scat)), ("gap_sleep", lambda: torch.cuda._sleep(2_000_000)),
                    ("gap_check", lambda: checkf(full))],
        }
        r = {}
        for _ in range(2):                        # two interleaved rounds
            for name, seq in seqs.items():
                for lab, t in timed(seq, args.reps).items():
                    r.setdefault(lab, []).extend(t)
        res[v] = {lab: round(statistics.median(t), 4) for lab, t in r.items()}
        for c in (full, comp, scat):
            c.close()
    print(json.dumps({"workload": args.workload, "median_ms": res}))


if __name__ == "__main__":
    main()
