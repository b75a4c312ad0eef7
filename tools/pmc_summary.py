#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/.

Reads the rocprofv3 CSVs (kernel trace + stats, FETCH_SIZE pass, WRITE_SIZE
pass) and writes
  profiles/<tag>/<workload>_kernel_stats.csv   (rocprofv3 --stats summary)
  profiles/<tag>/<workload>_pmc.json           (per-kernel counters)
  profiles/pmc_<workload>.json                 (what bench.py reads)
The element duration is the mean over all traced launches (what the
rocprofv3 --stats summary shows) and, as duration_ms_timed, over the last
<steps> launches of each kernel: bench.py's timed region, after its warm-up.
HBM bytes per launch of the element kernel =
  2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(FETCH_SIZE is in KiB and reads exactly half the bytes of a wide coalesced
stream on gfx950; WRITE_SIZE is exact for 16 B-per-lane stores and
uncalibrated for narrower ones -- MI355X_MICROARCH.md, HBM).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# element -> kernels one call launches (two-phase Set = compute + scatter;
# fixed-geometry l4_kernel or the variable-length l4_stream_kernel)
ELEMENT_KERNELS = {
    "CheckUDPHeader": ["l4_kernel<17, false", "l4_stream_kernel<17, false"],
    "SetUDPChecksum": ["l4_kernel<17, true", "l4_stream_kernel<17, true", "field_scatter_kernel<6>"],
    "CheckTCPHeader": ["l4_kernel<6, false", "l4_stream_kernel<6, false"],
    "SetTCPChecksum": ["l4_kernel<6, true", "l4_stream_kernel<6, true", "field_scatter_kernel<16>"],
    "CheckICMPHeader": ["l4_kernel<1, false", "l4_stream_kernel<1, false"],
    "CheckIPHeader": ["ip_header_kernel<0"],
    "SetIPChecksum": ["ip_header_kernel<2"],
    "DecIPTTL": ["dec_ttl_kernel"],
    "IPOutputCombo": ["ip_out_kernel<2"],
    # one launch (frag_write_kernel<true, false>), two (<true, true> + the flat pass) or three
    "IPFragmenter": ["frag_plan_kernel", "frag_scan_kernel", "frag_write_kernel", "frag_flat_kernel"],
}


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return hits[0] if hits else None


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    out, tag, wl = sys.argv[1:4]
    pdir = os.path.join(ROOT, sys.argv[4] if len(sys.argv) > 4 else "profiles", tag)
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    os.makedirs(pdir, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    trace = find(os.path.join(out, "trace"), "*kernel_trace.csv")
    res = {"workload": wl, "tag": tag}
    if stats:
        shutil.copy(stats, os.path.join(pdir, "%s_kernel_stats.csv" % wl))
    durs = {}
    if trace:
        for r in rows(trace):
            n = short(r["Kernel_Name"])
            durs.setdefault(n, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    durs = {k: [(e - b) * 1e-6 for b, e in sorted(v)] for k, v in durs.items()}     # launch order
    res["trace_ms"] = {k: {"calls": len(v), "mean_ms": statistics.mean(v), "min_ms": min(v)}
                       for k, v in durs.items()}
    counters = {}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write"), ("TCC_EA0_WRREQ_sum", "wrreq"),
                       ("TCC_EA0_WRREQ_64B_sum", "wrreq")):
        p = find(os.path.join(out, sub), "*counter_collection.csv")
        if not p:
            continue
        per = {}
        for r in rows(p):
            if r.get("Counter_Name") not in (cname, cname.replace("_sum", "")):
                continue
            n = short(r["Kernel_Name"])
            per.setdefault(n, []).append(float(r["Counter_Value"]))
        counters[cname] = {k: statistics.median(v) for k, v in per.items()}
    res["counters_kib"] = counters
    res["elements"] = {}
    for el, pats in ELEMENT_KERNELS.items():
        ks = [k for k in durs if any(k.startswith("clk::" + p) for p in pats)]
        if not ks:
            continue
        e = {"kernels": ks, "duration_ms": sum(statistics.mean(durs[k]) for k in ks)}
        if steps:
            e["duration_ms_timed"] = sum(statistics.mean(durs[k][-steps:]) for k in ks)
        if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
            f = sum(counters["FETCH_SIZE"].get(k, 0.0) for k in ks)
            w = sum(counters["WRITE_SIZE"].get(k, 0.0) for k in ks)
            e["fetch_bytes_raw"] = f * 1024
            e["fetch_bytes_corrected"] = 2 * f * 1024
            e["write_bytes"] = w * 1024
            e["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
        if "TCC_EA0_WRREQ_sum" in counters and "TCC_EA0_WRREQ_64B_sum" in counters:
            q = sum(counters["TCC_EA0_WRREQ_sum"].get(k, 0.0) for k in ks)
            q64 = sum(counters["TCC_EA0_WRREQ_64B_sum"].get(k, 0.0) for k in ks)
            e["write_requests"] = q
            e["write_requests_64B"] = q64
            e["write_requests_partial"] = q - q64     # (MI355X_MICROARCH.md: partial-line writes cost a read-modify-write)
        if len(ks) > 1:                          # each kernel's share
            e["per_kernel"] = {k: {"duration_ms": statistics.mean(durs[k]),
                                   "hbm_bytes": (2 * counters.get("FETCH_SIZE", {}).get(k, 0.0)
                                                 + counters.get("WRITE_SIZE", {}).get(k, 0.0)) * 1024,
                                   "write_requests_partial": (counters.get("TCC_EA0_WRREQ_sum", {}).get(k, 0.0)
                                                              - counters.get("TCC_EA0_WRREQ_64B_sum", {}).get(k, 0.0))}
                               for k in ks}
        res["elements"][el] = e
    with open(os.path.join(pdir, "%s_pmc.json" % wl), "w") as fh:
        json.dump(res, fh, indent=1)
    with open(os.path.join(os.path.dirname(pdir), "pmc_%s.json" % wl), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
