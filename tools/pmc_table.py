#!/usr/bin/env python3
"""Average each counter per dispatch, per kernel, over the passes that
tools/pmc_kernel.sh wrote (counter_collection.csv files), and derive the
wave-time split DESIGN.md quotes:
  wait_any    = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waiting on any counter: memory)
  wait_inst   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (waiting for an instruction to issue)
  active_inst = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (issuing)
Usage: pmc_table.py <out dir> [json path]"""
import collections
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, cs in acc.items():
    if not k.startswith("clk::"):
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    d = {"counters": {c: round(x, 1) for c, x in sorted(m.items())}, "dispatches": max(len(v) for v in cs.values())}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for name, c in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                        ("active_inst", "SQ_ACTIVE_INST_ANY")):
            if c in m:
                d[name] = round(m[c] / wc, 4)
    res[k] = d
    print(k)
    for c, x in sorted(m.items()):
        print("   %-32s %16.4g" % (c, x))
    for name in ("wait_any", "wait_inst", "active_inst"):
        if name in d:
            print("   %-32s %16.3f" % (name, d[name]))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as fh:
        json.dump(res, fh, indent=1)
