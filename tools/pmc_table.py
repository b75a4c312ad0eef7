#!/usr/bin/env python3
"""Average each counter per dispatch, per kernel, over the passes that
tools/pmc_kernel.sh wrote (counter_collection.csv files)."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"][:70]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if not k.startswith("clk::") and "l4" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-32s %16.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
