"""Debug: per-variant kernel durations from a rocprofv3 kernel_trace.csv of tools/tune.py
(variants load their own code objects; first-dispatch order = variant order)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat = sys.argv[2] if len(sys.argv) > 2 else "frag"
d = collections.OrderedDict()
meta = {}
for r in rows:
    n = r["Kernel_Name"]
    if pat not in n:
        continue
    k = (n.split("(")[0][-44:], r["Kernel_Id"])
    d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
for k, v in d.items():
    print(k, len(v), "median_ms", round(sorted(v)[len(v) // 2], 3), "vgpr/sgpr/lds/scratch", meta[k])
