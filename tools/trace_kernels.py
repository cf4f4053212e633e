"""Median duration per (kernel, grid) from a rocprofv3 kernel-trace CSV: python tools/trace_kernels.py <csv> [substr]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if sub not in n:
        continue
    key = (n.split("(")[0][-40:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"], r["VGPR_Count"])
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in agg.items():
    v = sorted(v)
    print(f"{k[0]:42s} grid {k[1]:>8s} x {k[2]:>3s} wg {k[3]:>4s} vgpr {k[4]:>4s}  n={len(v):4d}  median {v[len(v) // 2]:8.1f} us")
