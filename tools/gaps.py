"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (host-bound stretches).
  python tools/gaps.py <run_kernel_trace.csv> [min_gap_us]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
lo, hi = ends[-7], ends[-1]          # last 3 steps (2 adamw launches per step)
agg = defaultdict(lambda: [0, 0.0])
tot = 0.0
for i in range(lo + 1, hi + 1):
    g = (int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3
    if g > thr:
        k = rows[i - 1]["Kernel_Name"][:70] + "  ->  " + rows[i]["Kernel_Name"][:50]
        agg[k][0] += 1; agg[k][1] += g
    tot += max(g, 0)
print(f"total gap {tot / 3:.2f} ms/step")
for k, (n, g) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{g / 3:8.3f} ms/step n={n / 3:5.1f}  {k}")
