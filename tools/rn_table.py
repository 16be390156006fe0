"""Per-kernel table of one ResNet fwd+bwd (the last 'fuse=1' iteration of tools/resnet_bench.py)
from a rocprofv3 kernel trace: python tools/rn_table.py <run_kernel_trace.csv>"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# every fwd+bwd iteration starts with the stem input pack; iterations alternate fuse=1 / fuse=0,
# so the last complete fuse=1 one is the second-to-last start
firsts = [i for i, r in enumerate(rows) if "stem_pack" in r["Kernel_Name"]]
seg = rows[firsts[-2]:firsts[-1]]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
print(f"span {(t1 - t0) / 1e6:.2f} ms")
agg = collections.OrderedDict()
for r in seg:
    n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])[:100]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg.setdefault((n, r["Grid_Size_X"]), [0, 0.0])
    a[0] += 1
    a[1] += d
tot = 0.0
for (n, g), (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    tot += d
    print(f"{d:8.1f} us {c:3d}x grid {g:>9} {n}")
print(f"kernel sum {tot:.1f} us")
