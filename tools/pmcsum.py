"""Average rocprofv3 counter values per kernel: python tools/pmcsum.py <run_counter_collection.csv>... [name-filter]"""
import collections
import csv
import sys

paths = [a for a in sys.argv[1:] if a.endswith(".csv")]
flt = [a for a in sys.argv[1:] if not a.endswith(".csv")]
for p in paths:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if flt and not any(f in r["Kernel_Name"] for f in flt):
            continue
        agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{p.split('/')[-3]:>12} {c:28s} {sum(v) / len(v):16.1f}  n={len(v)}  {k}")
