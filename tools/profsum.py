"""Summarise a rocprofv3 kernel trace per training step.

  python tools/profsum.py <run_kernel_trace.csv> [last_steps] [top] [--grid] [--skip S]

Steps are delimited by the optimizer launches (adamw_kernel closes each step); only the last
`last_steps` steps are counted so setup work (initial shadow cast, warm-up) is excluded.
"""
import csv
import sys
from collections import defaultdict


def step_ends(rows, gap_ns=15_000_000):
    """row indices closing each training step: the last optimizer (adamw_kernel) launch of each
    cluster of launches that start within gap_ns of the previous one (2 per step serial, 4 with
    the overlapped update: front segments on the step stream, the rest on the update stream)"""
    ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    ends = []
    for j, i in enumerate(ad):
        nxt = ad[j + 1] if j + 1 < len(ad) else None
        if nxt is None or int(rows[nxt]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"]) > gap_ns:
            ends.append(i)
    return ends

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30


def load_rows(path):
    if path.endswith(".db"):   # rocprofv3 default (rocpd sqlite) output
        import sqlite3
        c = sqlite3.connect(path)
        q = ("select s.kernel_name, d.start, d.end, d.grid_size_x, d.grid_size_y, d.grid_size_z "
             "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        return [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b, "Grid_Size_X": x, "Grid_Size_Y": y,
                 "Grid_Size_Z": z} for n, a, b, x, y, z in c.execute(q)]
    return list(csv.DictReader(open(path)))


rows = sorted(load_rows(path), key=lambda r: int(r["Start_Timestamp"]))
ends = step_ends(rows)
# --skip S: leave out the last S steps (bench --quick appends 12 per-variant steps: none x4,
# audio_off x4, video_off x4, one lead-in + 3 timed each; the forced timed steps are the 4 before them)
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
if skip:
    ends = ends[:-skip]
if len(ends) > last:
    rows = rows[ends[-last - 1] + 1: ends[-1] + 1]
    steps = last
else:
    steps = max(1, len(ends))
by_grid = "--grid" in sys.argv
agg = defaultdict(lambda: [0.0, 0])
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    key = r["Kernel_Name"]
    if by_grid:
        key = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]} ' + key
    a = agg[key]
    a[0] += d
    a[1] += 1
tot = sum(v[0] for v in agg.values())
wall = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6 / steps
for name, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{t / 1e6 / steps:8.2f} ms/step {100 * t / tot:6.2f}% n={n / steps:6.1f}/step "
          f"avg={t / n / 1e3:8.1f}us  {name[:110]}")
print(f"kernel total {tot / 1e6 / steps:.2f} ms/step, span {wall:.2f} ms/step over {steps} steps")
