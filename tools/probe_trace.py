"""Average duration of the bench roofline probe kernel in a rocprofv3 kernel trace, selected
by kernel name and grid size (FFN1 fwd at C2 on the 192x128 tile: 1024 workgroups x 256 threads = 262144), to
cross-check bench.py's live HIP-event average.
  python tools/probe_trace.py <run_kernel_trace.csv> [grid_threads] [name_substring]"""
import csv
import sys

path = sys.argv[1]
grid = sys.argv[2] if len(sys.argv) > 2 else "262144"
sub = sys.argv[3] if len(sys.argv) > 3 else "dense_glds_kernel"
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(path))
       if sub in r["Kernel_Name"] and r["Grid_Size_X"] == grid and "true, gemmg" in r["Kernel_Name"]
       and "false, true" not in r["Kernel_Name"]]
if not dur:
    sys.exit(f"no {sub} launches with grid {grid}")
dur.sort()
trim = dur[len(dur) // 20: len(dur) - len(dur) // 20] or dur     # 5 % trimmed (a launch queued behind a sync)
print(f"probe kernel: {sub} (A, B k-major = forward), grid {grid} threads: n={len(dur)} "
      f"avg={sum(dur) / len(dur):.1f} us trimmed-avg={sum(trim) / len(trim):.1f} us median={dur[len(dur) // 2]:.1f} "
      f"min={min(dur):.1f} max={max(dur):.1f}")
