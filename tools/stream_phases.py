"""Per-step phase timeline of a rocprofv3 kernel trace: for each training step (delimited by
the AdamW launches) the forward / backward / optimizer spans, per-stream busy time inside each
span, and the union busy time (GPU idle = span - union).
usage: python tools/stream_phases.py run_kernel_trace.csv [last_steps] [--skip S]
(--skip S: leave out the last S steps, as in tools/profsum.py)"""
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

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "--skip" else 3
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
ends = step_ends(rows)
if skip:
    ends = ends[:-skip]
steps = list(zip(ends[:-1], ends[1:]))[-last:]


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def phase(seg, name):
    if not seg:
        return
    t0 = min(int(r["Start_Timestamp"]) for r in seg)
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    per = defaultdict(list)
    for r in seg:
        per[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    u = union([x for v in per.values() for x in v])
    busy = " ".join(f"s{k}:{union(v) / 1e6:6.2f}" for k, v in sorted(per.items()))
    work = sum(e - s for v in per.values() for s, e in v)
    print(f"  {name:9s} span {(t1 - t0) / 1e6:7.2f} ms  union {u / 1e6:6.2f}  idle {(t1 - t0 - u) / 1e6:5.2f}  "
          f"sum {work / 1e6:6.2f}  {busy}  n={len(seg)}")


for a, b in steps:
    seg = rows[a + 1:b + 1]
    # backward starts at the first kernel named *bwd* / dgrad after the loss kernels: use the
    # CTC backward (loss.hip ctc_bwd_kernel) as the boundary (it runs right after the forward)
    cut = next((i for i, r in enumerate(seg) if "ctc_bwd" in r["Kernel_Name"] or "lsm_bwd" in r["Kernel_Name"]), None)
    # optimizer: from the LAST gradient-norm pass of the step (the early one, engine.EARLY_NORM, runs
    # on the side stream inside the backward)
    opt = max((i for i, r in enumerate(seg) if "sumsq_kernel" in r["Kernel_Name"]), default=len(seg) - 2)
    print(f"step ({len(seg)} kernels)")
    phase(seg[:cut], "forward")
    phase(seg[cut:opt], "backward")
    phase(seg[opt:], "optimizer")
    phase(seg, "total")
