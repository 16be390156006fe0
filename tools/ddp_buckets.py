"""Multi-GPU readiness analysis (no hardware): when each 64 MiB gradient bucket of the arena
becomes ready in a measured single-GPU video-on step, and how much of its ring all-reduce an
8-GPU run could not hide, for one xGMI link (~153 GB/s) and for all 7.

  python tools/ddp_buckets.py layout.json trace.csv[.gz] [--skip S] [--world 8] [--bucket-mib 64]

layout.json: tools/arena_layout.py. trace: rocprofv3 --kernel-trace CSV of bench.py (video-on
steps); the analysed step is the last one before the --skip trailing steps (steps end at the second
adamw launch). Readiness follows the engine: after encoder layer i's backward the reducer
(parallel.GradReducer.ready) launches every bucket at or above layer i's first decay offset, once
both the step stream and the side stream (weight-gradients) reached that point: layer i's end =
max(its closing LayerNorm backward on the step stream, its QKV weight-gradient — the layer's last
side-stream GEMM). Buckets below layer 0 (frontends, ResNet) and the no-decay / frozen tail go at
the end of the backward. The comm stream runs the buckets back to back; exposed = its end minus
the backward's end."""
import csv
import gzip
import json
import sys

lay = json.load(open(sys.argv[1]))

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

path = sys.argv[2]
arg = lambda k, d: type(d)(sys.argv[sys.argv.index(k) + 1]) if k in sys.argv else d  # noqa: E731
skip, world, bmib = arg("--skip", 0), arg("--world", 8), arg("--bucket-mib", 64)
rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = step_ends(rows)
if skip:
    ends = ends[:-skip]
step = rows[ends[-2] + 1: ends[-1] + 1]
t0 = int(step[0]["Start_Timestamp"])
us = lambda r, k: (int(r[k]) - t0) / 1e3  # noqa: E731
main_q = max(set(r["Queue_Id"] for r in step), key=lambda q: sum(1 for r in step if r["Queue_Id"] == q))
# backward starts at the first attention dK/dV of the encoder (the decoder's come before it, on
# the step stream as well); per encoder layer: its dK/dV, the next LayerNorm backward on the step
# stream, and the next 192-block (QKV) weight-gradient
enc_dkdv = [i for i, r in enumerate(step) if "rb20attn_bwd_dkdv" in r["Kernel_Name"] or "rb::attn_bwd_dkdv" in r["Kernel_Name"]]
layer_end = []
for j, i in enumerate(enc_dkdv):
    ln = next(k for k in range(i, len(step)) if "ln_bwd_kernel" in step[k]["Kernel_Name"] and step[k]["Queue_Id"] == main_q)
    qkv = next(k for k in range(i, len(step)) if "wgrad_dual_kernel" in step[k]["Kernel_Name"] and
               int(step[k]["Grid_Size_X"]) == 192 * 512)
    layer_end.append(max(us(step[ln], "End_Timestamp"), us(step[qkv], "End_Timestamp")))
# the gradient-norm partials (sumsq) of finished arena segments run during the backward: the
# backward ends with the last other kernel before the first AdamW launch
opt0 = next(i for i, r in enumerate(step) if "adamw_kernel" in r["Kernel_Name"])
bwd_end = max(us(r, "End_Timestamp") for r in step[:opt0] if "sumsq" not in r["Kernel_Name"])
bwd_start = us(step[enc_dkdv[0]], "Start_Timestamp")
d0, d1 = lay["segments"]["decay"]
n = lay["total"]
step_el = bmib * (1 << 20) // 4
buckets, e = [], d1
while e > d0:
    s = max(d0, e - step_el)
    buckets.append((s, e))
    e = s
tail = [(a, min(n, a + step_el)) for a in range(d1, n, step_el)] + [(a, min(d0, a + step_el)) for a in range(0, d0, step_el)]
offs = lay["layer_decay_off"]                     # per layer index 0..23; backward visits 23 first
ready = []
for s, e in buckets:
    t = None
    for j, li in enumerate(range(len(offs) - 1, -1, -1)):      # j-th layer of the backward = layer li
        if j < len(layer_end) and offs[li] <= s:
            t = layer_end[j]
            break
    ready.append(bwd_end if t is None else t)
ready += [bwd_end] * len(tail)
sizes = [(e - s) * 4 for s, e in buckets + tail]
res = {"step_span_ms": round((us(step[-1], "End_Timestamp")) / 1e3, 2), "backward_ms": round((bwd_end - bwd_start) / 1e3, 2),
       "grad_bytes": sum(sizes), "buckets": []}
for i, ((s, e), t, b) in enumerate(zip(buckets + tail, ready, sizes)):
    res["buckets"].append({"i": i, "MiB": round(b / 2 ** 20, 1), "ready_ms_before_bwd_end": round((bwd_end - t) / 1e3, 2)})
for name, bw in (("1 link (153 GB/s)", 153e9), ("7 links (7 x 153 GB/s)", 7 * 153e9)):
    tcomm = 0.0
    for t, b in sorted(zip(ready, sizes)):
        dur = 2 * (world - 1) / world * b / bw * 1e6 + 30.0       # + ~30 us per collective launch
        tcomm = max(tcomm, t) + dur
    res[f"exposed_ms_{name}"] = round(max(0.0, tcomm - bwd_end) / 1e3, 2)
    res[f"comm_ms_{name}"] = round(sum(2 * (world - 1) / world * b / bw * 1e3 + 0.03 for b in sizes), 2)
print(json.dumps(res, indent=1))
