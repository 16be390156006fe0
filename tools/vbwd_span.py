"""Span (first launch start -> last end) of the ResNet backward in a rocprofv3 kernel trace,
per step that runs it (avgpool_bwd .. stem_wgrad_unpack), plus the summed kernel time of the
BN-backward kernels in that window. usage: python tools/vbwd_span.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
i = 0
while i < len(rows):
    if "avgpool_bwd" in rows[i]["Kernel_Name"]:
        j = i
        while j < len(rows) and "stem_wgrad_unpack" not in rows[j]["Kernel_Name"]:
            j += 1
        if j == len(rows):
            break
        seg = rows[i:j + 1]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in seg)
        bn = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg
                 if any(k in r["Kernel_Name"] for k in ("bn_bwd", "bn_ws_fold", "bn_grad_fin", "stem_bwd", "stem_pool")))
        print(f"video bwd span {(t1 - t0) / 1e6:7.3f} ms, BN-bwd kernels {bn / 1e6:6.3f} ms, {len(seg)} launches")
        i = j
    i += 1
