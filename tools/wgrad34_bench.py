"""ResNet stage-3 / stage-4 weight-grads at C2 (6000 images) in isolation: the patch-resident
kernel (conv_wgrad_patch + ordered slab reduce) against the general implicit-GEMM weight-grad
(option conv_wpatch = 0), HIP-event time per call, TFLOP/s and the relative difference of the
two results. usage: python tools/wgrad34_bench.py [out.json]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import _lib as L, ops  # noqa: E402

dev = torch.device("cuda")
N = 16 * 375
REPS = 10
res = {}
for hw, c in ((6, 256), (3, 512)):
    geom = ops.ConvGeom(N, hw, hw, c, c, 3, 3, (1, 1), (1, 1))
    x = torch.randn(N * hw * hw, c, device=dev).to(torch.bfloat16)
    dy = torch.randn(N * hw * hw, c, device=dev).to(torch.bfloat16)
    flop = 2.0 * N * hw * hw * c * 9 * c
    out = {}
    for name, opt in (("patch", 1), ("general", 0)):
        prev = L.set_option("conv_wpatch", opt)
        dw = torch.zeros(c, 3, 3, c, device=dev)
        ops.conv_bwd_weight(geom, x, dy, dw)
        ref = dw.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            ops.conv_bwd_weight(geom, x, dy, dw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / REPS
        L.set_option("conv_wpatch", prev)
        out[name] = {"us": round(us, 1), "tflops": round(flop / us / 1e6, 1), "frac": round(flop / us / 1e6 / 2500, 3)}
        out[name + "_dw"] = ref
    d = (out.pop("patch_dw") - out["general_dw"]).norm() / out["general_dw"].norm()
    out.pop("general_dw")
    out["rel_diff"] = float(d)
    res[f"{hw}x{hw}x{c}"] = out
    print(f"{hw}x{hw}x{c}", json.dumps(out), flush=True)
    del x, dy
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
