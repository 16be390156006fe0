"""Sweep the split-K factor of the conv weight-gradient kernel over the ResNet-18 shapes of C2
(6000 images per step) and print us / TFLOP/s per (shape, splits).
usage: python tools/wgrad_sweep.py [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
NIMG = 6000
SHAPES = [  # hw_in, cin, cout, k, stride
    (88, 8, 64, 7, 2), (22, 64, 64, 3, 1), (22, 64, 128, 3, 2), (11, 128, 128, 3, 1), (22, 64, 128, 1, 2),
    (11, 128, 256, 3, 2), (6, 256, 256, 3, 1), (6, 256, 512, 3, 2), (3, 512, 512, 3, 1)]
for hw, cin, cout, k, s in SHAPES:
    g = ops.ConvGeom(NIMG, hw, hw, cin, cout, k, k, stride=(s, s), pad=(k // 2, k // 2))
    x = torch.randn(g.in_pixels, cin, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(g.out_pixels, cout, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(cout, k, k, cin, device=dev)
    fl = 2.0 * g.out_pixels * cout * k * k * cin
    ref = None
    for sp in (0, 64, 128, 256, 512, 1024, 2048, 0):
        dw.zero_()
        ops.conv_bwd_weight(g, x, dy, dw, splitk=sp)
        torch.cuda.synchronize()
        if ref is None:
            ref = dw.clone()
        err = ((dw - ref).abs().max() / ref.abs().max()).item()
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            ops.conv_bwd_weight(g, x, dy, dw, splitk=sp)
        b.record(); torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        print(f"wgrad {hw}x{hw} {cin}->{cout} k{k} s{s} splits {sp:5d}: {ms * 1e3:8.1f} us "
              f"{fl / ms / 1e9:6.0f} TF/s  relerr {err:.1e}", flush=True)
