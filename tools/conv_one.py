"""Run one convolution N times (timing / rocprofv3 counter passes).
usage: python tools/conv_one.py [fwd|dgrad|wgrad] nimg hw cin cout k stride [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops

kind = sys.argv[1]
nimg, hw, cin, cout, k, s = (int(a) for a in sys.argv[2:8])
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 10
dev = torch.device("cuda")
g = ops.ConvGeom(nimg, hw, hw, cin, cout, k, k, stride=(s, s), pad=(k // 2, k // 2))
x = torch.randn(g.in_pixels, cin, device=dev, dtype=torch.bfloat16)
w = torch.randn(cout, k, k, cin, device=dev, dtype=torch.bfloat16) * 0.05
y = torch.empty(g.out_pixels, cout, device=dev, dtype=torch.bfloat16)
dw = torch.zeros(cout, k, k, cin, device=dev)
fn = {"fwd": lambda: ops.conv_fwd(g, x, w, y), "dgrad": lambda: ops.conv_bwd_data(g, y, w, x),
      "wgrad": lambda: ops.conv_bwd_weight(g, x, y, dw)}[kind]
fn()
torch.cuda.synchronize()
a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    fn()
b.record(); torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
fl = 2.0 * g.out_pixels * cout * k * k * cin
print(f"{kind} nimg{nimg} {hw}x{hw} {cin}->{cout} k{k} s{s}: {ms * 1e3:.1f} us  {fl / ms / 1e9:.0f} TF/s")
