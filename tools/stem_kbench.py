"""Stem conv (direct, bf16) in isolation at C2 geometry: 16 clips x 375 frames of 88x88.
usage: python tools/stem_kbench.py [iters]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from avsr_amd import ops  # noqa: E402

dev = torch.device("cuda")
B, T = 16, 375
it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
g = torch.Generator(device=dev).manual_seed(0)
video = torch.rand(B, 1, T, 88, 88, device=dev, generator=g)
w = torch.randn(64, 1, 5, 7, 7, device=dev, generator=g) * 0.05
wk = torch.empty(64, ops.STEM_K, device=dev, dtype=torch.bfloat16)
ops.stem_wpack2(w, wk)
h = torch.empty(B * T * 44 * 44, 64, device=dev, dtype=torch.bfloat16)
part = torch.empty(64, ops.stem_conv_tiles(B, T), 3, device=dev)
for _ in range(3):
    ops.stem_conv_fwd(video, wk, h, part)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(it):
    ops.stem_conv_fwd(video, wk, h, part)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / it
print(f"stem_conv_fwd {ms * 1e3:.1f} us  {2 * B * T * 44 * 44 * 64 * 245 / ms / 1e9:.1f} TFLOP/s useful", flush=True)
