"""Stem weight-gradient (the Conv3d stem as a 2-D conv over 8 time-stacked channels: 88x88x8 ->
44x44x64, 7x7, stride 2, pad 3) at C2 (6000 frames), HIP-event timed, the patch-resident kernel
(option stem_wpatch = 1) and the general implicit GEMM (0): python tools/stem_wgrad_kbench.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import _lib, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
N = 16 * 375
xp = torch.randn(N, 88, 88, 8, generator=g).to(dev, torch.bfloat16)
xp[..., 5:] = 0
dh0 = torch.randn(N * 44 * 44, 64, generator=g).to(dev, torch.bfloat16)
gs = ops.ConvGeom(N, 88, 88, 8, 64, 7, 7, (2, 2), (3, 3))
gp = torch.zeros(64, 7, 7, 8, device=dev)
fn = lambda: ops.conv_bwd_weight(gs, xp, dh0, gp)      # noqa: E731
fl = 2.0 * N * 44 * 44 * 64 * 7 * 7 * 8
for opt in (1, 0):
    _lib.set_option("stem_wpatch", opt)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    print(f"stem weight-grad (stem_wpatch={opt}): median {ts[len(ts) // 2]:.1f} us "
          f"({fl / ts[len(ts) // 2] / 1e6:.0f} TF/s on the 8-channel K), "
          f"dz {dh0.numel() * 2 / 1e9:.2f} GB, input {xp.numel() * 2 / 1e9:.2f} GB", flush=True)
