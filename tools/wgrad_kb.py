"""Stage-1 / stage-2 patch-resident weight-grads at C2 (6000 images), 5 launches each: a short
program for rocprofv3 --pmc passes (tools/gpu_pmc.sh PROGS=wgrad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402

dev = torch.device("cuda")
N = 16 * 375
for hw, c in ((22, 64), (11, 128)):
    geom = ops.ConvGeom(N, hw, hw, c, c, 3, 3, (1, 1), (1, 1))
    x = torch.randn(N * hw * hw, c, device=dev).to(torch.bfloat16)
    dy = torch.randn(N * hw * hw, c, device=dev).to(torch.bfloat16)
    dw = torch.zeros(c, 3, 3, c, device=dev)
    for _ in range(5):
        ops.conv_bwd_weight(geom, x, dy, dw)
    torch.cuda.synchronize()
    del x, dy
print("ok")
