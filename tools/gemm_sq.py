"""bf16 GEMM cores on square and encoder shapes (random [-1,1) operands, HIP-graph timed):
library option gemm_tile in {auto, 128, pp, 256}. usage: python tools/gemm_sq.py [cfg,cfg,...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402
from tools.gemm_table import timed  # noqa: E402

dev = torch.device("cuda")
cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["128", "pp", "256"]
shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (6144, 4096, 1024), (6000, 4096, 1024), (6000, 3072, 1024),
          (6000, 1024, 4096), (6000, 1024, 1024)]
for M, N, K in shapes:
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    W = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    fl = 2.0 * M * N * K
    line = f"M{M:5d} N{N:5d} K{K:5d}"
    for c in cfgs:
        ops.L.set_option("gemm_tile", c)
        us = timed(lambda: ops.linear_fwd(x, W), n=5 if M > 4096 else 10)
        line += f"  {c}: {us:8.1f}us {fl / us / 1e6:6.0f}TF"
    ops.L.set_option("gemm_tile", "auto")
    print(line, flush=True)
