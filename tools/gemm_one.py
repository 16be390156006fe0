"""Run one GEMM shape/layout N times (for rocprofv3 counter passes).
usage: python tools/gemm_one.py M N K [fwd|ffn1|dgrad|wgrad] [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops

M, N, K = (int(a) for a in sys.argv[1:4])
kind = sys.argv[4] if len(sys.argv) > 4 else "fwd"
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
dev = torch.device("cuda")
ops.L.set_option("gemm_tile", os.environ.get("GEMM_TILE", "auto"))
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
dW = torch.zeros(N, K, device=dev)
bias = torch.zeros(N, device=dev)
h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
fn = {"fwd": lambda: ops.linear_fwd(x, W),
      "ffn1": lambda: ops.linear_fwd(x, W, bias, act=1, preact=h, drop_p=0.1, seed=7),   # bench probe's epilogue
      "dgrad": lambda: ops.linear_dgrad(dy, W),
      "wgrad": lambda: ops.linear_wgrad(dy, x, dW)}[kind]
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", M, N, K, kind, os.environ.get("GEMM_TILE", "auto"))
