"""Micro-benchmark of the HIP GEMM (fwd / dgrad / wgrad shapes of the encoder) vs torch.matmul.
AVSR_GEMM_NOGLDS=1 selects the register-staged core for A/B comparisons."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n


dev = torch.device("cuda")
tag = "noglds" if os.environ.get("AVSR_GEMM_NOGLDS") == "1" else "glds"
for (M, N, K) in [(6000, 1024, 1024), (6000, 3072, 1024), (6000, 4096, 1024), (6000, 1024, 4096), (6000, 5056, 1024),
                  (8192, 8192, 8192)]:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    dW = torch.zeros(N, K, device=dev)
    fl = 2 * M * N * K
    a = t(lambda: ops.linear_fwd(x, W))
    b = t(lambda: ops.linear_dgrad(dy, W))
    c = t(lambda: ops.linear_wgrad(dy, x, dW))
    r = t(lambda: x @ W.t())
    print(f"[{tag}] M{M} N{N} K{K}: fwd {fl/a/1e9:.0f} TF/s  dgrad {fl/b/1e9:.0f}  wgrad {fl/c/1e9:.0f}  "
          f"torch {fl/r/1e9:.0f}", flush=True)
