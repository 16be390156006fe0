"""GEMM time vs K at fixed M x N (fixed per-tile overhead vs main-loop rate), per tile config.
  AVSR_GEMM_TILE=<cfg> python tools/gemm_k.py [M N]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops


def t(fn, n=10, reps=5):
    """ms per call, n calls captured in one HIP graph, replayed reps times"""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    g.replay()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / (n * reps)


M = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dev = torch.device("cuda")
tag = os.environ.get("AVSR_GEMM_TILE", "auto")
for K in (64, 128, 256, 512, 1024, 2048, 4096):
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    a = t(lambda: ops.linear_fwd(x, W, out=y))
    bias = torch.zeros(N, device=dev)
    h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ae = t(lambda: ops.linear_fwd(x, W, bias, act=1, preact=h, out=y))
    print(f"[{tag}] M{M} N{N} K{K}: {a * 1e3:8.1f} us ({2 * M * N * K / a / 1e9:6.0f} TF/s)  gelu+preact {ae * 1e3:8.1f} us",
          flush=True)
