"""Split-K sweep of the Linear weight gradient dW[N][K] += dy^T x (tokens M=6000) on the
encoder / decoder-head shapes, with the slab workspace. usage: python tools/lin_wgrad_sweep.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops


def t(fn, n=10, reps=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / (n * reps)



dev = torch.device("cuda")
M = 6000
for N, K in [(1024, 1024), (3072, 1024), (4096, 1024), (1024, 4096), (5056, 1024), (1024, 2048)]:
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dW = torch.zeros(N, K, device=dev)
    fl = 2.0 * M * N * K
    out = []
    for sk in (1, 2, 3, 4, 6, 8):
        ws = torch.empty(sk * N * K, device=dev) if sk > 1 else None
        ms = t(lambda: ops.gemm(dy, x, dW, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=N, ldb=K, ldc=K,
                                alpha=1.0, beta=1.0, splitk=sk, ws=ws))
        out.append(f"sk{sk} {ms * 1e3:6.1f}us {fl / ms / 1e9:4.0f}TF")
    print(f"[{os.environ.get('AVSR_GEMM_TILE', 'auto')}] wgrad N{N} K{K}: " + "  ".join(out), flush=True)
