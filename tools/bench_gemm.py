"""Micro-benchmark of the HIP GEMM on the encoder's fwd / dgrad / wgrad shapes vs torch.matmul.
Launches are captured in a HIP graph (no host launch overhead in the timing).
AVSR_GEMM_TILE=128|256|256x128|128x256 forces a tile configuration; AVSR_GEMM_NOGLDS=1 selects
the register-staged core."""
import sys, os
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
tag = os.environ.get("AVSR_GEMM_TILE", "auto") + ("/noglds" if os.environ.get("AVSR_GEMM_NOGLDS") == "1" else "")
shapes = [(6000, 1024, 1024), (6000, 3072, 1024), (6000, 4096, 1024), (6000, 1024, 4096), (6000, 5056, 1024)]
if len(sys.argv) > 1 and sys.argv[1] == "big":
    shapes.append((8192, 8192, 8192))
for (M, N, K) in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    dW = torch.zeros(N, K, device=dev)
    fl = 2 * M * N * K
    a = t(lambda: ops.linear_fwd(x, W))
    bias = torch.zeros(N, device=dev)
    h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ae = t(lambda: ops.linear_fwd(x, W, bias, act=1, preact=h, drop_p=0.1, seed=7))
    b = t(lambda: ops.linear_dgrad(dy, W))
    c = t(lambda: ops.linear_wgrad(dy, x, dW))
    r = t(lambda: x @ W.t())
    print(f"[{tag}] M{M} N{N} K{K}: fwd {fl/a/1e9:.0f} TF/s ({a*1e3:.1f}us) fwd+gelu/drop/preact {fl/ae/1e9:.0f}  dgrad {fl/b/1e9:.0f}  "
          f"wgrad(splitk=1) {fl/c/1e9:.0f}  torch {fl/r/1e9:.0f}", flush=True)
