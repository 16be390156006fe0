"""Fused AdamW (+ bf16 shadow) over 325 M fp32 parameters (the C2 trainable arena size): time and
effective HBM rate (30 B per element) per kernel variant (AVSR_ADAMW_VAR / AVSR_ADAMW_GRID).
usage: python tools/adamw_bench.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from avsr_amd import ops  # noqa: E402

dev = torch.device("cuda")
n = 325_000_000
P = torch.randn(n, device=dev) * 0.02
G = torch.randn(n, device=dev) * 1e-3
M = torch.zeros(n, device=dev); V = torch.zeros(n, device=dev)
S = torch.empty(n, device=dev, dtype=torch.bfloat16)
ss = torch.ones(1, device=dev)
ref = None
for var, grid in (("0", "4096"), ("1", "4096"), ("2", "4096"), ("3", "4096"), ("4", "4096"), ("3", "2048"), ("3", "8192"), ("0", "4096")):
    os.environ["AVSR_ADAMW_VAR"] = var; os.environ["AVSR_ADAMW_GRID"] = grid
    P1, M1, V1 = P.clone(), M.clone(), V.clone()
    fn = lambda: ops.adamw(P1, G, M1, V1, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.005, step=3,
                           shadow=S, sumsq_buf=ss, max_norm=1.0)
    fn(); torch.cuda.synchronize()
    if ref is None:
        ref = (P1.clone(), M1.clone(), V1.clone())
    else:
        assert torch.equal(P1, ref[0]) and torch.equal(M1, ref[1]) and torch.equal(V1, ref[2]), var
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        fn()
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    print(f"var {var} grid {grid}: {ms * 1e3:8.1f} us  {30 * n / ms / 1e9:6.2f} TB/s", flush=True)
    del P1, M1, V1
