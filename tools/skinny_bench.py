"""Few-row (decoder-step) linears: per-launch time of the decoder's shapes at M rows, fp32,
split on / off, the matrix-core kernel vs the vector-ALU one (AVSR_SKINNY_VALU, read per launch).
python tools/skinny_bench.py [M]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda")
SHAPES = [("self qkv", 3072, 1024), ("out / cross q", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096),
          ("output", 5049, 1024)]


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


g = torch.Generator().manual_seed(0)
for name, N, K in SHAPES:
    x = torch.randn(M, K, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(M, N, generator=g).to(dev)
    out = torch.empty(M, N, device=dev)
    row = [f"{name:14s} N={N:5d} K={K:5d}"]
    for valu in ("0", "1"):
        os.environ["AVSR_SKINNY_VALU"] = valu
        for split in (True, False):
            us = timeit(lambda: ops.linear_fwd(x, W, b, res=r, out=out, skinny_split=split))
            gbs = N * K * 4 / us / 1e3
            row.append(f"{'valu' if valu == '1' else 'mma '} split={int(split)} {us:6.1f} us ({gbs:5.0f} GB/s)")
    os.environ["AVSR_SKINNY_VALU"] = "0"
    print("  ".join(row), flush=True)
