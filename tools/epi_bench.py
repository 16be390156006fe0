"""Cost of the fused GEMM epilogues on the encoder's C2 shapes (M = 6000 tokens): each
engine GEMM timed with its real epilogue and with pieces removed (HIP-graph timed, random
operands). python tools/epi_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops, _lib as L  # noqa: E402
from tools.gemm_table import timed  # noqa: E402

dev = torch.device("cuda")
M, D, F = 6000, 1024, 4096


def r(*s):
    return (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)


def main():
    x, W1, W2, Wo = r(M, D), r(F, D), r(D, F), r(D, D)
    b1, b2 = torch.randn(F, device=dev), torch.randn(D, device=dev)
    h, act, res = r(M, F), r(M, F), r(M, D)
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    g2 = r(M, D)
    dh = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    G = L.ACT_GELU
    cases = [
        ("ffn1 fwd plain", 2 * M * F * D, lambda: ops.linear_fwd(x, W1, out=act)),
        ("ffn1 fwd +bias", 2 * M * F * D, lambda: ops.linear_fwd(x, W1, b1, out=act)),
        ("ffn1 fwd +bias+gelu", 2 * M * F * D, lambda: ops.linear_fwd(x, W1, b1, act=G, out=act)),
        ("ffn1 fwd +bias+gelu+preact", 2 * M * F * D, lambda: ops.linear_fwd(x, W1, b1, act=G, preact=h, out=act)),
        ("ffn1 fwd full (+dropout)", 2 * M * F * D,
         lambda: ops.linear_fwd(x, W1, b1, act=G, preact=h, drop_p=0.1, seed=7, out=act)),
        ("ffn2 fwd plain", 2 * M * F * D, lambda: ops.linear_fwd(act, W2, out=y)),
        ("ffn2 fwd full (+bias+res+dropout)", 2 * M * F * D,
         lambda: ops.linear_fwd(act, W2, b2, res=res, drop_p=0.1, seed=9, out=y)),
        ("ffn2 dgrad plain", 2 * M * F * D, lambda: ops.linear_dgrad(g2, W2, out=dh)),
        ("ffn2 dgrad +gelu'", 2 * M * F * D, lambda: ops.linear_dgrad(g2, W2, gate=h, act=G, out=dh)),
        ("ffn2 dgrad full (+dropout)", 2 * M * F * D,
         lambda: ops.linear_dgrad(g2, W2, gate=h, act=G, drop_p=0.1, seed=7, out=dh)),
        ("out fwd plain", 2 * M * D * D, lambda: ops.linear_fwd(x, Wo, out=y)),
        ("out fwd full (+bias+res+dropout)", 2 * M * D * D,
         lambda: ops.linear_fwd(x, Wo, b2, res=res, drop_p=0.1, seed=3, out=y)),
    ]
    for name, fl, fn in cases:
        us = timed(fn, n=10)
        print(f"{name:36s} {us:7.1f} us {fl / us / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
