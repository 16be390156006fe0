"""Row-split GEMM dispatch experiment: the 256x256 core on the rows that fill whole rounds of
256 CUs, the 128x128 core on the remaining rows, vs the 128x128 core alone (FFN1 / QKV forward
with the engine epilogue, FFN2 data-grad). HIP-graph timed. python tools/msplit_bench.py"""
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


def fwd(x, W, b, h, y, tile, act=True):
    os.environ["AVSR_GEMM_TILE"] = tile
    if act:
        ops.linear_fwd(x, W, b, act=L.ACT_GELU, preact=h, drop_p=0.1, seed=3, out=y)
    else:
        ops.linear_fwd(x, W, b, out=y)


def dgrad(g, W, h, dh, tile):
    os.environ["AVSR_GEMM_TILE"] = tile
    ops.linear_dgrad(g, W, gate=h, act=L.ACT_GELU, drop_p=0.1, seed=3, out=dh)


def main():
    x, W1, Wq, W2 = r(M, D), r(F, D), r(3 * D, D), r(D, F)
    b1, bq = torch.randn(F, device=dev), torch.randn(3 * D, device=dev)
    h, y = r(M, F), r(M, F)
    g2, dh = r(M, D), r(M, F)
    q = r(M, 3 * D)
    for name, full, parts in [
        ("ffn1 fwd", lambda t: fwd(x, W1, b1, h, y, t),
         lambda mp: (fwd(x[:mp], W1, b1, h[:mp], y[:mp], "pp"), fwd(x[mp:], W1, b1, h[mp:], y[mp:], "128"))),
        ("qkv fwd", lambda t: fwd(x, Wq, bq, None, q, t, act=False),
         lambda mp: (fwd(x[:mp], Wq, bq, None, q[:mp], "pp", act=False), fwd(x[mp:], Wq, bq, None, q[mp:], "128", act=False))),
        ("ffn2 dgrad", lambda t: dgrad(g2, W2, h, dh, t),
         lambda mp: (dgrad(g2[:mp], W2, h[:mp], dh[:mp], "pp"), dgrad(g2[mp:], W2, h[mp:], dh[mp:], "128"))),
    ]:
        N = y.shape[1] if name != "qkv fwd" else 3 * D
        ct = N // 256
        mp = (256 // ct) * 256
        line = f"{name:10s} 128: {timed(lambda: full('128'), n=10):6.1f} us  pp: {timed(lambda: full('pp'), n=10):6.1f} us"
        for m2 in sorted({mp, 4096, 5120}):
            if m2 < M:
                line += f"  split@{m2}: {timed(lambda: parts(m2), n=10):6.1f} us"
        print(line, flush=True)
    os.environ.pop("AVSR_GEMM_TILE", None)


if __name__ == "__main__":
    main()
