"""The teacher-forced decoder's GEMMs at C2 (M = 16 x 41 = 656 target rows, d = 1024, dunits = 3072,
vocabulary 5056 padded) forward and data-grad, under the small-grid tile configurations (64x64
with 2 / 4 LDS stages) and the automatic choice, HIP-graph timed (tools/gemm_table.timed).
  python tools/dec_gemm_table.py [cfg,cfg,...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402
from tools.gemm_table import timed  # noqa: E402

dev = torch.device("cuda")
M = 656
SHAPES = {"self_qkv": (3072, 1024), "attn_out": (1024, 1024), "ffn1": (3072, 1024), "ffn2": (1024, 3072),
          "vocab": (5056, 1024)}   # (N, K) of y = x W^T


def main():
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["auto", "64", "64s4"]
    g = torch.Generator(device="cpu").manual_seed(0)
    tot = {c: 0.0 for c in cfgs}
    for name, (N, K) in SHAPES.items():
        x = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
        W = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        dy = (torch.randn(M, N, generator=g) * 0.5).to(dev, torch.bfloat16)
        for op, fn in (("fwd", lambda: ops.linear_fwd(x, W)), ("dgrad", lambda: ops.linear_dgrad(dy, W))):
            res = {}
            for c in cfgs:
                ops.L.set_option("gemm_tile", c)
                res[c] = timed(fn)
                tot[c] += res[c]
            ops.L.set_option("gemm_tile", "auto")
            print(f"{name:9s} {op:5s} N{N if op == 'fwd' else K:5d} K{K if op == 'fwd' else N:5d} " +
                  " ".join(f"{c}:{res[c]:6.1f}us" for c in cfgs), flush=True)
    print("sum " + " ".join(f"{c}:{tot[c]:7.1f}us" for c in cfgs))


if __name__ == "__main__":
    main()
