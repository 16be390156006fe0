"""Library ceiling for the encoder GEMM shapes: torch.mm (hipBLASLt / rocBLAS) on the 12 GEMMs of
one encoder layer at C2 (M = 6000, d = 1024, F = 4096), bf16 in / bf16 out, and the weight-grads
also with fp32 output (out_dtype). Same HIP-graph timing as tools/gemm_table.py. A measurement
aid only (nothing on the product path calls a library GEMM).

  python tools/blas_ref.py [out.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.gemm_table import timed, wgrad  # noqa: E402
from avsr_amd import ops  # noqa: E402

PEAK = 2500.0
dev = torch.device("cuda")
M, D, F = 6000, 1024, 4096
LAYERS = {"qkv": (3 * D, D), "out": (D, D), "ffn1": (F, D), "ffn2": (D, F)}


def main():
    g = torch.Generator(device="cpu").manual_seed(0)
    rows = []
    for name, (N, K) in LAYERS.items():
        x = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
        W = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        dy = (torch.randn(M, N, generator=g) * 0.5).to(dev, torch.bfloat16)
        dW = torch.zeros(N, K, device=dev)
        fl = 2.0 * M * N * K
        cases = [("fwd", "torch", lambda: torch.mm(x, W.t())),
                 ("fwd", "avsr", lambda: ops.linear_fwd(x, W)),
                 ("dgrad", "torch", lambda: torch.mm(dy, W)),
                 ("dgrad", "avsr", lambda: ops.linear_dgrad(dy, W)),
                 ("wgrad", "torch", lambda: torch.mm(dy.t(), x)),
                 ("wgrad", "torch_f32out", lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)),
                 ("wgrad", "avsr", lambda: wgrad(dy, x, dW))]
        for op, who, fn in cases:
            try:
                us = timed(fn)
            except Exception as e:   # noqa: BLE001
                print(name, op, who, "failed:", e, flush=True)
                continue
            tf = fl / us / 1e6
            r = {"gemm": f"{name} {op}", "impl": who, "us": round(us, 1), "tflops": round(tf, 1),
                 "frac": round(tf / PEAK, 4)}
            rows.append(r)
            print(json.dumps(r), flush=True)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
