"""LayerNorm backward (6000 x 1024 bf16, residual grad + dgamma/dbeta) alone, HIP-graph timed,
under each AVSR_LN_BWD launch shape. usage: python tools/ln_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402
from tools.gemm_table import timed  # noqa: E402

dev = torch.device("cuda")
for rows, N in ((6000, 1024), (656, 512), (6000, 2048)):
    x = torch.randn(rows, N, device=dev).to(torch.bfloat16)
    g = 1 + 0.1 * torch.randn(N, device=dev)
    b = 0.1 * torch.randn(N, device=dev)
    y, mean, rstd = ops.layernorm_fwd(x, g, b, 1e-5)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    dg = torch.zeros(N, device=dev)
    db = torch.zeros(N, device=dev)
    line = f"rows {rows} N {N}:"
    ref = None
    for shape in ("4,1", "2,1", "2,2", "4,2", "8,1", "8,2", "16,1", "16,2"):
        os.environ["AVSR_LN_BWD"] = shape
        dg.zero_(); db.zero_()
        dx = ops.layernorm_bwd(dy, x, g, mean, rstd, dres=dres, dgamma=dg, dbeta=db)
        torch.cuda.synchronize()
        if ref is None:
            ref = (dx.float().clone(), dg.clone(), db.clone())
        else:
            e = max((dx.float() - ref[0]).abs().max().item(), (dg - ref[1]).abs().max().item() / ref[1].abs().max().item())
            assert e < 1e-2, (shape, e)
        us = timed(lambda: ops.layernorm_bwd(dy, x, g, mean, rstd, dres=dres, dgamma=dg, dbeta=db))
        line += f"  {shape}: {us:6.1f}us"
    os.environ.pop("AVSR_LN_BWD", None)
    print(line, f" ({4 * rows * N * 2 / 1e3:.0f} KB moved)", flush=True)
