"""stem_conv_fwd run twice at C2: where do the BN partials differ? (diagnostic)"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
for (B, T) in ((2, 7), (16, 375)):
    video = torch.randn(B, 1, T, 88, 88, generator=g).to(dev)
    w = (torch.randn(64, 1, 5, 7, 7, generator=g) * 0.05).to(dev)
    wk = torch.empty(64, ops.STEM_K, device=dev, dtype=torch.bfloat16)
    ops.stem_wpack2(w, wk)
    tiles = ops.stem_conv_tiles(B, T)
    outs = []
    for rep in range(3):
        h = torch.empty(B * T * 1936, 64, device=dev, dtype=torch.bfloat16)
        st = torch.full((64, tiles, 3), float("nan"), device=dev)
        ops.stem_conv_fwd(video, wk, h, st)
        torch.cuda.synchronize()
        outs.append((h, st))
    d = (outs[0][1] - outs[1][1]).abs()
    bad = (d > 0) | torch.isnan(d)
    info = {"B": B, "T": T, "tiles": tiles, "h_equal": bool(torch.equal(outs[0][0], outs[1][0])),
            "stats_equal": bool(torch.equal(outs[0][1], outs[1][1])), "nan": int(torch.isnan(outs[0][1]).sum()),
            "bad": int(bad.sum()), "bad_tiles": sorted(set(bad.nonzero()[:, 1].tolist()))[:20],
            "bad_fields": sorted(set(bad.nonzero()[:, 2].tolist())), "maxdiff": float(d[~torch.isnan(d)].max()) if bad.any() else 0.0}
    print(json.dumps(info), flush=True)
