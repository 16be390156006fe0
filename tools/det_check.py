"""Determinism bisection at C2 (bf16, dropouts 0): the same train step twice must give bit-identical
video-frontend features, losses and gradients. Prints which stage first differs, for the stem
conv straight from the video on and off. usage: python tools/det_check.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import engine as E  # noqa: E402
from avsr_amd import ops  # noqa: E402
from avsr_amd.avhubert_avsr_model import AVHubertAVSR  # noqa: E402
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig  # noqa: E402
from bench import synthetic_batch  # noqa: E402
from oracle.weights import NO_DROPOUT  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
m = AVHubertAVSR(AVHubertAVSRConfig(odim=5049, **NO_DROPOUT)).train()
m.setup_engine(dev, torch.bfloat16)
eng = m.avsr.engine()
v, a, lens, lab = synthetic_batch(16, 375, 40)
v, a = v.to(dev), a.to(dev)
res = {}
for direct in (True, False):
    E._STEM_DIRECT = direct
    outs = []
    for rep in range(2):
        feat, _ = eng.video_fwd(v, True, False)
        B, T = 16, 375
        h0 = None
        wk = torch.empty(64, ops.STEM_K, device=dev, dtype=torch.bfloat16)
        R = "encoder.feature_extractor_video.resnet."
        ops.stem_wpack2(eng.arena.master(R + "frontend3D.0.weight"), wk)
        h0 = torch.empty(B * T * 1936, 64, device=dev, dtype=torch.bfloat16)
        part = torch.empty(64, ops.stem_conv_tiles(B, T), 3, device=dev)
        ops.stem_conv_fwd(v.contiguous(), wk, h0, part)
        eng.arena.zero_grad()
        out4, ctx = eng.forward(v, a, lens, lab, train=True, need_grad=True, seed=5)
        eng.backward(ctx, torch.full((1,), 0.1, device=dev), torch.full((1,), 0.9, device=dev))
        torch.cuda.synchronize()
        outs.append((feat.clone(), h0.clone(), part.clone(), out4.clone(), eng.arena.grad.clone()))
        del ctx
    names = ["feat", "stem_h0", "stem_stats", "loss", "grad"]
    res[f"direct={direct}"] = {n: bool(torch.equal(x, y)) for n, x, y in zip(names, outs[0], outs[1])}
print(json.dumps(res))
