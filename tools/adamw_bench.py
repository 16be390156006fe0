"""Fused clip + AdamW timing: the bench model's own arena (FusedAdamW.step: sumsq + the two
segment launches) and fresh tensors of the same length, against a float4 copy of one fp32
array. usage: python tools/adamw_bench.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from avsr_amd import ops
from avsr_amd.avhubert_avsr_model import AVHubertAVSR
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from avsr_amd.optim import FusedAdamW

dev = torch.device("cuda")


def tm(fn, n=10):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


model = AVHubertAVSR(AVHubertAVSRConfig(odim=5049)).train()
model.setup_engine(dev, torch.bfloat16)
arena = model.avsr.engine().arena
opt = FusedAdamW(arena, lr=1e-4, weight_decay=0.005, max_grad_norm=1.0)
d0, _ = arena.segments["decay"]
_, n1 = arena.segments["no_decay"]
n = n1 - d0
arena.grad.normal_()
print(f"trainable elements {n / 1e6:.1f} M, arena {arena.data.numel() / 1e6:.1f} M")
us = tm(lambda: opt.step())
print(f"FusedAdamW.step (sumsq + adamw, model arena): {us:8.1f} us  {30 * n / us / 1e6:.2f} TB/s at 30 B/elem")
us = tm(lambda: opt.grad_sumsq())
print(f"grad_sumsq alone:                              {us:8.1f} us  {4 * n / us / 1e6:.2f} TB/s")
us = tm(lambda: opt.step(sumsq_ready=True))
print(f"adamw launches alone (model arena):            {us:8.1f} us  {30 * n / us / 1e6:.2f} TB/s")
del model, opt
p, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
v.abs_()
sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
ss = torch.ones(1, device=dev)
us = tm(lambda: ops.adamw(p, g, m, v, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.005, step=3,
                          shadow=sh, sumsq_buf=ss, max_norm=1.0))
print(f"adamw fresh tensors:                           {us:8.1f} us  {30 * n / us / 1e6:.2f} TB/s")
us = tm(lambda: m.copy_(p))
print(f"fp32 copy (torch):                             {us:8.1f} us  {8 * n / us / 1e6:.2f} TB/s")
# where does the arena's extra time come from: one launch over the arena's own buffers, and fresh
# tensors with each arena buffer swapped in
model = AVHubertAVSR(AVHubertAVSRConfig(odim=5049)).train()
model.setup_engine(dev, torch.bfloat16)
ar = model.avsr.engine().arena
ar.init_optimizer()
ar.grad.normal_()
arr = {"p": ar.data[d0:n1], "g": ar.grad[d0:n1], "m": ar.exp_avg[d0:n1], "v": ar.exp_avg_sq[d0:n1], "sh": ar.shadow[d0:n1]}
fresh = {"p": p, "g": g, "m": m, "v": v, "sh": sh}


def run(src):
    t = {k: (arr if k in src else fresh)[k] for k in fresh}
    return tm(lambda: ops.adamw(t["p"], t["g"], t["m"], t["v"], lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8,
                                weight_decay=0.005, step=3, shadow=t["sh"], sumsq_buf=ss, max_norm=1.0))


for src in ((), ("p", "g", "m", "v", "sh"), ("p",), ("g",), ("m",), ("v",), ("sh",)):
    us = run(src)
    print(f"arena buffers {','.join(src) or '-':14s}: {us:8.1f} us  {30 * n / us / 1e6:.2f} TB/s")
