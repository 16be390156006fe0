"""Stem backward apply (argmax-routed, 2x2 blocks) in isolation at C2 geometry (6000 frames,
44 x 44 x 64 bf16): time and effective HBM rate. usage: python tools/stem_apply_kbench.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from avsr_amd import ops  # noqa: E402

dev = torch.device("cuda")
n, H, W, C = 6000, 44, 44, 64
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(n * H * W, C, device=dev, generator=g).to(torch.bfloat16)
st = ops.BnState(C, dev)
st.mean.normal_(0, 0.1, generator=g); st.invstd.uniform_(0.5, 2, generator=g); st.scale.uniform_(0.5, 2, generator=g)
dz = torch.randn(n * 22 * 22, C, device=dev, generator=g).to(torch.bfloat16)
am = torch.randint(0, 9, (n * 22 * 22, C), device=dev, generator=g, dtype=torch.uint8)
sums = torch.randn(C, 3, device=dev, generator=g)
dh = torch.empty_like(h)
ref = None
for u in ("1", "1"):
    ops.stem_pool_bwd_apply(dz, am, h, n, H, W, st, sums, dh)
    torch.cuda.synchronize()
    if ref is None:
        ref = dh.clone()
    assert torch.equal(ref, dh), u
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        ops.stem_pool_bwd_apply(dz, am, h, n, H, W, st, sums, dh)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    byt = 2 * h.numel() * 2 + dz.numel() * 2 + am.numel()
    print(f"U={u}: {ms * 1e3:7.1f} us  {byt / ms / 1e9:5.2f} TB/s (h read + dh write + pooled dz / argmax once)", flush=True)
