"""Encoder self-attention fwd / bwd timing at C2 (B=16, H=16, L=375, dh=64), without and with
probability dropout, the dropout hashed per element or read from the stored keep mask
(avsr_attn_dropmask, also timed). usage: python tools/attn_bench.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops

dev = torch.device("cuda")
B, H, L, D = 16, 16, 375, 64
qkv = torch.randn(B * L, 3 * H * D, device=dev, dtype=torch.bfloat16)
q, k, v = qkv[:, :1024], qkv[:, 1024:2048], qkv[:, 2048:]
o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * H * L, device=dev)
do = torch.randn_like(o)
dq = torch.empty_like(o); dk = torch.empty_like(o); dv = torch.empty_like(o)
delta = torch.empty(B * H * L, device=dev)
klen = torch.full((B,), L, device=dev, dtype=torch.int32)
mask = torch.empty(ops.attn_mask_words(B, H, L, L), device=dev, dtype=torch.int64)
fl = 4.0 * B * H * L * L * D


def tm(fn, n=50):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for p, stored in ((0.0, False), (0.1, False), (0.1, True)):
    m = ops.attn_dropmask(mask, B=B, H=H, Lq=L, Lk=L, drop_p=p, seed=3) if stored else None
    f = tm(lambda: ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, klen=klen, drop_p=p, seed=3, mask=m))
    g = tm(lambda: ops.attn_bwd(do, q, k, v, o, lse, None, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, klen=klen,
                                drop_p=p, seed=3, dq=dq, mask=m))
    print(f"drop {p} {'stored mask' if stored else 'hashed'}: fwd {f * 1e3:.1f} us ({fl / f / 1e9:.0f} TF/s)  "
          f"bwd(dkdv+dq) {g * 1e3:.1f} us ({2.5 * fl / g / 1e9:.0f} TF/s)", flush=True)
t = tm(lambda: ops.attn_dropmask(mask, B=B, H=H, Lq=L, Lk=L, drop_p=0.1, seed=3))
print(f"dropmask ({mask.numel() * 8 / 1e6:.1f} MB): {t * 1e3:.1f} us", flush=True)
