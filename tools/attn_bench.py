"""Encoder self-attention fwd / bwd timing at C2 (B=16, H=16, L=375, dh=64), with and without
probability dropout; with `db` also the fused q/k/v bias-gradient variant of the backward against
the separate column-sum pass. usage: python tools/attn_bench.py [db]"""
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
fl = 4.0 * B * H * L * L * D


def tm(fn, n=20):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for p in (0.0, 0.1):
    f = tm(lambda: ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, klen=klen, drop_p=p, seed=3))
    g = tm(lambda: ops.attn_bwd(do, q, k, v, o, lse, None, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, klen=klen,
                                drop_p=p, seed=3, dq=dq))
    print(f"drop {p}: fwd {f * 1e3:.1f} us ({fl / f / 1e9:.0f} TF/s)  bwd(prep+dkdv+dq) {g * 1e3:.1f} us "
          f"({2.5 * fl / g / 1e9:.0f} TF/s)", flush=True)
db = torch.zeros(3 * H * D, device=dev)
for p in ((0.0, 0.1) if "db" in sys.argv[1:] else ()):   # `python tools/attn_bench.py db`
    g0 = tm(lambda: ops.attn_bwd(do, q, k, v, o, lse, None, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, klen=klen,
                                 drop_p=p, seed=3, dq=dq))
    g1 = tm(lambda: ops.attn_bwd(do, q, k, v, o, lse, None, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, klen=klen,
                                 drop_p=p, seed=3, dq=dq, db=db))
    g2 = tm(lambda: ops.ew_bwd(qkv, db=db))
    print(f"drop {p}: bwd {g0 * 1e3:.1f} us, with fused q/k/v bias grads {g1 * 1e3:.1f} us; "
          f"separate column-sum pass over dqkv {g2 * 1e3:.1f} us", flush=True)
