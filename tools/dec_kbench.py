"""decode-step kernels in isolation (warm caches): log-softmax + top-P at K = 1 / 7 rows 40 x 5049,
grouped cross-attention (G = 5, 375 keys, key split 1 / 2), self-attention (G = 1), CTC prefix.
python tools/dec_kbench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402

dev = torch.device("cuda")


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


g = torch.Generator().manual_seed(0)
R, V = 40, 5049
x = torch.randn(R, 5056, generator=g).to(dev)
lp = torch.empty(R, V, device=dev)
for K in (1, 7):
    ids = torch.empty(R, K, device=dev, dtype=torch.int32)
    print(f"log_softmax_topk K={K}: {timeit(lambda: ops.log_softmax_topk(x, V, lp, K, ids)):.1f} us", flush=True)
print(f"log_softmax_rows alone: {timeit(lambda: ops.log_softmax_rows(x, V, lp)):.1f} us", flush=True)
# grouped cross-attention over 8 utterances x 375 frames, beam 5, 16 heads
U, T, H, G = 8, 375, 16, 5
D = 64 * H
mem = torch.randn(U * T, 2 * D, generator=g).to(dev)
q = torch.randn(U * G, D, generator=g).to(dev)
o = torch.empty(U * G, D, device=dev)
uidx = torch.arange(U * G, dtype=torch.int32).div(G, rounding_mode="floor").to(dev, torch.int32)
klen = torch.full((U * G,), T, dtype=torch.int32, device=dev)
for ks in (1, 2, 4):
    us = timeit(lambda: ops.dec_attn(q, mem[:, :D], mem[:, D:], o, n=U * G, H=H, klen_max=T, k_bstride=T * mem.stride(0),
                                     v_bstride=T * mem.stride(0), kidx=uidx, klen=klen, group=G, ksplit=ks))
    print(f"cross dec_attn G=5 klen=375 ksplit={ks}: {us:.1f} us", flush=True)
us = timeit(lambda: ops.dec_attn(q, mem[:, :D], mem[:, D:], o, n=U * G, H=H, klen_max=T, k_bstride=T * mem.stride(0),
                                 v_bstride=T * mem.stride(0), kidx=uidx, klen=klen, group=1))
print(f"cross dec_attn G=1 klen=375: {us:.1f} us", flush=True)
for kl in (16, 188, 375):
    kk = torch.full((U * G,), kl, dtype=torch.int32, device=dev)
    us = timeit(lambda: ops.dec_attn(q, mem[:, :D], mem[:, D:], o, n=U * G, H=H, klen_max=T, k_bstride=T * mem.stride(0),
                                     v_bstride=T * mem.stride(0), kidx=uidx, klen=kk, group=G))
    print(f"cross dec_attn G=5 klen={kl}: {us:.1f} us", flush=True)
