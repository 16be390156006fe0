"""Fused attention fwd/bwd vs a torch fp64 reference (encoder key-padding mask, decoder
causal self-attention, decoder source attention, probability dropout)."""
import math

import pytest
import torch

from avsr_amd import ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _ref(q, k, v, B, H, Lq, Lk, klen, causal, scale, mask_mult=None):
    qh = q.view(B, Lq, H, 64).transpose(1, 2)
    kh = k.view(B, Lk, H, 64).transpose(1, 2)
    vh = v.view(B, Lk, H, 64).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale
    m = torch.ones(B, 1, Lq, Lk, dtype=torch.bool)
    if klen is not None:
        m &= (torch.arange(Lk)[None, :] < torch.tensor(klen)[:, None])[:, None, None, :]
    if causal:
        m &= torch.tril(torch.ones(Lq, Lk, dtype=torch.bool))[None, None]
    s = s.masked_fill(~m, float("-inf"))
    p = torch.softmax(s, -1)
    if mask_mult is not None:
        p = p * mask_mult
    return (p @ vh).transpose(1, 2).reshape(B * Lq, H * 64)


CASES = [
    # B, H, Lq, Lk, klen, causal
    (3, 4, 75, 75, [75, 60, 33], False),
    (2, 2, 41, 41, None, True),
    (3, 2, 41, 150, [150, 77, 129], False),
    (2, 16, 375, 375, [375, 301], False),
    (1, 2, 520, 520, [517], False),          # Lk > 384: streamed kernels only
    (2, 3, 200, 130, [130, 65], False),      # cross-shaped, two q-blocks, the last one partial
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES)
def test_attention(dev, dtype, case):
    B, H, Lq, Lk, klen, causal = case
    D = H * 64
    g = torch.Generator().manual_seed(B * 1000 + Lq)
    qkv = torch.randn(B * Lq, 3 * D, generator=g)          # fused layout [q | k | v]
    kv = torch.randn(B * Lk, 2 * D, generator=g)
    q = qkv[:, :D]
    if Lq == Lk:
        k, v = qkv[:, D:2 * D], qkv[:, 2 * D:]
    else:
        k, v = kv[:, :D], kv[:, D:]
    scale = 1 / math.sqrt(64)
    qr, kr, vr = (t.double().clone().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, B, H, Lq, Lk, klen, causal, scale)
    dout = torch.randn(B * Lq, D, generator=g)
    ref.backward(dout.double())
    # device copies (q/k/v as column slices of one buffer where the layout is fused)
    if Lq == Lk:
        buf = qkv.to(dev, dtype)
        qd, kd, vd = buf[:, :D], buf[:, D:2 * D], buf[:, 2 * D:]
    else:
        qd = q.contiguous().to(dev, dtype)
        kvd = kv.to(dev, dtype)
        kd, vd = kvd[:, :D], kvd[:, D:]
    o = torch.empty(B * Lq, D, device=dev, dtype=dtype)
    lse = torch.empty(B, H, Lq, device=dev)
    kl = None if klen is None else torch.tensor(klen, dtype=torch.int32, device=dev)
    ops.attn_fwd(qd, kd, vd, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, klen=kl, causal=causal, scale=scale)
    tol = 3e-5 if dtype == torch.float32 else 2e-2
    assert _rel(o, ref) < tol
    dq = torch.zeros(B * Lq, D, device=dev)
    dk = torch.empty(B * Lk, D, device=dev, dtype=dtype)
    dv = torch.empty(B * Lk, D, device=dev, dtype=dtype)
    delta = torch.empty(B, H, Lq, device=dev)
    ops.attn_bwd(dout.to(dev, dtype), qd, kd, vd, o, lse, dq, dk, dv, delta, B=B, H=H, Lq=Lq, Lk=Lk,
                 klen=kl, causal=causal, scale=scale)
    gt = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(dq, qr.grad) < gt
    assert _rel(dk, kr.grad) < gt
    assert _rel(dv, vr.grad) < gt
    if dtype == torch.bfloat16:      # dQ written straight in bf16 (the engine's path)
        dqb = torch.empty(B * Lq, D, device=dev, dtype=dtype)
        ops.attn_bwd(dout.to(dev, dtype), qd, kd, vd, o, lse, None, dk, dv, delta, B=B, H=H, Lq=Lq, Lk=Lk,
                     klen=kl, causal=causal, scale=scale, dq=dqb)
        assert _rel(dqb, qr.grad) < gt


def test_attention_dropout(dev):
    """Recover the dropout mask through V = one-hot rows (Lk <= 64), then check fwd/bwd
    against the reference with that mask applied."""
    B, H, L, p, seed = 2, 2, 48, 0.1, 77
    D = H * 64
    g = torch.Generator().manual_seed(1)
    q = torch.randn(B * L, D, generator=g); k = torch.randn(B * L, D, generator=g)
    eye = torch.zeros(B * L, D)
    for b in range(B):
        for j in range(L):
            for h in range(H):
                eye[b * L + j, h * 64 + j] = 1.0
    qd, kd = q.to(dev), k.to(dev)
    o = torch.empty(B * L, D, device=dev)
    lse = torch.empty(B, H, L, device=dev)
    ops.attn_fwd(qd, kd, eye.to(dev), o, lse, B=B, H=H, Lq=L, Lk=L, scale=0.125, drop_p=p, seed=seed)
    pm = o.cpu().double().view(B, L, H, 64)[..., :L].permute(0, 2, 1, 3)       # P' (B, H, L, L)
    qh = q.double().view(B, L, H, 64).transpose(1, 2); kh = k.double().view(B, L, H, 64).transpose(1, 2)
    pr = torch.softmax(qh @ kh.transpose(-1, -2) * 0.125, -1)
    mult = (pm / pr).round(decimals=3)
    kept = (mult > 0.5)
    assert 0.85 < kept.double().mean().item() < 0.95
    assert torch.allclose(mult[kept], torch.full_like(mult[kept], 1 / (1 - p)), atol=1e-3)
    mask_mult = kept.double() / (1 - p)
    v = torch.randn(B * L, D, generator=g)
    qr, kr, vr = (t.double().clone().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, B, H, L, L, None, False, 0.125, mask_mult)
    dout = torch.randn(B * L, D, generator=g)
    ref.backward(dout.double())
    vd = v.to(dev)
    ops.attn_fwd(qd, kd, vd, o, lse, B=B, H=H, Lq=L, Lk=L, scale=0.125, drop_p=p, seed=seed)
    assert _rel(o, ref) < 3e-5
    dq = torch.zeros(B * L, D, device=dev)
    dk = torch.empty(B * L, D, device=dev); dv = torch.empty(B * L, D, device=dev)
    delta = torch.empty(B, H, L, device=dev)
    ops.attn_bwd(dout.to(dev), qd, kd, vd, o, lse, dq, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, scale=0.125,
                 drop_p=p, seed=seed)
    assert _rel(dq, qr.grad) < 1e-4
    assert _rel(dk, kr.grad) < 1e-4
    assert _rel(dv, vr.grad) < 1e-4


def test_attention_dropout_bf16(dev):
    """bf16 streaming kernels with probability dropout: the mask (same counter hash as the
    fp32 kernels) is recovered through one-hot V rows in fp32, then the bf16 fwd / bwd
    (dK, dV and both dQ outputs) are checked against the reference with that mask."""
    B, H, L, p, seed = 2, 2, 150, 0.1, 4242
    D = H * 64
    g = torch.Generator().manual_seed(2)
    q = torch.randn(B * L, D, generator=g); k = torch.randn(B * L, D, generator=g)
    qd, kd = q.to(dev), k.to(dev)
    lse = torch.empty(B, H, L, device=dev)
    mult = torch.empty(B, H, L, L, dtype=torch.float64)
    for j0 in range(0, L, 64):       # 64 one-hot key columns per pass
        eye = torch.zeros(B * L, D)
        for b in range(B):
            for j in range(j0, min(L, j0 + 64)):
                for h in range(H):
                    eye[b * L + j, h * 64 + j - j0] = 1.0
        o = torch.empty(B * L, D, device=dev)
        ops.attn_fwd(qd, kd, eye.to(dev), o, lse, B=B, H=H, Lq=L, Lk=L, scale=0.125, drop_p=p, seed=seed)
        n = min(L, j0 + 64) - j0
        mult[..., j0:j0 + n] = o.cpu().double().view(B, L, H, 64)[..., :n].permute(0, 2, 1, 3)
    qh = q.double().view(B, L, H, 64).transpose(1, 2); kh = k.double().view(B, L, H, 64).transpose(1, 2)
    pr = torch.softmax(qh @ kh.transpose(-1, -2) * 0.125, -1)
    kept = (mult / pr).round(decimals=3) > 0.5
    assert 0.85 < kept.double().mean().item() < 0.95
    mask_mult = kept.double() / (1 - p)
    v = torch.randn(B * L, D, generator=g)
    qr, kr, vr = (t.double().clone().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, B, H, L, L, None, False, 0.125, mask_mult)
    dout = torch.randn(B * L, D, generator=g)
    ref.backward(dout.double())
    bf = torch.bfloat16
    qb, kb, vb = q.to(dev, bf), k.to(dev, bf), v.to(dev, bf)
    o = torch.empty(B * L, D, device=dev, dtype=bf)
    ops.attn_fwd(qb, kb, vb, o, lse, B=B, H=H, Lq=L, Lk=L, scale=0.125, drop_p=p, seed=seed)
    assert _rel(o, ref) < 2e-2
    dq = torch.zeros(B * L, D, device=dev)
    dqb = torch.empty(B * L, D, device=dev, dtype=bf)
    dk = torch.empty(B * L, D, device=dev, dtype=bf); dv = torch.empty(B * L, D, device=dev, dtype=bf)
    delta = torch.empty(B, H, L, device=dev)
    db = dout.to(dev, bf)
    ops.attn_bwd(db, qb, kb, vb, o, lse, dq, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, scale=0.125, drop_p=p, seed=seed)
    assert _rel(dq, qr.grad) < 3e-2
    assert _rel(dk, kr.grad) < 3e-2
    assert _rel(dv, vr.grad) < 3e-2
    ops.attn_bwd(db, qb, kb, vb, o, lse, None, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, scale=0.125, drop_p=p,
                 seed=seed, dq=dqb)
    assert _rel(dqb, qr.grad) < 3e-2


@pytest.mark.parametrize("B,H,L,klen", [(2, 16, 375, [375, 301]), (3, 2, 200, [200, 129, 64])])
def test_attention_sq_matches_resident(dev, monkeypatch, B, H, L, klen, lib_opt):
    """The query-tiled forward (K/V streamed through the LDS-DMA ring, sq::attn_fwd_kernel)
    against the resident-K/V forward on the same bf16 inputs with dropout: the same dropout
    mask (zero pattern of P' through one-hot V rows is covered by test_attention_dropout_bf16;
    here every output row agrees to bf16 rounding of P) and the same log-sum-exp."""
    D = H * 64
    g = torch.Generator().manual_seed(L + H)
    bf = torch.bfloat16
    qkv = torch.randn(B * L, 3 * D, generator=g).to(dev, bf)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    kl = torch.tensor(klen, dtype=torch.int32, device=dev)

    def run():
        o = torch.empty(B * L, D, device=dev, dtype=bf)
        lse = torch.empty(B, H, L, device=dev)
        ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, klen=kl, scale=0.125, drop_p=0.1, seed=99)
        return o, lse
    o1, l1 = run()
    o1b, l1b = run()
    assert torch.equal(o1, o1b) and torch.equal(l1, l1b)
    lib_opt("attn_sq_fwd", 0)
    o0, l0 = run()
    assert _rel(o1, o0) < 1e-2
    assert (l1 - l0).abs().max().item() < 1e-4


@pytest.mark.parametrize("B,H,L,klen", [(2, 16, 375, [375, 301]), (3, 2, 200, [200, 129, 64])])
def test_attention_sq_backward_matches_resident(dev, monkeypatch, B, H, L, klen, lib_opt):
    """The query-tiled backward (dQ kernel computing delta, then dK / dV streaming Q, dO, lse,
    delta; the default only past 384 frames) against the resident backward on the same bf16
    inputs with dropout: dQ / dK / dV agree to bf16 rounding."""
    D = H * 64
    g = torch.Generator().manual_seed(L + 7)
    bf = torch.bfloat16
    qkv = torch.randn(B * L, 3 * D, generator=g).to(dev, bf)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    dout = torch.randn(B * L, D, generator=g).to(dev, bf)
    kl = torch.tensor(klen, dtype=torch.int32, device=dev)
    o = torch.empty(B * L, D, device=dev, dtype=bf)
    lse = torch.empty(B, H, L, device=dev)
    ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, klen=kl, scale=0.125, drop_p=0.1, seed=5)

    def bwd():
        dq = torch.empty(B * L, D, device=dev, dtype=bf)
        dk = torch.empty(B * L, D, device=dev, dtype=bf)
        dv = torch.empty(B * L, D, device=dev, dtype=bf)
        delta = torch.empty(B, H, L, device=dev)
        ops.attn_bwd(dout, q, k, v, o, lse, None, dk, dv, delta, B=B, H=H, Lq=L, Lk=L, klen=kl, scale=0.125,
                     drop_p=0.1, seed=5, dq=dq)
        return dq, dk, dv
    ref = bwd()
    lib_opt("attn_sq_bwd", 1)
    got = bwd()
    again = bwd()
    for a_, b_, c_ in zip(got, ref, again):
        assert torch.equal(a_, c_)
        assert _rel(a_, b_) < 2e-2
