"""Fused attention fwd/bwd vs a torch fp64 reference (encoder key-padding mask, decoder
causal self-attention, decoder source attention, probability dropout)."""
import math

import numpy as np
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


# ---------------------------------------------------------------------------------------------
# Dropout mask identity (verdict r4 item 2): the kept / dropped pattern of every (query, key)
# pair is recovered exactly from each kernel that applies or regenerates it, and must be the
# same bit for bit. With Q.K = 0 for every pair (Q and K in orthogonal halves of the head
# dimension, or zero) the probabilities are uniform over the allowed keys, so
#  - forward: V rows one-hot over a chunk of 64 keys -> O[i, t] != 0 iff pair (i, c + t) kept;
#  - dK/dV kernel: dO rows one-hot over a chunk of 64 queries -> dV[j, t] != 0 iff (c + t, j) kept;
#  - dQ and dK: V = dO = ones gives dS_ij = P (64 m_ij / (1 - p) - delta_i); with Q one-hot over
#    a 32-query chunk in dims 0-31 and K one-hot over a 32-key chunk in dims 32-63,
#    dQ[i, 32 + t] = s dS_{i, c + t} and dK[j, t] = s dS_{c + t, j}; dS + P delta is 64P / (1 - p)
#    when kept and 0 when dropped (a gap of ~70P against bf16 rounding of < P).
# ---------------------------------------------------------------------------------------------
MASK_CASES = [
    # name, B, H, Lq, Lk, klen, causal: the C2 encoder self-attention, and the teacher-forced
    # decoder's causal self-attention and source attention at C2 (16 x 41 labels, 375 frames)
    ("enc_c2", 16, 16, 375, 375, [375, 301] * 8, False),
    ("dec_self", 16, 16, 41, 41, None, True),
    ("dec_src", 16, 16, 41, 375, [375, 301] * 8, False),
]


def _allowed(dev, B, H, Lq, Lk, klen, causal):
    m = torch.ones(B, 1, Lq, Lk, dtype=torch.bool, device=dev)
    if klen is not None:
        m &= (torch.arange(Lk, device=dev)[None, :] < torch.tensor(klen, device=dev)[:, None])[:, None, None, :]
    if causal:
        m &= torch.tril(torch.ones(Lq, Lk, dtype=torch.bool, device=dev))[None, None]
    return m.expand(B, H, Lq, Lk)


def _onehot_rows(rows, H, L, c, n, col0, dev, dt):
    """rows x (H*64) zeros with row c+t of every clip holding 1 at column h*64 + col0 + t (t < n)"""
    x = torch.zeros(rows // L, L, H, 64, device=dev, dtype=dt)
    if n > 0:
        x[:, c:c + n, :, col0:col0 + n] = torch.eye(n, device=dev, dtype=dt)[None, :, None, :]
    return x.view(rows, H * 64)


def _masks(dev, dt, B, H, Lq, Lk, klen, causal, p, seed, stored=False):
    """(forward mask, dV mask, dQ mask, dK mask) recovered from the kernels the current library
    options select, each restricted to the allowed pairs; stored: the kernels read the keep mask
    of avsr_attn_dropmask instead of hashing"""
    D = H * 64
    kl = None if klen is None else torch.tensor(klen, dtype=torch.int32, device=dev)
    kw = dict(B=B, H=H, Lq=Lq, Lk=Lk, klen=kl, causal=causal, scale=0.125, drop_p=p, seed=seed)
    if stored:
        kw["mask"] = ops.attn_dropmask(torch.empty(ops.attn_mask_words(B, H, Lq, Lk), dtype=torch.int64, device=dev),
                                       B=B, H=H, Lq=Lq, Lk=Lk, drop_p=p, seed=seed)
    allowed = _allowed(dev, B, H, Lq, Lk, klen, causal)
    lse = torch.empty(B, H, Lq, device=dev)
    zq, zk = torch.zeros(B * Lq, D, device=dev, dtype=dt), torch.zeros(B * Lk, D, device=dev, dtype=dt)

    def bwd(dout, q, k, v, o):
        dk = torch.empty(B * Lk, D, device=dev, dtype=dt)
        dv = torch.empty(B * Lk, D, device=dev, dtype=dt)
        delta = torch.empty(B, H, Lq, device=dev)
        if dt == torch.bfloat16:
            dq = torch.empty(B * Lq, D, device=dev, dtype=dt)
            ops.attn_bwd(dout, q, k, v, o, lse, None, dk, dv, delta, dq=dq, **kw)
        else:
            dq = torch.zeros(B * Lq, D, device=dev)
            ops.attn_bwd(dout, q, k, v, o, lse, dq, dk, dv, delta, **kw)
        return dq, dk, dv

    fwd = torch.zeros(B, H, Lq, Lk, dtype=torch.bool, device=dev)
    for c in range(0, Lk, 64):
        n = min(64, Lk - c)
        o = torch.empty(B * Lq, D, device=dev, dtype=dt)
        ops.attn_fwd(zq, zk, _onehot_rows(B * Lk, H, Lk, c, n, 0, dev, dt), o, lse, **kw)
        fwd[..., c:c + n] = o.view(B, Lq, H, 64)[..., :n].permute(0, 2, 1, 3) != 0
    o = torch.empty(B * Lq, D, device=dev, dtype=dt)
    ops.attn_fwd(zq, zk, zk, o, lse, **kw)
    dvm = torch.zeros_like(fwd)
    for c in range(0, Lq, 64):
        n = min(64, Lq - c)
        _, _, dv = bwd(_onehot_rows(B * Lq, H, Lq, c, n, 0, dev, dt), zq, zk, zk, o)
        dvm[:, :, c:c + n, :] = dv.view(B, Lk, H, 64)[..., :n].permute(0, 2, 3, 1) != 0
    nkeys = allowed.sum(-1, keepdim=True).double()                  # uniform P = 1 / nkeys
    ones_q, ones_k = torch.ones(B * Lq, D, device=dev, dtype=dt), torch.ones(B * Lk, D, device=dev, dtype=dt)
    dqm, dkm = torch.zeros_like(fwd), torch.zeros_like(fwd)
    for r in range(max(-(-Lq // 32), -(-Lk // 32))):
        cq, ck = 32 * r, 32 * r
        nq, nk = max(0, min(32, Lq - cq)), max(0, min(32, Lk - ck))
        q = _onehot_rows(B * Lq, H, Lq, cq, nq, 0, dev, dt)
        k = _onehot_rows(B * Lk, H, Lk, ck, nk, 32, dev, dt)
        ob = torch.empty(B * Lq, D, device=dev, dtype=dt)
        ops.attn_fwd(q, k, ones_k, ob, lse, **kw)
        dq, dk, _ = bwd(ones_q, q, k, ones_k, ob)
        delta = ob.double().view(B, Lq, H, 64).sum(-1).permute(0, 2, 1)[..., None]     # (B, H, Lq, 1)
        pd = delta / nkeys                                                             # P * delta
        thr = 32.0 / (1 - p) / nkeys                                                   # P * 32 / (1 - p)
        if nk:
            ds = dq.double().view(B, Lq, H, 64)[..., 32:32 + nk].permute(0, 2, 1, 3) / 0.125
            dqm[..., ck:ck + nk] = ds + pd > thr
        if nq:
            ds = dk.double().view(B, Lk, H, 64)[..., :nq].permute(0, 2, 3, 1) / 0.125    # (B, H, nq, Lk)
            dkm[:, :, cq:cq + nq, :] = ds + pd[:, :, cq:cq + nq] > thr[:, :, cq:cq + nq]
    return tuple(m & allowed for m in (fwd, dvm, dqm, dkm)), allowed


@pytest.mark.parametrize("case", MASK_CASES, ids=[c[0] for c in MASK_CASES])
def test_attention_dropout_mask_bitexact(dev, lib_opt, case):
    """every attention kernel of the training step applies or regenerates exactly the same
    dropout mask: the query-tiled and resident forwards, the resident backward (dK/dV and dQ
    kernels), each hashing or reading the stored keep mask of avsr_attn_dropmask (the encoder's
    production path; causal launches ignore it and hash), bf16 and the fp32 parity kernels —
    torch.equal on the recovered kept / dropped pattern of every allowed (query, key) pair"""
    name, B, H, Lq, Lk, klen, causal = case
    p, seed = 0.1, 0x5EED + Lq
    bf = torch.bfloat16
    runs = {}
    for fwd_sq in (1, 0):
        for stored in (True, False):
            lib_opt("attn_sq_fwd", fwd_sq)
            runs[f"bf16 fwd_sq={fwd_sq} stored={stored}"], allowed = _masks(dev, bf, B, H, Lq, Lk, klen, causal, p, seed,
                                                                            stored)
    lib_opt("attn_sq_fwd", 1)
    runs["fp32"], _ = _masks(dev, torch.float32, B, H, Lq, Lk, klen, causal, p, seed)
    ref = runs["bf16 fwd_sq=1 stored=True"][0]          # the production forward's mask
    frac = ref.sum().item() / allowed.sum().item()
    assert 0.88 < frac < 0.92, frac                  # keep probability 1 - p
    for label, masks in runs.items():
        for kind, m in zip(("fwd", "dV", "dQ", "dK"), masks):
            assert torch.equal(m, ref), (label, kind, (m ^ ref).sum().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES)
def test_attention_bias_grad(dev, dtype, case):
    """avsr_attn_params.db: += the column sums of the dQ | dK | dV the backward stores (the fused
    q/k/v bias gradients, one pass over the outputs after the backward kernels) — against fp64
    sums of the stored tensors, dropout on"""
    B, H, Lq, Lk, klen, causal = case
    D = H * 64
    g = torch.Generator().manual_seed(B * 7 + Lk)
    q = torch.randn(B * Lq, D, generator=g).to(dev, dtype)
    kv = torch.randn(B * Lk, 2 * D, generator=g).to(dev, dtype)
    k, v = kv[:, :D], kv[:, D:]
    o = torch.empty(B * Lq, D, device=dev, dtype=dtype)
    lse = torch.empty(B, H, Lq, device=dev)
    kl = None if klen is None else torch.tensor(klen, dtype=torch.int32, device=dev)
    kw = dict(B=B, H=H, Lq=Lq, Lk=Lk, klen=kl, causal=causal, scale=0.125, drop_p=0.1, seed=99)
    ops.attn_fwd(q, k, v, o, lse, **kw)
    dout = torch.randn(B * Lq, D, generator=g).to(dev, dtype)
    dk = torch.empty(B * Lk, D, device=dev, dtype=dtype)
    dv = torch.empty(B * Lk, D, device=dev, dtype=dtype)
    delta = torch.empty(B, H, Lq, device=dev)
    modes = ["f32"] + (["bf16"] if dtype == torch.bfloat16 else [])
    for mode in modes:
        db0 = torch.randn(3 * D, generator=g).to(dev)
        db = db0.clone()
        if mode == "bf16":
            dq = torch.empty(B * Lq, D, device=dev, dtype=dtype)
            ops.attn_bwd(dout, q, k, v, o, lse, None, dk, dv, delta, dq=dq, db=db, **kw)
        else:
            dq = torch.zeros(B * Lq, D, device=dev)
            ops.attn_bwd(dout, q, k, v, o, lse, dq, dk, dv, delta, db=db, **kw)
        want = torch.cat([t.double().sum(0) for t in (dq, dk, dv)]).cpu()
        mag = torch.cat([t.double().abs().sum(0) for t in (dq, dk, dv)]).cpu()
        got = (db.double() - db0.double()).cpu()
        assert ((got - want).abs() <= 2e-6 * mag + 1e-5).all(), (mode, (got - want).abs().max().item())


# ---------------------------------------------------------------------------------------------
# Stored dropout keep masks (avsr_attn_dropmask): the layout of include/avsr_hip.h against a
# numpy restatement of the attention dropout's counter hash (AttnDrop, attention.hip: pair index
# g = ((b*H + h) * Lq + q) * ceil(Lk / 2) + k / 2, fmix32(g * 0x9E3779B1 ^ pre), 16-bit half by
# key parity, kept iff >= round(p * 65536)); and kernel outputs with the stored mask == hashed.
# ---------------------------------------------------------------------------------------------
def _fmix32(h):
    h = h ^ (h >> np.uint64(16)); h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h = h ^ (h >> np.uint64(13)); h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    return h ^ (h >> np.uint64(16))


def _keep_ref(B, H, Lq, Lk, p, seed):
    """[B*H, Lq, Lk] bool keep decisions of the attention dropout (32-bit index form)"""
    seed = np.uint64(seed)
    lo, hi = seed & np.uint64(0xFFFFFFFF), seed >> np.uint64(32)
    pre = lo ^ _fmix32(np.uint64(0) ^ hi ^ np.uint64(0x68E31DA4))
    thr = int(np.float32(p) * np.float32(65536.0) + np.float32(0.5))
    npair = (Lk + 1) // 2
    bh = np.arange(B * H, dtype=np.uint64)[:, None, None]
    q = np.arange(Lq, dtype=np.uint64)[None, :, None]
    k = np.arange(Lk, dtype=np.uint64)[None, None, :]
    g = ((bh * np.uint64(Lq) + q) * np.uint64(npair) + (k >> np.uint64(1))) & np.uint64(0xFFFFFFFF)
    h = _fmix32(((g * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)) ^ pre)
    u = np.where((k & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    return u >= thr


def _unpack_mask(words, B, H, Lq, Lk):
    """the lane-mask layout of AVSR_ATTN_MASK_WORDS back to [B*H, Lq, Lk] bools"""
    NQB, NKB = -(-Lq // 32), 2 * (-(-Lk // 64))
    w = words.view(np.uint64)
    bits = ((w[:, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)   # [W, 64]
    r = np.arange(16)[:, None]
    l = np.arange(64)[None, :]
    qi = np.broadcast_to(l & 31, (16, 64))
    ki = np.broadcast_to((r & 3) + 8 * (r >> 2) + 4 * (l >> 5), (16, 64))
    t = bits.reshape(B * H, NQB, NKB, 16, 64)
    full = np.zeros((B * H, NQB * 32, NKB * 32), dtype=bool)
    for qb in range(NQB):
        for kb in range(NKB):
            full[:, 32 * qb + qi, 32 * kb + ki] = t[:, qb, kb]
    return full[:, :Lq, :Lk]


@pytest.mark.parametrize("B,H,Lq,Lk,p,seed", [(2, 3, 75, 70, 0.1, 0x1234ABCD5678), (1, 2, 41, 375, 0.3, 7),
                                             (2, 1, 130, 200, 0.05, 2 ** 63 + 11)])
def test_attention_dropmask_layout(dev, B, H, Lq, Lk, p, seed):
    """avsr_attn_dropmask writes the documented lane-mask layout of exactly the hash's keep bits
    (bits past Lq / Lk zero)"""
    n = ops.attn_mask_words(B, H, Lq, Lk)
    m = torch.full((n,), -1, dtype=torch.int64, device=dev)
    ops.attn_dropmask(m, B=B, H=H, Lq=Lq, Lk=Lk, drop_p=p, seed=seed)
    words = m.cpu().numpy()
    want = _keep_ref(B, H, Lq, Lk, p, seed)
    assert 0.9 * (1 - p) < want.mean() < 1.1 * (1 - p)
    got = _unpack_mask(words, B, H, Lq, Lk)
    assert np.array_equal(got, want), (got ^ want).sum()
    assert np.unpackbits(words.view(np.uint8)).sum() == want.sum()            # nothing set past Lq / Lk


@pytest.mark.parametrize("B,H,L,klen", [(16, 16, 375, [375, 301] * 8), (3, 2, 200, [200, 129, 64])])
def test_attention_stored_mask_outputs_identical(dev, B, H, L, klen):
    """the encoder's production path (bf16, keep mask from avsr_attn_dropmask) returns exactly the
    forward output and the dQ / dK / dV of the hashing kernels: torch.equal"""
    D = H * 64
    g = torch.Generator().manual_seed(L + 3)
    bf = torch.bfloat16
    qkv = torch.randn(B * L, 3 * D, generator=g).to(dev, bf)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    dout = torch.randn(B * L, D, generator=g).to(dev, bf)
    kl = torch.tensor(klen, dtype=torch.int32, device=dev)
    kw = dict(B=B, H=H, Lq=L, Lk=L, klen=kl, scale=0.125, drop_p=0.1, seed=31337)
    mask = ops.attn_dropmask(torch.empty(ops.attn_mask_words(B, H, L, L), dtype=torch.int64, device=dev),
                             B=B, H=H, Lq=L, Lk=L, drop_p=0.1, seed=31337)
    res = []
    for mk in (None, mask):
        o = torch.empty(B * L, D, device=dev, dtype=bf)
        lse = torch.empty(B, H, L, device=dev)
        ops.attn_fwd(q, k, v, o, lse, mask=mk, **kw)
        dq = torch.empty(B * L, D, device=dev, dtype=bf)
        dk = torch.empty(B * L, D, device=dev, dtype=bf)
        dv = torch.empty(B * L, D, device=dev, dtype=bf)
        delta = torch.empty(B, H, L, device=dev)
        ops.attn_bwd(dout, q, k, v, o, lse, None, dk, dv, delta, dq=dq, mask=mk, **kw)
        res.append((o, lse, dq, dk, dv))
    for name, a, b in zip(("o", "lse", "dq", "dk", "dv"), *res):
        assert torch.equal(a, b), (name, (a.float() - b.float()).abs().max().item())


