"""Loss kernels (CTC alpha/beta + grad, label smoothing + accuracy) and the elementwise /
packing / optimizer kernels vs torch fp64 references."""
import math

import pytest
import torch
import torch.nn.functional as F

from avsr_amd import ops, _lib as L

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("T,lens,in_len", [(375, (40, 33), (375, 300)), (240, (150, 7), (240, 240))])
def test_ctc_multi_chunk(dev, T, lens, in_len):
    """C2-length inputs (several LDS emission chunks per recursion; S = 301 -> 20-step chunks)
    against torch's CTC in fp64: nll and the logits gradient."""
    B, V, Vp = 2, 5049, 5056
    g = torch.Generator().manual_seed(T)
    x = torch.randn(B * T, Vp, generator=g) * 2
    x[:, V:] = 0
    labels = [torch.randint(1, V - 1, (n,), generator=g).tolist() for n in lens]
    labels[0][3] = labels[0][4]                       # a repeat (no skip transition)
    Lmax = max(lens)
    lab = torch.full((B, Lmax), -1, dtype=torch.int32)
    for b, l in enumerate(labels):
        lab[b, :len(l)] = torch.tensor(l)
    xd = x.to(dev)
    lse = torch.empty(B * T, device=dev)
    ops.row_lse(xd, V, lse)
    S = 2 * Lmax + 1
    alpha = torch.empty(B, T, S, device=dev); gamma = torch.empty(B, T, S, device=dev)
    nll = torch.empty(B, device=dev)
    p = ops.ctc_params(xd, B, T, V, lab.to(dev), torch.tensor(list(lens), dtype=torch.int32, device=dev),
                       torch.tensor(list(in_len), dtype=torch.int32, device=dev), lse, alpha, gamma, nll)
    ops.ctc_fwd(p)
    xr = x.double()[:, :V].view(B, T, V).transpose(0, 1).contiguous().requires_grad_()
    tgt = torch.cat([torch.tensor(l) for l in labels])
    ref = F.ctc_loss(xr.log_softmax(-1), tgt, torch.tensor(list(in_len)), torch.tensor(list(lens)), blank=0,
                     reduction="none", zero_infinity=True)
    assert _rel(nll, ref) < 1e-5
    ref.sum().backward()
    gref = xr.grad.transpose(0, 1).reshape(B * T, V)
    dx = torch.empty(B * T, Vp, device=dev)
    ops.ctc_bwd(p, torch.tensor([1.0], device=dev), 1.0, dx)
    # fp32 log-space recursions over T steps: held to torch's own fp32 CTC error (as test_ctc)
    x32 = x.float()[:, :V].view(B, T, V).transpose(0, 1).contiguous().requires_grad_()
    F.ctc_loss(x32.log_softmax(-1), tgt, torch.tensor(list(in_len)), torch.tensor(list(lens)), blank=0,
               reduction="none", zero_infinity=True).sum().backward()
    e32 = _rel(x32.grad.transpose(0, 1).reshape(B * T, V), gref)
    err = _rel(dx[:, :V], gref)
    assert err < max(3 * e32, 1e-4), (err, e32)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ctc(dev, dtype):
    B, T, V, Vp = 4, 50, 5049, 5056
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B * T, Vp, generator=g) * 3
    x[:, V:] = 0
    labels = [[5, 5, 17, 301, 4000, 17], [77, 5047, 1, 2], [9] * 30, [3, 4]]   # repeats; [9]*30 infeasible at T=20
    in_len = [50, 41, 20, 7]
    Lmax = max(len(l) for l in labels)
    lab = torch.full((B, Lmax), -1, dtype=torch.int32)
    for b, l in enumerate(labels):
        lab[b, :len(l)] = torch.tensor(l)
    xd = x.to(dev, dtype)
    lse = torch.empty(B * T, device=dev)
    ops.row_lse(xd, V, lse)
    S = 2 * Lmax + 1
    alpha = torch.empty(B, T, S, device=dev); gamma = torch.empty(B, T, S, device=dev)
    nll = torch.empty(B, device=dev)
    p = ops.ctc_params(xd, B, T, V, lab.to(dev), torch.tensor([len(l) for l in labels], dtype=torch.int32, device=dev),
                       torch.tensor(in_len, dtype=torch.int32, device=dev), lse, alpha, gamma, nll)
    ops.ctc_fwd(p)
    # reference: torch CTC on fp64 log-softmax of the same (device-rounded) logits
    xr = xd.double().cpu()[:, :V].view(B, T, V).transpose(0, 1).contiguous().requires_grad_()
    lp = xr.log_softmax(-1)
    tgt = torch.cat([torch.tensor(l) for l in labels])
    ref = F.ctc_loss(lp, tgt, torch.tensor(in_len), torch.tensor([len(l) for l in labels]), blank=0,
                     reduction="none", zero_infinity=True)
    assert ref[2].item() == 0.0
    assert _rel(nll, ref) < (1e-5 if dtype == torch.float32 else 1e-3)
    (ref.sum() * 0.7 / B).backward()
    dloss = torch.tensor([0.7], device=dev)
    dx = torch.empty(B * T, Vp, device=dev, dtype=dtype)
    ops.ctc_bwd(p, dloss, 1.0 / B, dx)
    gref = xr.grad.transpose(0, 1).reshape(B * T, V)
    # log-space alpha/beta in fp32 carry ~T*eps*|log p| absolute error: judge the fp32 kernel
    # against torch's own fp32 CTC (the reference's arithmetic) on the same logits
    x32 = xd.float().cpu()[:, :V].view(B, T, V).transpose(0, 1).contiguous().requires_grad_()
    r32 = F.ctc_loss(x32.log_softmax(-1), tgt, torch.tensor(in_len), torch.tensor([len(l) for l in labels]),
                     blank=0, reduction="none", zero_infinity=True)
    (r32.sum() * 0.7 / B).backward()
    e32 = _rel(x32.grad.transpose(0, 1).reshape(B * T, V), gref)
    err = _rel(dx[:, :V], gref)
    assert err < (max(3 * e32, 1e-4) if dtype == torch.float32 else 1e-2), (err, e32)
    assert dx[:, V:].abs().max().item() == 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_label_smoothing(dev, dtype):
    R, V, Vp, sm, B = 90, 5049, 5056, 0.1, 3
    g = torch.Generator().manual_seed(4)
    x = torch.randn(R, Vp, generator=g) * 2
    tg = torch.randint(1, V, (R,), generator=g)
    tg[::7] = -1
    xd = x.to(dev, dtype)
    lse = torch.empty(R, device=dev); rl = torch.empty(R, device=dev)
    rc = torch.empty(R, dtype=torch.int32, device=dev)
    tgd = tg.to(torch.int32).to(dev)
    ops.lsm_fwd(xd, V, tgd, sm, lse, rl, rc)
    xr = xd.double().cpu()[:, :V].requires_grad_()
    ign = tg == -1
    q = torch.full((R, V), sm / (V - 1), dtype=torch.float64)
    q.scatter_(1, tg.masked_fill(ign, 0).unsqueeze(1), 1 - sm)
    kl = (q * (q.log() - xr.log_softmax(1))).masked_fill(ign.unsqueeze(1), 0)
    ref_rows = kl.sum(1)
    assert _rel(rl, ref_rows) < (1e-5 if dtype == torch.float32 else 1e-3)
    pred = xr.detach().argmax(1)
    corr = ((pred == tg) & ~ign).sum().item()
    assert int((rc == 1).sum()) == corr and int((rc == -1).sum()) == int(ign.sum())
    (kl.sum() / B * 0.9).backward()
    dx = torch.empty(R, Vp, device=dev, dtype=dtype)
    ops.lsm_bwd(xd, V, tgd, sm, lse, torch.tensor([0.9], device=dev), 1.0 / B, dx)
    assert _rel(dx[:, :V], xr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    out = torch.empty(4, device=dev)
    nll = torch.tensor([1.0, 2.0, 3.0], device=dev)
    ops.loss_finalize(B, nll, rl, rc, 0.1, out)
    lc, la = 6.0 / B, ref_rows.sum().item() / B
    assert abs(out[1].item() - lc) < 1e-5 and abs(out[2].item() - la) / la < 1e-4
    assert abs(out[0].item() - (0.1 * lc + 0.9 * la)) / la < 1e-4
    assert abs(out[3].item() - corr / int((~ign).sum())) < 1e-6


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ew_bwd_and_dropout(dev, dtype):
    R, N = 300, 3072
    dy = torch.randn(R, N, device=dev, dtype=dtype)
    gate = torch.randn(R, N, device=dev, dtype=dtype)
    out = torch.empty_like(dy)
    db = torch.zeros(N, device=dev)
    ops.ew_bwd(dy, out=out, gate=gate, act=L.ACT_RELU, db=db, alpha=2.0)
    ref = dy.double() * 2 * (gate.double() > 0)
    assert _rel(out, ref) < 1e-2
    assert _rel(db, ref.sum(0)) < 1e-2
    y = torch.empty_like(dy)
    dy = dy.abs() + 0.5           # no exact zeros: y == 0 iff dropped
    ops.dropout_fwd(dy, y, 0.3, 99)
    kept = y != 0
    assert 0.65 < kept.float().mean().item() < 0.75
    ops.ew_bwd(torch.ones_like(dy), out=out, drop_p=0.3, seed=99)
    mism = ((out != 0) != kept).nonzero()
    assert mism.shape[0] == 0, (mism[:5].tolist(), [(dy[r, c].item(), y[r, c].item(), out[r, c].item()) for r, c in mism[:5].tolist()])


def test_embed_mask_cast_pack(dev):
    V, D, R, Lq = 100, 256, 3 * 7, 7
    table = torch.randn(V, D, device=dev)
    tok = torch.randint(0, V, (R,), device=dev, dtype=torch.int32)
    pe = torch.randn(Lq, D, device=dev)
    y = torch.empty(R, D, device=dev)
    ops.embed_fwd(tok, table, pe, 16.0, y, Lq)
    ref = table[tok.long()] * 16 + pe.repeat(3, 1)
    assert _rel(y, ref) < 1e-6
    dt = torch.zeros(V, D, device=dev)
    dy = torch.randn(R, D, device=dev)
    ops.embed_bwd(tok, dy, 16.0, dt, Lq)
    rt = torch.zeros(V, D, device=dev).index_add_(0, tok.long(), dy * 16)
    assert _rel(dt, rt) < 1e-6
    x = torch.randn(2 * 5 * 3, 64, device=dev)
    ops.mask_rows(x.view(-1, 64), 2, 15, torch.tensor([15, 9], dtype=torch.int32, device=dev))
    assert x[15 + 9:].abs().sum() == 0 and x[:15 + 9].abs().sum() > 0
    a = torch.randn(3, 104, 11, device=dev)
    ap = torch.empty(33, 104, device=dev, dtype=torch.bfloat16)
    ops.audio_pack(a, ap)
    assert _rel(ap, a.transpose(1, 2).reshape(33, 104)) < 1e-2
    s = torch.randn(40, 24, device=dev)
    d = torch.ones(40, 32, device=dev, dtype=torch.bfloat16)[:, 4:28]
    ops.cast(s, d, alpha=2.0, beta=1.0)
    assert _rel(d, 2 * s + 1) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_as_2d_conv(dev, dtype):
    """Conv3d(1, 64, (5,7,7), stride (1,2,2), pad (2,3,3)) == time-stacked 2-D conv."""
    B, T = 2, 6
    g = torch.Generator().manual_seed(8)
    vid = torch.randn(B, 1, T, 88, 88, generator=g)
    w = torch.randn(64, 1, 5, 7, 7, generator=g) * 0.05
    ref = F.conv3d(vid.double(), w.double(), stride=(1, 2, 2), padding=(2, 3, 3))    # (B,64,T,44,44)
    xp = torch.empty(B * T, 88, 88, 8, device=dev, dtype=dtype)
    ops.stem_pack(vid.to(dev).contiguous(), xp)
    wp = torch.empty(64, 7, 7, 8, device=dev, dtype=dtype)
    ops.stem_wpack(w.to(dev), wp)
    geom = ops.ConvGeom(B * T, 88, 88, 8, 64, 7, 7, (2, 2), (3, 3))
    y = torch.empty(B * T, 44, 44, 64, device=dev, dtype=dtype)
    ops.conv_fwd(geom, xp, wp, y)
    out = y.view(B, T, 44, 44, 64).permute(0, 4, 1, 2, 3)
    assert _rel(out, ref) < (3e-5 if dtype == torch.float32 else 2e-2)
    # weight grad through the packed layout
    dyt = torch.randn(B, 64, T, 44, 44, generator=g)
    wr = w.double().requires_grad_()
    F.conv3d(vid.double(), wr, stride=(1, 2, 2), padding=(2, 3, 3)).backward(dyt.double())
    gp = torch.zeros(64, 7, 7, 8, device=dev)
    ops.conv_bwd_weight(geom, xp, dyt.permute(0, 2, 3, 4, 1).contiguous().to(dev, dtype).view(-1, 64), gp)
    gw = torch.zeros(64, 1, 5, 7, 7, device=dev)
    ops.stem_wgrad_unpack(gp, gw)
    assert _rel(gw, wr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("O,K,C", [(96, 16, 8), (1024, 128, 64), (40, 6, 6)])
def test_weightnorm(dev, O, K, C):
    """weight norm over dims (0, 1) of the torch (out, in/groups, k) weight: vectorised
    reduction (C % 4 == 0, incl. the pos-conv shape) and the scalar one (C = 6)"""
    g = torch.Generator().manual_seed(2)
    v = torch.randn(O, C, K, generator=g)          # torch layout (out, in/groups, k)
    gg = 1 + 0.1 * torch.randn(1, 1, K, generator=g)
    vr = v.double().requires_grad_(); gr = gg.double().requires_grad_()
    w = torch._weight_norm(vr, gr, 2)
    vd = v.permute(0, 2, 1).contiguous().to(dev)   # [o][k][c]
    gd = gg.flatten().to(dev)
    norm = torch.empty(K, device=dev)
    wd = torch.empty(O, K, C, device=dev)
    ops.weightnorm_fwd(vd, gd, norm, wd)
    assert _rel(wd, w.permute(0, 2, 1)) < 1e-5
    dw = torch.randn(O, C, K, generator=g)
    w.backward(dw.double())
    dv = torch.zeros(O, K, C, device=dev); dg = torch.zeros(K, device=dev); scr = torch.empty(K, device=dev)
    ops.weightnorm_bwd(vd, gd, norm, dw.permute(0, 2, 1).contiguous().to(dev), dv, dg, scr)
    assert _rel(dv, vr.grad.permute(0, 2, 1)) < 1e-5
    assert _rel(dg, gr.grad.flatten()) < 1e-5


def test_adamw_clip(dev):
    n = 10000
    g = torch.Generator().manual_seed(1)
    p0 = torch.randn(n, generator=g); gr = torch.randn(n, generator=g) * 3
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.005)
    for step in range(1, 4):
        ref.grad = gr.clone() * step
        torch.nn.utils.clip_grad_norm_([ref], 1.0)
        opt.step()
    pd = p0.to(dev); m = torch.zeros(n, device=dev); v = torch.zeros(n, device=dev)
    sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in range(1, 4):
        gd = (gr * step).to(dev)
        ss = torch.zeros(1, device=dev)
        ops.sumsq(gd, ss)
        ops.adamw(pd, gd, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.005, step=step,
                  shadow=sh, sumsq_buf=ss, max_norm=1.0)
    # fp32 params of magnitude ~1 after updates of ~1e-3: compare the params themselves
    assert (pd.cpu() - ref.detach()).abs().max().item() < 2e-6
    assert _rel(sh, pd) < 1e-2


def test_adamw_grid_cap_bit_identical(dev):
    """avsr_adamw_params.max_blocks (the overlapped update's grid cap) changes only the grid:
    parameters, moments and the bf16 shadow equal the full-grid launch bit for bit (unaligned
    head elements included)"""
    n = 3_000_003
    g = torch.Generator().manual_seed(3)
    base = [torch.randn(n, generator=g) for _ in range(4)]
    base[3] = base[3].abs()
    out = []
    for cap in (0, 64, 512):
        p, gr, m, v = (t.to(dev) for t in base)
        sh = torch.zeros(n, device=dev, dtype=torch.bfloat16)     # element 0 is outside the update
        ss = torch.zeros(1, device=dev)
        ops.sumsq(gr, ss)                       # (16-byte aligned input; the value only sets the clip)
        ops.adamw(p[1:], gr[1:], m[1:], v[1:], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01,
                  step=3, shadow=sh[1:], sumsq_buf=ss, max_norm=1.0, max_blocks=cap)
        out.append((p.cpu(), m.cpu(), v.cpu(), sh.cpu()))
    for other in out[1:]:
        for a, b in zip(out[0], other):
            assert torch.equal(a, b)
    # avsr_adamw_params.grad_clear: the same update, and every gradient element it read is 0 after
    p, gr, m, v = (t.to(dev) for t in base)
    sh = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    ss = torch.zeros(1, device=dev)
    ops.sumsq(gr, ss)
    ops.adamw(p[1:], gr[1:], m[1:], v[1:], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01,
              step=3, shadow=sh[1:], sumsq_buf=ss, max_norm=1.0, max_blocks=128, clear_grad=True)
    for a, b in zip(out[0], (p.cpu(), m.cpu(), v.cpu(), sh.cpu())):
        assert torch.equal(a, b)
    assert gr[1:].abs().max().item() == 0.0 and gr[0].item() == base[1][0].item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_pack_exact(dev, dtype):
    """time-stacked stem input: channel c of frame t = frame t + c - 2 (zero outside the clip,
    channels 5..7 zero); T spans several frame chunks of the kernel with a ragged last one"""
    B, T = 2, 37
    g = torch.Generator().manual_seed(9)
    vid = torch.randn(B, 1, T, 88, 88, generator=g)
    xp = torch.full((B * T, 88, 88, 8), float("nan"), device=dev, dtype=dtype)
    ops.stem_pack(vid.to(dev).contiguous(), xp)
    ref = torch.zeros(B, T, 88, 88, 8)
    for c in range(5):
        for t in range(T):
            tt = t + c - 2
            if 0 <= tt < T:
                ref[:, t, :, :, c] = vid[:, 0, tt]
    assert torch.equal(xp.cpu().float().view(B, T, 88, 88, 8), ref.to(dtype).float())
