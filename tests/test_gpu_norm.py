"""LayerNorm / BatchNorm(+PReLU, +residual) / stem max-pool / avg-pool kernels vs torch fp64."""
import pytest
import torch
import torch.nn.functional as F

from avsr_amd import ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _tol(dtype, f32=2e-5, b16=2e-2):
    return f32 if dtype == torch.float32 else b16


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,eps,rows", [(1024, 1e-5, 777), (2048, 1e-5, 777), (256, 1e-12, 777), (1024, 1e-5, 3001)])
def test_layernorm(dev, dtype, N, eps, rows):
    """rows = 3001: each of the backward's 1024 waves walks 2-3 rows through both register stages"""
    g = torch.Generator().manual_seed(N)
    x = torch.randn(rows, N, generator=g) * 2 + 0.5
    gam = 1 + 0.1 * torch.randn(N, generator=g)
    bet = 0.1 * torch.randn(N, generator=g)
    dy = torch.randn(rows, N, generator=g)
    dres = torch.randn(rows, N, generator=g)
    xd = x.to(dev, dtype)
    y, mean, rstd = ops.layernorm_fwd(xd, gam.to(dev), bet.to(dev), eps)
    xr = xd.double().cpu().requires_grad_(); gr = gam.double().requires_grad_(); br = bet.double().requires_grad_()
    ref = F.layer_norm(xr, (N,), gr, br, eps)
    assert _rel(y, ref) < _tol(dtype, 1e-5)
    ref.backward(dy.double())
    dg = torch.zeros(N, device=dev); db = torch.zeros(N, device=dev)
    dx = ops.layernorm_bwd(dy.to(dev, dtype), xd, gam.to(dev), mean, rstd, dres=dres.to(dev, dtype), dgamma=dg, dbeta=db)
    assert _rel(dx, xr.grad + dres.double()) < _tol(dtype, 1e-5)
    assert _rel(dg, gr.grad) < _tol(dtype, 1e-5)
    assert _rel(db, br.grad) < _tol(dtype, 1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm_bwd_fused_dropout_bias(dev, dtype, p):
    """The residual-branch dropout backward + bias gradient fused into the LayerNorm backward
    (engine._ln_bwd ew=...) equals LayerNorm backward followed by ew_bwd, bit for bit."""
    g = torch.Generator().manual_seed(11)
    rows, N = 613, 1024
    x = (torch.randn(rows, N, generator=g) * 2 + 0.5).to(dev, dtype)
    gam = (1 + 0.1 * torch.randn(N, generator=g)).to(dev)
    bet = (0.1 * torch.randn(N, generator=g)).to(dev)
    dy = torch.randn(rows, N, generator=g).to(dev, dtype)
    dres = torch.randn(rows, N, generator=g).to(dev, dtype)
    _, mean, rstd = ops.layernorm_fwd(x, gam, bet, 1e-5)
    outs = []
    for fused in (True, False):
        dg = torch.zeros(N, device=dev); dbt = torch.zeros(N, device=dev); dbias = torch.full((N,), 0.5, device=dev)
        gout = torch.empty(rows, N, device=dev, dtype=dtype)
        if fused:
            dx = ops.layernorm_bwd(dy, x, gam, mean, rstd, dres=dres, dgamma=dg, dbeta=dbt, g=gout, drop_p=p,
                                   seed=1234, db=dbias)
        else:
            dx = ops.layernorm_bwd(dy, x, gam, mean, rstd, dres=dres, dgamma=dg, dbeta=dbt)
            ops.ew_bwd(dx, out=gout, drop_p=p, seed=1234, db=dbias)
        torch.cuda.synchronize()
        outs.append((dx.clone(), gout.clone(), dg.clone(), dbt.clone(), dbias.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b) or _rel(a, b) < 1e-6
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def _partials(h, chunks=7):
    """(count, mean, M2) per channel per row-chunk, layout [C][tiles][3]."""
    parts = []
    for c in h.double().chunk(chunks, 0):
        n = torch.full((h.shape[1],), float(c.shape[0]), dtype=torch.float64)
        m = c.mean(0)
        parts.append(torch.stack([n, m, ((c - m) ** 2).sum(0)], -1))
    return torch.stack(parts, 1).float()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["plain", "identity", "downsample"])
def test_bn_act(dev, dtype, mode):
    g = torch.Generator().manual_seed(11)
    M, C = 3000, 128
    h = torch.randn(M, C, generator=g) * 1.5 + 0.3
    r = torch.randn(M, C, generator=g) * 0.7 - 0.2
    gam = 1 + 0.1 * torch.randn(C, generator=g); bet = 0.1 * torch.randn(C, generator=g)
    gam2 = 1 + 0.1 * torch.randn(C, generator=g); bet2 = 0.1 * torch.randn(C, generator=g)
    a = 0.25 + 0.05 * torch.randn(C, generator=g)
    rm = 0.1 * torch.randn(C, generator=g); rv = 0.5 + torch.rand(C, generator=g)
    hd, rd = h.to(dev, dtype), r.to(dev, dtype)
    st = ops.BnState(C, dev)
    rmd, rvd = rm.clone().to(dev), rv.clone().to(dev)
    ops.bn_finalize(st, gam.to(dev), bet.to(dev), rmd, rvd, partials=_partials(hd.float().cpu()).to(dev))
    st2 = None
    if mode == "downsample":
        st2 = ops.BnState(C, dev)
        ops.bn_finalize(st2, gam2.to(dev), bet2.to(dev), None, None, partials=_partials(rd.float().cpu()).to(dev))
    y = torch.empty_like(hd)
    ops.bn_act_fwd(hd, st, a.to(dev), y, res=None if mode == "plain" else rd, st2=st2)
    # torch reference (train-mode BN, momentum 0.1, unbiased running var)
    hr = hd.double().cpu().requires_grad_(); rr = rd.double().cpu().requires_grad_()
    P = [t.double().requires_grad_() for t in (gam, bet, gam2, bet2, a)]
    rm2, rv2 = rm.double().clone(), rv.double().clone()
    z = F.batch_norm(hr, rm2, rv2, P[0], P[1], training=True, momentum=0.1, eps=1e-5)
    if mode == "identity":
        z = z + rr
    elif mode == "downsample":
        z = z + F.batch_norm(rr, None, None, P[2], P[3], training=True, eps=1e-5)
    ref = F.prelu(z, P[4])
    assert _rel(y, ref) < _tol(dtype, 1e-5)
    assert _rel(rmd, rm2) < 1e-5 and _rel(rvd, rv2) < 1e-5
    dy = torch.randn(M, C, generator=g)
    ref.backward(dy.double())
    dh = torch.empty_like(hd); dh2 = torch.empty_like(hd) if mode == "downsample" else None
    grads = [torch.zeros(C, device=dev) for _ in range(5)]
    dz = ops.bn_act_bwd(dy.to(dev, dtype), hd, st, a.to(dev), dh, res=None if mode == "plain" else rd, st2=st2,
                        dh2=dh2, dprelu=grads[4], dgamma=grads[0], dbeta=grads[1],
                        dgamma2=grads[2] if st2 else None, dbeta2=grads[3] if st2 else None)
    tol = _tol(dtype, 1e-4, 3e-2)
    assert _rel(dh, hr.grad) < tol
    if mode == "identity":
        assert _rel(dz, rr.grad) < tol
    if mode == "downsample":
        assert _rel(dh2, rr.grad) < tol
        assert _rel(grads[2], P[2].grad) < tol and _rel(grads[3], P[3].grad) < tol
    assert _rel(grads[0], P[0].grad) < tol and _rel(grads[1], P[1].grad) < tol
    assert _rel(grads[4], P[4].grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_pool(dev, dtype):
    g = torch.Generator().manual_seed(5)
    n, H, W, C = 6, 44, 44, 64
    h = torch.randn(n, H, W, C, generator=g)
    gam = 1 + 0.1 * torch.randn(C, generator=g); bet = 0.1 * torch.randn(C, generator=g)
    a = 0.25 + 0.05 * torch.randn(C, generator=g)
    hd = h.to(dev, dtype)
    st = ops.BnState(C, dev)
    ops.bn_finalize(st, gam.to(dev), bet.to(dev), None, None, partials=_partials(hd.float().cpu().view(-1, C)).to(dev))
    y = torch.empty(n, 22, 22, C, device=dev, dtype=dtype)
    am = torch.empty(n, 22, 22, C, device=dev, dtype=torch.uint8)
    hmax = torch.empty(n, 22, 22, C, device=dev, dtype=dtype)
    ops.stem_pool_fwd(hd, n, H, W, st, a.to(dev), y, am, hmax=hmax)
    # hmax = h at the recorded argmax window position
    q = am.long().cpu()
    ih = (2 * torch.arange(22).view(1, 22, 1, 1) - 1 + q // 3).clamp(0, H - 1)
    iw = (2 * torch.arange(22).view(1, 1, 22, 1) - 1 + q % 3).clamp(0, W - 1)
    hc = hd.cpu()
    pick = hc[torch.arange(n).view(n, 1, 1, 1), ih, iw, torch.arange(C).view(1, 1, 1, C)]
    assert torch.equal(pick, hmax.cpu())
    hr = hd.double().cpu().permute(0, 3, 1, 2).requires_grad_()
    P = [t.double().requires_grad_() for t in (gam, bet, a)]
    z = F.prelu(F.batch_norm(hr, None, None, P[0], P[1], training=True, eps=1e-5), P[2])
    ref = F.max_pool2d(z, 3, 2, 1)
    assert _rel(y.permute(0, 3, 1, 2), ref) < _tol(dtype, 1e-5)
    dy = torch.randn(n, C, 22, 22, generator=g)
    ref.backward(dy.double())
    dh = torch.empty_like(hd)
    grads = [torch.zeros(C, device=dev) for _ in range(3)]
    ops.stem_pool_bwd(dy.permute(0, 2, 3, 1).contiguous().to(dev, dtype), am, hmax, hd, n, H, W, st, a.to(dev), dh,
                      dgamma=grads[0], dbeta=grads[1], dprelu=grads[2])
    tol = _tol(dtype, 1e-4, 3e-2)
    assert _rel(dh.permute(0, 3, 1, 2), hr.grad) < tol
    for gg, pp in zip(grads, P):
        assert _rel(gg, pp.grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,H,W", [(6, 44, 44), (3, 12, 16), (3, 10, 14), (2, 9, 7)])
def test_stem_bwd_apply_block_kernel(dev, dtype, monkeypatch, n, H, W, lib_opt):
    """the 2x2-block stem backward apply (even H, W) reproduces the per-pixel kernel (same windows,
    same addition order; the final fma contraction may differ: 1e-6 relative); odd sizes take
    the per-pixel kernel either way"""
    C = 64
    g = torch.Generator().manual_seed(n * H + W)
    hd = torch.randn(n, H, W, C, generator=g).to(dev, dtype)
    st = ops.BnState(C, dev)
    ops.bn_finalize(st, (1 + 0.1 * torch.randn(C, generator=g)).to(dev), (0.1 * torch.randn(C, generator=g)).to(dev),
                    None, None, partials=_partials(hd.float().cpu().view(-1, C)).to(dev))
    a = (0.25 + 0.05 * torch.randn(C, generator=g)).to(dev)
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    fw = []
    for pix in ("1", "0"):          # forward: 2x2 output blocks (even Ho, Wo) vs per-output windows
        lib_opt("stem_pool_2x2", 1 - int(pix))
        y = torch.full((n, Ho, Wo, C), float("nan"), device=dev, dtype=dtype)
        am = torch.full((n, Ho, Wo, C), 255, device=dev, dtype=torch.uint8)
        hmax = torch.full((n, Ho, Wo, C), float("nan"), device=dev, dtype=dtype)
        ops.stem_pool_fwd(hd, n, H, W, st, a, y, am, hmax=hmax)
        torch.cuda.synchronize()
        fw.append((y, am, hmax))
    for t0, t1 in zip(*fw):
        assert torch.equal(t0, t1)
    y, am, hmax = fw[1]
    dy = torch.randn(n, Ho, Wo, C, generator=g).to(dev, dtype)
    out = []
    for pix in ("1", "0"):
        lib_opt("stem_pool_2x2", 1 - int(pix))
        dh = torch.full_like(hd, float("nan"))
        grads = [torch.zeros(C, device=dev) for _ in range(3)]
        ops.stem_pool_bwd(dy, am, hmax, hd, n, H, W, st, a, dh, dgamma=grads[0], dbeta=grads[1], dprelu=grads[2])
        torch.cuda.synchronize()
        out.append((dh, grads))
    assert _rel(out[0][0], out[1][0]) < (1e-6 if dtype == torch.float32 else 8e-3)
    for g0, g1 in zip(out[0][1], out[1][1]):
        assert torch.equal(g0, g1)
    # the engine's pipelined stem backward: one reduction, then the apply over image ranges
    # (m_total = the whole batch's pixels) -> the same dh bit for bit
    lib_opt("stem_pool_2x2", 1)
    dzp, sums = ops.stem_pool_bwd_reduce(dy, hmax, n, H, W, st, a, dgamma=torch.zeros(C, device=dev),
                                         dbeta=torch.zeros(C, device=dev), dprelu=torch.zeros(C, device=dev))
    dzp = dzp.view(n, Ho, Wo, C)
    dh_full = ops.stem_pool_bwd_apply(dzp, am, hd, n, H, W, st, sums, torch.full_like(hd, float("nan")))
    dh_rng = torch.full_like(hd, float("nan"))
    for f0, f1 in ((0, 1), (1, n // 2 + 1), (n // 2 + 1, n)):
        if f1 > f0:
            ops.stem_pool_bwd_apply(dzp[f0:], am[f0:], hd[f0:], f1 - f0, H, W, st, sums, dh_rng[f0:],
                                    m_total=n * H * W)
    torch.cuda.synchronize()
    assert torch.equal(dh_full, dh_rng)
    assert torch.equal(dh_full, out[1][0])


BNR_CASES = [
    # nimg, hw (dgrad output = BN input grid), BN channels (conv cin), cout, k, stride, pad, residual
    (6, 22, 64, 64, 3, 1, 1, "identity"),       # 256x64 tiles, layer 1
    (5, 22, 64, 128, 1, 2, 0, "downsample"),    # a block's downsample dgrad into the previous bn2
    (7, 6, 256, 256, 3, 1, 1, "plain"),         # 128x128 tiles, bn1 of layer 3
    (9, 3, 512, 512, 3, 1, 1, "identity"),      # layer 4, ragged last row tile
    (4, 11, 128, 256, 3, 2, 1, "identity"),     # stride 2 by parity class, odd grid
    (4, 11, 128, 256, 1, 2, 0, "downsample"),   # 1x1 stride 2: three classes epilogue-only
]


@pytest.mark.parametrize("case", BNR_CASES)
def test_conv_dgrad_bn_epilogue(dev, case):
    """conv_bwd_data_bnr (BN + PReLU backward reduction in the data-grad epilogue) vs fp64:
    dz = prelu'(z) * (conv^T(dy) + beta*dx_old) and the folded sums / parameter gradients."""
    n, hw, cin, cout, k, s, p, mode = case
    g = torch.Generator().manual_seed(n * 1000 + cin)
    geom = ops.ConvGeom(n, hw, hw, cin, cout, k, k, (s, s), (p, p))
    ho = geom.hout
    M = n * hw * hw
    bf = torch.bfloat16
    dyt = torch.randn(n, cout, ho, ho, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) * (cout * k * k) ** -0.5
    h = (torch.randn(M, cin, generator=g) * 1.3 + 0.2).to(bf)
    r = (torch.randn(M, cin, generator=g) * 0.8 - 0.1).to(bf)
    old = torch.randn(M, cin, generator=g).to(bf)
    beta = 0.0 if mode == "plain" else 1.0

    def state():
        st = ops.BnState(cin, dev)
        st.mean.copy_(0.1 * torch.randn(cin, generator=g)); st.invstd.copy_(0.5 + torch.rand(cin, generator=g))
        st.scale.copy_(1 + 0.2 * torch.randn(cin, generator=g)); st.shift.copy_(0.2 * torch.randn(cin, generator=g))
        return st
    st = state()
    st2 = state() if mode == "downsample" else None
    a = 0.25 + 0.05 * torch.randn(cin, generator=g)
    dx = old.to(dev).clone()
    ws, tiles = ops.conv_bwd_data_bnr(geom, dyt.permute(0, 2, 3, 1).contiguous().to(dev, bf),
                                      wt.permute(0, 2, 3, 1).contiguous().to(dev, bf), dx, h.to(dev), st, a.to(dev),
                                      res=None if mode == "plain" else r.to(dev), st2=st2, beta=beta)
    grads = [torch.zeros(cin, device=dev) for _ in range(5)]
    sums = ops.bn_bwd_finalize(ws, tiles, cin, dbeta=grads[0], dgamma=grads[1], dprelu=grads[4],
                               dbeta2=grads[2] if st2 else None, dgamma2=grads[3] if st2 else None)
    # fp64 reference from the same bf16 operands
    xr = torch.zeros(n, cin, hw, hw, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wt.to(bf).double(), stride=s, padding=p).backward(dyt.to(bf).double())
    v = xr.grad.permute(0, 2, 3, 1).reshape(M, cin) + beta * old.double()
    cpu = lambda t: t.double().cpu()
    hd, rd = h.double(), r.double()
    z = hd * cpu(st.scale) + cpu(st.shift)
    if mode == "identity":
        z = z + rd
    elif mode == "downsample":
        z = z + rd * cpu(st2.scale) + cpu(st2.shift)
    dz = torch.where(z > 0, v, v * a.double())
    assert _rel(dx.view(M, cin), dz) < 2e-2
    s0 = dz.sum(0)
    s1 = (dz * (hd - cpu(st.mean)) * cpu(st.invstd)).sum(0)
    s3 = torch.where(z > 0, torch.zeros_like(v), v * z).sum(0)
    tol = 1e-2
    assert _rel(sums[:, 0], s0) < tol and _rel(sums[:, 1], s1) < tol
    assert _rel(grads[0], s0) < tol and _rel(grads[1], s1) < tol and _rel(grads[4], s3) < tol
    if st2 is not None:
        s2 = (dz * (rd - cpu(st2.mean)) * cpu(st2.invstd)).sum(0)
        assert _rel(sums[:, 2], s2) < tol and _rel(grads[3], s2) < tol and _rel(grads[2], s0) < tol


def test_avgpool(dev):
    x = torch.randn(50, 9, 512, device=dev)
    y = torch.empty(50, 512, device=dev)
    ops.avgpool_fwd(x, 50, 9, 512, y)
    assert _rel(y, x.mean(1)) < 1e-6
    dx = torch.empty_like(x)
    ops.avgpool_bwd(y, 50, 9, 512, dx)
    assert _rel(dx, y[:, None, :].expand_as(x) / 9) < 1e-6


@pytest.mark.parametrize("case", [(140, 22, 128, 128, 3, 1, 1, "identity"), (150, 22, 128, 128, 3, 1, 1, "plain")])
def test_conv_192_tiles_match_128(dev, monkeypatch, case, lib_opt):
    """the 192x128 row tiles of the forward / data-grad convolutions (library option conv_192, chosen for
    the large-M ResNet stages) against 128x128: identical stored outputs (same K order), BN
    partial statistics and fused BN-backward sums equal up to the per-tile grouping (1e-5)."""
    n, hw, cin, cout, k, s, p, mode = case
    g = torch.Generator().manual_seed(n + hw)
    geom = ops.ConvGeom(n, hw, hw, cin, cout, k, k, (s, s), (p, p))
    M = n * hw * hw
    bf = torch.bfloat16
    x = torch.randn(M, cin, generator=g).to(dev, bf)
    w = (torch.randn(cout, k, k, cin, generator=g) * (cin * k * k) ** -0.5).to(dev, bf)
    dy = torch.randn(geom.out_pixels, cout, generator=g).to(dev, bf)
    h = (torch.randn(M, cin, generator=g) * 1.3 + 0.2).to(dev, bf)
    r = (torch.randn(M, cin, generator=g) * 0.8 - 0.1).to(dev, bf)
    st = ops.BnState(cin, dev)
    st.mean.copy_(0.1 * torch.randn(cin, generator=g)); st.invstd.copy_(0.5 + torch.rand(cin, generator=g))
    st.scale.copy_(1 + 0.2 * torch.randn(cin, generator=g)); st.shift.copy_(0.2 * torch.randn(cin, generator=g))
    a = (0.25 + 0.05 * torch.randn(cin, generator=g)).to(dev)
    out = {}
    for flag in ("0", "1"):
        lib_opt("conv_192", int(flag))
        y = torch.empty(geom.out_pixels, cout, device=dev, dtype=bf)
        part = torch.empty(cout, ops.conv_stat_tiles(geom, ops.dtype_code(x)), 3, device=dev)
        ops.conv_fwd(geom, x, w, y, stats=part)
        bst = ops.BnState(cout, dev)
        ops.bn_finalize(bst, torch.ones(cout, device=dev), torch.zeros(cout, device=dev), None, None, partials=part)
        dx = torch.zeros(M, cin, device=dev, dtype=bf)
        ws, tiles = ops.conv_bwd_data_bnr(geom, dy, w, dx, h, st, a, res=None if mode == "plain" else r,
                                          beta=0.0)
        sums = ops.bn_bwd_finalize(ws, tiles, cin)
        torch.cuda.synchronize()
        out[flag] = (y, bst.mean.clone(), bst.invstd.clone(), dx, sums, part.shape[1], tiles)
    o0, o1 = out["0"], out["1"]
    assert o1[5] < o0[5] and o1[6] < o0[6], "the 192-row tiles were not selected"
    assert torch.equal(o0[0], o1[0]) and torch.equal(o0[3], o1[3])
    assert _rel(o1[1], o0[1]) < 1e-5 and _rel(o1[2], o0[2]) < 1e-5
    assert _rel(o1[4], o0[4]) < 1e-5


@pytest.mark.parametrize("case", [(40, 22, 64, 64, 3, 1, 1, "identity"), (33, 22, 64, 64, 3, 1, 1, "plain")])
def test_conv_patch_matches_general(dev, monkeypatch, case, lib_opt):
    """the patch-resident 3x3 stride-1 kernel (library option conv_patch, ResNet stage 1: one LDS image of
    the padded input patch per 256-pixel block) against the general implicit-GEMM kernel:
    same tiles, same K order -> bit-identical forward outputs, BN partial statistics, data-grads
    with the fused BN-backward epilogue and their column sums, and plain data-grads
    accumulated into an existing dx (beta = 1). Ragged last tile (M % 256 != 0)."""
    n, hw, cin, cout, k, s, p, mode = case
    g = torch.Generator().manual_seed(n + hw + 7)
    geom = ops.ConvGeom(n, hw, hw, cin, cout, k, k, (s, s), (p, p))
    M = n * hw * hw
    assert M % 256
    bf = torch.bfloat16
    x = torch.randn(M, cin, generator=g).to(dev, bf)
    w = (torch.randn(cout, k, k, cin, generator=g) * (cin * k * k) ** -0.5).to(dev, bf)
    dy = torch.randn(geom.out_pixels, cout, generator=g).to(dev, bf)
    h = (torch.randn(M, cin, generator=g) * 1.3 + 0.2).to(dev, bf)
    r = (torch.randn(M, cin, generator=g) * 0.8 - 0.1).to(dev, bf)
    dx0 = (torch.randn(M, cin, generator=g) * 0.3).to(dev, bf)
    st = ops.BnState(cin, dev)
    st.mean.copy_(0.1 * torch.randn(cin, generator=g)); st.invstd.copy_(0.5 + torch.rand(cin, generator=g))
    st.scale.copy_(1 + 0.2 * torch.randn(cin, generator=g)); st.shift.copy_(0.2 * torch.randn(cin, generator=g))
    a = (0.25 + 0.05 * torch.randn(cin, generator=g)).to(dev)
    out = {}
    for flag in ("0", "1"):
        lib_opt("conv_patch", int(flag))
        y = torch.empty(geom.out_pixels, cout, device=dev, dtype=bf)
        part = torch.empty(cout, ops.conv_stat_tiles(geom, ops.dtype_code(x)), 3, device=dev)
        ops.conv_fwd(geom, x, w, y, stats=part)
        dx = dx0.clone()
        ws, tiles = ops.conv_bwd_data_bnr(geom, dy, w, dx, h, st, a, res=None if mode == "plain" else r,
                                          beta=1.0)
        dxp = dx0.clone()
        ops.conv_bwd_data(geom, dy, w, dxp, beta=1.0)
        torch.cuda.synchronize()
        out[flag] = (y, part.clone(), dx, ws[:tiles * 4 * cin].clone(), dxp)
    for t0, t1 in zip(out["0"], out["1"]):
        assert torch.equal(t0, t1)
    # and the forward is a convolution (fp64 reference)
    xr = x.double().view(n, hw, hw, cin).permute(0, 3, 1, 2)
    wr = w.double().permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xr, wr, padding=1).permute(0, 2, 3, 1).reshape(M, cout)
    assert _rel(out["1"][0], ref) < 2e-2


@pytest.mark.parametrize("tiles,C", [(257, 64), (3000, 64), (11337, 128), (1000, 200)])
def test_bn_finalize_fold_matches_fp64(dev, tiles, C):
    """avsr_bn_bwd_finalize over > 256 partial rows (the fold into ceil(tiles / 16) slices,
    one wave per slice and 64 channels) vs fp64 column sums of the partials, and the parameter-gradient accumulation"""
    g = torch.Generator().manual_seed(tiles + C)
    part = torch.randn(tiles, 4, C, generator=g)
    ws = torch.zeros(ops.bn_fin_ws(tiles, C), device=dev)
    ws[:tiles * 4 * C] = part.reshape(-1).to(dev)
    db, dg, dp = (torch.full((C,), 0.5, device=dev) for _ in range(3))
    sums = ops.bn_bwd_finalize(ws, tiles, C, dbeta=db, dgamma=dg, dprelu=dp)
    want = part.double().sum(0)                                   # (4, C)
    got = torch.stack([sums.view(C, 3)[:, 0], sums.view(C, 3)[:, 1], sums.view(C, 3)[:, 2]]).double().cpu()
    scale = part.double().abs().sum(0)
    assert ((got - want[:3]).abs() <= 1e-5 * scale[:3] + 1e-6).all()
    for t, q in ((db, 0), (dg, 1), (dp, 3)):
        assert ((t.double().cpu() - 0.5 - want[q]).abs() <= 1e-5 * scale[q] + 1e-5).all(), q
