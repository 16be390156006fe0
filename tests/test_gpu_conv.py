"""Implicit-GEMM convolution kernels vs torch fp64 convolution (NCHW reference)."""
import pytest
import torch
import torch.nn.functional as F

from avsr_amd import ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


CASES = [
    # nimg, h, w, cin, cout, k, stride, pad
    (6, 22, 22, 64, 64, 3, 1, 1),
    (5, 22, 22, 64, 128, 3, 2, 1),
    (5, 22, 22, 64, 128, 1, 2, 0),
    (7, 6, 6, 256, 512, 3, 2, 1),
    (5, 11, 11, 128, 256, 3, 2, 1),   # odd input: parity classes of unequal size
    (5, 11, 11, 128, 256, 1, 2, 0),
    (4, 3, 3, 512, 512, 3, 1, 1),
    (3, 88, 88, 8, 64, 7, 2, 3),      # stem as 2-D conv over 8 packed channels
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES)
def test_conv2d(dev, dtype, case):
    n, h, w, cin, cout, k, s, p = case
    g = torch.Generator().manual_seed(n * 100 + cin)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) * (cin * k * k) ** -0.5
    ref = F.conv2d(x.double(), wt.double(), stride=s, padding=p)
    ho, wo = ref.shape[2], ref.shape[3]
    geom = ops.ConvGeom(n, h, w, cin, cout, k, k, (s, s), (p, p))
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, dtype)
    wd = wt.permute(0, 2, 3, 1).contiguous().to(dev, dtype)
    y = torch.empty(n, ho, wo, cout, device=dev, dtype=dtype)
    tiles = ops.conv_stat_tiles(geom, ops.dtype_code(xd))
    stats = torch.empty(cout, tiles, 3, device=dev)
    ops.conv_fwd(geom, xd, wd, y, stats)
    tol = 3e-5 if dtype == torch.float32 else 2e-2
    assert _rel(y.permute(0, 3, 1, 2), ref) < tol
    # BN partial statistics combine to the batch mean / biased variance
    cnt, mean, m2 = stats[..., 0].double(), stats[..., 1].double(), stats[..., 2].double()
    tot = cnt.sum(1, keepdim=True)
    gm = (cnt * mean).sum(1, keepdim=True) / tot
    var = ((m2 + cnt * (mean - gm) ** 2).sum(1, keepdim=True) / tot).flatten()
    gm = gm.flatten()
    rm = ref.mean(dim=(0, 2, 3)); rv = ref.var(dim=(0, 2, 3), unbiased=False)
    assert _rel(gm, rm) < (1e-4 if dtype == torch.float32 else 3e-2) or (gm - rm).abs().max() < 1e-3
    assert _rel(var, rv) < (1e-4 if dtype == torch.float32 else 3e-2)
    # data grad and weight grad
    dyt = torch.randn(n, cout, ho, wo, generator=g)
    xr = x.double().requires_grad_(); wr = wt.double().requires_grad_()
    F.conv2d(xr, wr, stride=s, padding=p).backward(dyt.double())
    dy = dyt.permute(0, 2, 3, 1).contiguous().to(dev, dtype)
    dx = torch.empty(n, h, w, cin, device=dev, dtype=dtype)
    ops.conv_bwd_data(geom, dy, wd, dx)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < tol
    dw = torch.zeros(cout, k, k, cin, device=dev)
    ops.conv_bwd_weight(geom, xd, dy, dw)
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_posconv_grouped_1d(dev, dtype):
    """Wav2Vec2PositionalConvEmbedding conv: Conv1d(D, D, k=128, pad=64, groups=16), drop last frame."""
    B, T, D, G, K = 3, 37, 256, 16, 128
    cg = D // G
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B, T, D, generator=g)
    wt = torch.randn(D, cg, K, generator=g) * (cg * K) ** -0.5
    ref = F.conv1d(x.double().transpose(1, 2), wt.double(), padding=K // 2, groups=G)[:, :, :-1].transpose(1, 2)
    geom = ops.ConvGeom(B, T, 1, cg, cg, K, 1, (1, 1), (K // 2, 0), groups=G, hout=T, wout=1)
    xd = x.contiguous().to(dev, dtype)
    wd = wt.permute(0, 2, 1).contiguous().to(dev, dtype)         # [D][K][cg] = [cout][kh][kw=1][cin]
    y = torch.empty(B, T, D, device=dev, dtype=dtype)
    ops.conv_fwd(geom, xd, wd, y)
    tol = 3e-5 if dtype == torch.float32 else 2e-2
    assert _rel(y, ref) < tol
    dyt = torch.randn(B, T, D, generator=g)
    xr = x.double().requires_grad_(); wr = wt.double().requires_grad_()
    out = F.conv1d(xr.transpose(1, 2), wr, padding=K // 2, groups=G)[:, :, :-1].transpose(1, 2)
    out.backward(dyt.double())
    dy = dyt.to(dev, dtype)
    dx = torch.empty(B, T, D, device=dev, dtype=dtype)
    ops.conv_bwd_data(geom, dy, wd, dx)
    assert _rel(dx, xr.grad) < tol
    dw = torch.zeros(D, K, cg, device=dev)
    ops.conv_bwd_weight(geom, xd, dy, dw)
    assert _rel(dw.permute(0, 2, 1), wr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


def test_gemm_splitk(dev):
    M, N, K = 64, 576, 20000
    a = torch.randn(K, M, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    c = torch.zeros(M, N, device=dev)
    ops.gemm(a, b, c, M=M, N=N, K=K, a_kmajor=False, b_kmajor=False, lda=M, ldb=N, ldc=N, splitk=16)
    ref = a.double().t() @ b.double()
    assert _rel(c, ref) < 1e-2


@pytest.mark.parametrize("splitk", [0, 1, 3, 40])
@pytest.mark.parametrize("case", [(40, 22, 22, 64, 64, 3, 1, 1), (30, 11, 11, 128, 256, 3, 2, 1),
                                  (12, 88, 88, 8, 64, 7, 2, 3)])     # stem geometry
def test_wgrad_slab_accumulates(dev, case, splitk):
    """Split-K weight gradient through the fp32 slab workspace (+ chunked reduce) matches the
    atomic path and torch, accumulates into a non-zero dw, and tolerates a 4-byte-aligned dw view."""
    n, h, w, cin, cout, k, s, p = case
    g = torch.Generator().manual_seed(n + cout)
    x = torch.randn(n, cin, h, w, generator=g)
    geom = ops.ConvGeom(n, h, w, cin, cout, k, k, (s, s), (p, p))
    ho, wo = geom.hout, geom.wout
    dyt = torch.randn(n, cout, ho, wo, generator=g)
    xr = x.double().requires_grad_()
    wr = torch.zeros(cout, cin, k, k, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, stride=s, padding=p).backward(dyt.double())
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    dy = dyt.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    init = torch.randn(cout, k, k, cin, generator=g)
    buf = torch.zeros(1 + init.numel(), device=dev)
    dw = buf[1:].view(cout, k, k, cin)                   # offset by one float
    dw.copy_(init.to(dev))
    ops.conv_bwd_weight(geom, xd, dy, dw, splitk=splitk)
    dwa = init.to(dev).clone()
    ops.conv_bwd_weight(geom, xd, dy, dwa, splitk=splitk, slab=False)
    ref = wr.grad.permute(0, 2, 3, 1) + init.double()
    assert _rel(dw, ref) < 2e-2
    assert _rel(dw - init.to(dev), dwa - init.to(dev)) < 1e-4


S2_CASES = [(5, 22, 22, 64, 128, 3, 2, 1), (5, 11, 11, 128, 256, 3, 2, 1), (7, 6, 6, 256, 512, 3, 2, 1),
            (5, 11, 11, 128, 256, 1, 2, 0), (3, 22, 22, 64, 128, 1, 2, 0)]


@pytest.mark.parametrize("beta", [0.0, 1.0])
@pytest.mark.parametrize("case", S2_CASES)
def test_stride2_dgrad_parity_classes_match_full(dev, case, beta, monkeypatch, lib_opt):
    """The stride-2 data-grad split into input-pixel parity classes (conv.hip s2_launch) adds
    the same non-zero products in the same order as the full col2im GEMM: bit-identical."""
    n, h, w, cin, cout, k, s, p = case
    g = torch.Generator().manual_seed(n * 7 + cin + k)
    geom = ops.ConvGeom(n, h, w, cin, cout, k, k, (s, s), (p, p))
    bf = torch.bfloat16
    dy = torch.randn(n, geom.hout, geom.wout, cout, generator=g).to(dev, bf)
    wd = (torch.randn(cout, k, k, cin, generator=g) * (cin * k * k) ** -0.5).to(dev, bf)
    old = torch.randn(n, h, w, cin, generator=g).to(dev, bf)
    outs = []
    for mode in ("1", "0"):
        lib_opt("conv_s2phase", int(mode))
        dx = old.clone()
        ops.conv_bwd_data(geom, dy, wd, dx, beta=beta)
        outs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_stats_at_192_eligible_shape(dev, dtype):
    """the s3h fault's regression on the device: a stage-2 conv with enough rows for the
    192-row bf16 tile (M = 3000 x 11 x 11 = 363,000), BN partials sized by conv_stat_tiles for
    the dtype, statistics combining to the batch moments; a buffer sized for the other
    dtype's tile count is refused before launch."""
    n, h, c = 3000, 11, 128
    geom = ops.ConvGeom(n, h, h, c, c, 3, 3, (1, 1), (1, 1))
    tiles = ops.conv_stat_tiles(geom, ops.dtype_code(torch.empty(0, dtype=dtype)))
    other = ops.conv_stat_tiles(geom, ops.dtype_code(torch.empty(0, dtype=torch.bfloat16 if dtype == torch.float32
                                                                   else torch.float32)))
    M = n * h * h
    assert tiles == -(-M // (192 if dtype == torch.bfloat16 else 128)) and tiles != other
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, h, h, c, generator=g).to(dev, dtype)
    w = (torch.randn(c, 3, 3, c, generator=g) * (9 * c) ** -0.5).to(dev, dtype)
    y = torch.empty(n, h, h, c, device=dev, dtype=dtype)
    if other < tiles:
        with pytest.raises(ValueError):
            ops.conv_fwd(geom, x, w, y, torch.empty(c, other, 3, device=dev))
    guard = torch.full((c * tiles * 3 + 4096,), 12345.0, device=dev)
    stats = guard[:c * tiles * 3].view(c, tiles, 3)
    ops.conv_fwd(geom, x, w, y, stats)
    torch.cuda.synchronize()
    assert bool((guard[c * tiles * 3:] == 12345.0).all()), "statistics written past the buffer"
    cnt, mean, m2 = stats[..., 0].double(), stats[..., 1].double(), stats[..., 2].double()
    assert torch.allclose(cnt.sum(1), torch.full((c,), float(M), device=dev, dtype=torch.float64))
    tot = cnt.sum(1, keepdim=True)
    gm = (cnt * mean).sum(1, keepdim=True) / tot
    var = ((m2 + cnt * (mean - gm) ** 2).sum(1, keepdim=True) / tot).flatten()
    yf = y.double().reshape(-1, c)
    assert _rel(gm.flatten(), yf.mean(0)) < 1e-3 or (gm.flatten() - yf.mean(0)).abs().max() < 1e-4
    assert _rel(var, yf.var(0, unbiased=False)) < 1e-3


@pytest.mark.parametrize("B,T", [(2, 7), (1, 375)])
def test_stem_conv_direct(dev, B, T):
    """stem Conv3d (k 5x7x7, stride 1x2x2, pad 2x3x3) straight from the fp32 video
    (stem.hip, K = 288 grouped (frame, row) x 8 columns) vs fp64 conv3d on the same
    bf16-rounded operands; BN partial statistics combine to the batch moments. T = 7: frames
    outside the clip (time padding) are hit at both ends by one run; T = 375: 23 runs of 17
    frames per band, the last one a single frame (the ring's frames loaded ahead of a run's end)."""
    g = torch.Generator().manual_seed(11)
    video = torch.randn(B, 1, T, 88, 88, generator=g)
    w = torch.randn(64, 1, 5, 7, 7, generator=g) * 0.05
    ref = F.conv3d(video.bfloat16().double(), w.bfloat16().double(), stride=(1, 2, 2), padding=(2, 3, 3))
    ref = ref.permute(0, 2, 3, 4, 1).reshape(B * T * 44 * 44, 64)
    wk = torch.empty(64, ops.STEM_K, device=dev, dtype=torch.bfloat16)
    ops.stem_wpack2(w.to(dev), wk)
    tiles = ops.stem_conv_tiles(B, T)
    h = torch.empty(B * T * 44 * 44, 64, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(64, tiles, 3, device=dev)
    ops.stem_conv_fwd(video.to(dev), wk, h, stats)
    torch.cuda.synchronize()
    assert _rel(h, ref) < 8e-3
    cnt, mean, m2 = stats[..., 0].double(), stats[..., 1].double(), stats[..., 2].double()
    assert torch.all(cnt.sum(1) == B * T * 44 * 44)
    tot = cnt.sum(1, keepdim=True)
    gm = (cnt * mean).sum(1, keepdim=True) / tot
    var = ((m2 + cnt * (mean - gm) ** 2).sum(1, keepdim=True) / tot).flatten()
    assert (gm.flatten().cpu() - ref.mean(0)).abs().max() < 1e-3 * ref.abs().max()
    assert _rel(var, ref.var(0, unbiased=False)) < 2e-3
    h2 = torch.empty_like(h)
    ops.stem_conv_fwd(video.to(dev), wk, h2)          # statistics optional (eval)
    torch.cuda.synchronize()
    assert torch.equal(h, h2)


@pytest.mark.parametrize("hw,c", [(22, 64), (11, 128), (6, 256), (3, 512)])
@pytest.mark.parametrize("nimg", [1, 37, 600])
def test_wgrad_patch_matches_general(dev, nimg, hw, c, monkeypatch, lib_opt):
    """Patch-resident weight-grad of the stage-1..4 3x3 convolutions (persistent blocks,
    per-block slabs, ordered reduce; stages 3-4: several images per tile, a part tile at the end
    when nimg is not a multiple) vs the general implicit-GEMM weight-grad and fp64 torch;
    blocks without tiles (nimg = 1), accumulation into a non-zero dw, run-to-run bit-identical."""
    g = torch.Generator().manual_seed(nimg + c)
    geom = ops.ConvGeom(nimg, hw, hw, c, c, 3, 3, (1, 1), (1, 1))
    x = torch.randn(nimg, c, hw, hw, generator=g)
    dyt = torch.randn(nimg, c, hw, hw, generator=g)
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    dy = dyt.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    init = torch.randn(c, 3, 3, c, generator=g).to(dev)
    dw1 = init.clone()
    ops.conv_bwd_weight(geom, xd, dy, dw1)
    dw1b = init.clone()
    ops.conv_bwd_weight(geom, xd, dy, dw1b)
    assert torch.equal(dw1, dw1b)
    lib_opt("conv_wpatch", 0)
    dw2 = init.clone()
    ops.conv_bwd_weight(geom, xd, dy, dw2)
    assert _rel(dw1 - init, dw2 - init) < 1e-4
    xr = xd.double().cpu().permute(0, 3, 1, 2).requires_grad_()
    wr = torch.zeros(c, c, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, padding=1).backward(dy.double().cpu().permute(0, 3, 1, 2))
    assert _rel(dw1 - init, wr.grad.permute(0, 2, 3, 1)) < 1e-4


@pytest.mark.parametrize("nimg", [1, 13, 600])
def test_stem_wgrad_patch_matches_general(dev, nimg, lib_opt):
    """Patch-resident stem weight-grad (packed 8-channel input, 7 x 7 / stride 2 / pad 3,
    persistent blocks over 4-row tiles, per-block slabs, ordered reduce) vs the general
    implicit-GEMM weight-grad and fp64 torch: blocks without tiles (nimg = 1), tile ranges
    spanning images, accumulation into a non-zero dw, run-to-run bit-identical."""
    g = torch.Generator().manual_seed(nimg)
    geom = ops.ConvGeom(nimg, 88, 88, 8, 64, 7, 7, (2, 2), (3, 3))
    x = torch.randn(nimg, 88, 88, 8, generator=g)
    x[..., 5:] = 0                                   # the packing's zero channels
    xd = x.to(dev, torch.bfloat16)
    dy = torch.randn(nimg * 44 * 44, 64, generator=g).to(dev, torch.bfloat16)
    init = torch.randn(64, 7, 7, 8, generator=g).to(dev)
    dw1 = init.clone()
    ops.conv_bwd_weight(geom, xd, dy, dw1)
    dw1b = init.clone()
    ops.conv_bwd_weight(geom, xd, dy, dw1b)
    assert torch.equal(dw1, dw1b)
    lib_opt("stem_wpatch", 0)
    dw2 = init.clone()
    ops.conv_bwd_weight(geom, xd, dy, dw2)
    assert _rel(dw1 - init, dw2 - init) < 1e-4
    if nimg <= 13:
        xr = xd.double().cpu().permute(0, 3, 1, 2)
        wr = torch.zeros(64, 8, 7, 7, dtype=torch.float64, requires_grad=True)
        F.conv2d(xr, wr, stride=2, padding=3).backward(dy.double().cpu().view(nimg, 44, 44, 64).permute(0, 3, 1, 2))
        assert _rel(dw1 - init, wr.grad.permute(0, 2, 3, 1)) < 1e-5
