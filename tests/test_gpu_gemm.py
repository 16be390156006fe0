"""GEMM kernel parity vs a torch fp32 reference (float64 for the parity-mode check)."""
import pytest
import torch

from avsr_amd import ops, _lib as L

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (6000, 1024, 1024), (257, 5049, 104), (656, 96, 4096), (33, 17, 8)])
def test_linear_fwd(dev, dtype, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).to(dev, dtype)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, dtype)
    b = torch.randn(N, generator=g).to(dev)
    y = ops.linear_fwd(x, W, b)
    ref = x.double() @ W.double().t() + b.double()
    tol = 3e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, ref) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_epilogues(dev, dtype):
    M, N, K = 300, 384, 256
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(M, K, generator=g).to(dev, dtype)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, dtype)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(M, N, generator=g).to(dev, dtype)
    h = torch.empty(M, N, device=dev, dtype=dtype)
    y = ops.linear_fwd(x, W, b, act=L.ACT_GELU, preact=h, res=r)
    href = x.double() @ W.double().t() + b.double()
    yref = torch.nn.functional.gelu(href) + r.double()
    tol = 3e-5 if dtype == torch.float32 else 2e-2
    assert _rel(h, href) < tol
    assert _rel(y, yref) < tol
    # relu variant
    y2 = ops.linear_fwd(x, W, b, act=L.ACT_RELU)
    assert _rel(y2, torch.relu(href)) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_backward(dev, dtype):
    M, N, K = 500, 256, 192
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(M, K, generator=g).to(dev, dtype)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, dtype)
    dy = torch.randn(M, N, generator=g).to(dev, dtype)
    hgate = torch.randn(M, K, generator=g).to(dev, dtype)
    dx = ops.linear_dgrad(dy, W)
    ref = dy.double() @ W.double()
    tol = 3e-5 if dtype == torch.float32 else 2e-2
    assert _rel(dx, ref) < tol
    dx2 = ops.linear_dgrad(dy, W, gate=hgate, act=L.ACT_GELU)
    hd = hgate.double().requires_grad_()
    torch.nn.functional.gelu(hd).backward(ref)
    assert _rel(dx2, hd.grad) < tol
    dW = torch.zeros(N, K, device=dev, dtype=torch.float32)
    ops.linear_wgrad(dy, x, dW)
    wref = dy.double().t() @ x.double()
    assert _rel(dW, wref) < tol
    ops.linear_wgrad(dy, x, dW, beta=1.0)
    assert _rel(dW, 2 * wref) < tol


def test_dropout_epilogue_consistent(dev):
    M, N, K = 256, 512, 128
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev) * 0.1
    y = ops.linear_fwd(x, W, None, drop_p=0.25, seed=1234)
    ref = x @ W.t()
    kept = y != 0
    frac = kept.float().mean().item()
    assert 0.72 < frac < 0.78
    assert _rel(y[kept], ref[kept] / 0.75) < 1e-5
    # backward recomputes the same mask from the same (seed, index)
    dy = torch.ones(M, N, device=dev)
    Wi = torch.eye(N, device=dev)
    dx = ops.linear_dgrad(dy, Wi, drop_p=0.25, seed=1234)
    assert torch.equal(dx != 0, kept)


def _ref_gemm(A, B, a_kmajor, b_kmajor):
    """torch fp32 reference of avsr_gemm: C[m,n] = sum_k A(m,k) B(n,k) for the four layouts."""
    Af = A.float() if a_kmajor else A.float().t()
    Bf = B.float() if b_kmajor else B.float().t()
    return Af @ Bf.t()


@pytest.fixture(params=["auto", "128", "256", "256x128", "128x256", "128s3", "128w8s3", "pp", "192", "192x256", "64"])
def gemm_tile(request, lib_opt):
    """forces each LDS-DMA tile configuration (library option gemm_tile, read per launch by avsr_gemm)"""
    lib_opt("gemm_tile", request.param)
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("a_kmajor,b_kmajor", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K,splitk", [(296, 200, 200, 1), (128, 136, 64, 1), (1000, 384, 1000, 3), (6000, 1024, 512, 2)])
def test_gemm_layouts_bf16(dev, gemm_tile, a_kmajor, b_kmajor, M, N, K, splitk):
    """Every operand layout through the bf16 LDS-DMA path (M, N >= 128) and the register-staged
    path, ragged M/N/K edges, split-K into an fp32 C; tolerance: fp32 accumulation of bf16
    products vs torch fp32 on the same bf16 inputs (2e-3 relative to the output scale)."""
    g = torch.Generator().manual_seed(M + N + K)
    A = (torch.randn(M, K, generator=g) if a_kmajor else torch.randn(K, M, generator=g)).to(dev, torch.bfloat16)
    B = (torch.randn(N, K, generator=g) if b_kmajor else torch.randn(K, N, generator=g)).to(dev, torch.bfloat16)
    ref = _ref_gemm(A, B, a_kmajor, b_kmajor)
    C = torch.zeros(M, N, device=dev, dtype=torch.float32)
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_kmajor, b_kmajor=b_kmajor,
             lda=A.shape[1], ldb=B.shape[1], ldc=N, splitk=splitk)
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err
    if splitk > 1:   # slab workspace mode: C = 0.5 * A.B + 1.0 * C_old, no atomics
        C0 = torch.randn(M, N, device=dev)
        C2 = C0.clone()
        ws = torch.full((ops.slab_ws(1, splitk, M, N),), float("nan"), device=dev)
        ops.gemm(A, B, C2, M=M, N=N, K=K, a_kmajor=a_kmajor, b_kmajor=b_kmajor,
                 lda=A.shape[1], ldb=B.shape[1], ldc=N, splitk=splitk, ws=ws, alpha=0.5, beta=1.0)
        err = (C2 - (0.5 * ref + C0)).abs().max().item() / ref.abs().max().item()
        assert err < 2e-3, err
    if splitk == 1:
        Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        ops.gemm(A, B, Cb, M=M, N=N, K=K, a_kmajor=a_kmajor, b_kmajor=b_kmajor,
                 lda=A.shape[1], ldb=B.shape[1], ldc=N)
        err = (Cb.float() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 8e-3, err


@pytest.mark.parametrize("M,N,K,splitk", [(1024, 1024, 6000, 4), (3072, 1024, 6000, 1), (256, 384, 1000, 1),
                                           (136, 200, 328, 1), (1024, 1024, 1000, 3), (640, 512, 64, 1),
                                           (1024, 1024, 6000, 1), (200, 136, 999, 1)])
def test_wgrad_dual_kernel(dev, monkeypatch, M, N, K, splitk, lib_opt):
    """Weight-gradient GEMM dW[M][N] = beta*dW + alpha * dy^T x (both operands r-contiguous, the
    in-block split-K kernel: two wave groups per block over halves of the K range, one LDS
    reduction; with splitk > 1 also split over blocks into slabs): vs fp64, ragged K (a group
    whose last tile is empty), ragged M / N edges, beta accumulation; bit-identical run to run;
    and within fp32 re-association of the 4-wave core (library option wgrad_dual = 0)."""
    g = torch.Generator().manual_seed(M + N + K)
    dy = torch.randn(K, M, generator=g).to(dev, torch.bfloat16)
    x = torch.randn(K, N, generator=g).to(dev, torch.bfloat16)
    C0 = torch.randn(M, N, generator=g).to(dev)
    ref = 0.5 * (dy.double().t() @ x.double()) + C0.double()

    def run():
        C = C0.clone()
        ws = torch.full((ops.slab_ws(1, splitk, M, N),), float("nan"), device=dev) if splitk > 1 else None
        ops.gemm(dy, x, C, M=M, N=N, K=K, a_kmajor=False, b_kmajor=False, lda=M, ldb=N, ldc=N,
                 alpha=0.5, beta=1.0, splitk=splitk, ws=ws)
        return C
    a, b = run(), run()
    assert torch.equal(a, b)
    assert _rel(a, ref) < 1e-5 * (K ** 0.5)
    if splitk > 1:
        # the in-kernel slab reduction (last-arriving split per tile) equals the separate pass
        monkeypatch.setattr(ops, "SLAB_FUSED_REDUCE", False)
        assert torch.equal(run(), a)
        monkeypatch.setattr(ops, "SLAB_FUSED_REDUCE", True)
    lib_opt("wgrad_dual", 0)
    c = run()
    assert _rel(a, c.double()) < 1e-5 * (K ** 0.5)


@pytest.mark.gpu
@pytest.mark.parametrize("shapes", [[(6000, 3072, 1024), (6000, 1024, 1024)],          # encoder QKV + out-proj
                                    [(700, 256, 384), (700, 136, 200), (96, 128, 128)],   # ragged; 3 problems
                                    [(640, 120, 256), (640, 256, 256)]])                  # one not groupable
def test_wgrad_group_matches_single(dev, shapes):
    """avsr_gemm_wgrad_group (several weight-gradients dW += alpha dy^T x in one grid) equals each
    problem's own avsr_gemm launch (unsplit weight-gradient kernel) bit for bit, beta accumulation
    included; a problem of another shape (N = 120 < 128: not the weight-gradient core) falls back to
    one-by-one launches"""
    g = torch.Generator().manual_seed(sum(a + b + c for a, b, c in shapes))
    probs = []
    for M, N, K in shapes:          # dy [M][N], x [M][K], dW [N][K]
        probs.append((torch.randn(M, N, generator=g).to(dev, torch.bfloat16), torch.randn(M, K, generator=g).to(dev, torch.bfloat16),
                      torch.randn(N, K, generator=g).to(dev), 0.5))
    got = [dW.clone() for _, _, dW, _ in probs]
    ops.wgrad_group([(dy, x, w, al) for (dy, x, _, al), w in zip(probs, got)])
    for (dy, x, dW, al), gw in zip(probs, got):
        M, N = dy.shape
        K = x.shape[1]
        want = dW.clone()
        ops.gemm(dy, x, want, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=dy.stride(0), ldb=x.stride(0),
                 ldc=want.stride(0), alpha=al, beta=1.0)
        assert torch.equal(gw, want), (M, N, K, (gw - want).abs().max().item())
        ref = al * (dy.double().t() @ x.double()) + dW.double()
        assert _rel(gw, ref) < 1e-5 * (M ** 0.5)


@pytest.mark.gpu
def test_gemm_batched_strided_bf16(dev, gemm_tile):
    """batch > 1 with operand / output strides (attention-style batched products)."""
    g = torch.Generator().manual_seed(5)
    Bt, M, N, K = 3, 256, 192, 96
    A = torch.randn(Bt, M, K, generator=g).to(dev, torch.bfloat16)
    B = torch.randn(Bt, K, N, generator=g).to(dev, torch.bfloat16)
    C = torch.zeros(Bt, M, N, device=dev, dtype=torch.float32)
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=True, b_kmajor=False, lda=K, ldb=N, ldc=N, batch=Bt,
             strideA=M * K, strideB=K * N, strideC=M * N)
    ref = torch.bmm(A.float(), B.float())
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1000, 1024, 4096), (6000, 256, 1024), (200, 512, 136), (96, 512, 256)])
def test_dgrad_fused_bias_grad(dev, gemm_tile, M, N, K):
    """linear_dgrad(..., db=) reduces the bias gradient of its output (column sums of the stored
    values, here after GELU' and dropout) in the GEMM epilogue, per row tile of every tile
    configuration; ragged M, and M < 128 (separate reduction pass). Reference: fp64 column sums
    of the returned bf16 tensor (the fused sums use the fp32 values before rounding: 2e-3)."""
    g = torch.Generator().manual_seed(M + N)
    dy = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * N ** -0.5).to(dev, torch.bfloat16)
    h = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    db0 = torch.randn(K, generator=g).to(dev)
    db = db0.clone()
    out = ops.linear_dgrad(dy, W, gate=h, act=L.ACT_GELU, drop_p=0.1, seed=11, db=db)
    ref = out.double().sum(0)
    err = ((db.double() - db0.double()) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("tile", ["192", "192x256", "256x128", "pp", "64", "64s4"])
def test_tile_configs_bit_identical(dev, monkeypatch, tile, lib_opt):
    """Every tile configuration accumulates each output over the same K order (64-deep K-tiles,
    the same 16x16x32 MFMA sequence), so the fused-epilogue results must equal the 128x128
    tile's bit for bit: FFN1-style forward (bias, GELU, pre-activation store, residual,
    dropout) and FFN2-style data-grad (GELU' gate, dropout, fused bias gradient); ragged M/N/K."""
    M, N, K = 1000, 776, 328
    g = torch.Generator().manual_seed(17)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    dy = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    hg = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)

    def run():
        h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        y = ops.linear_fwd(x, W, b, act=L.ACT_GELU, preact=h, res=r, drop_p=0.1, seed=7)
        db = torch.zeros(K, device=dev)
        dx = ops.linear_dgrad(dy, W, gate=hg, act=L.ACT_GELU, drop_p=0.1, seed=9, db=db)
        torch.cuda.synchronize()
        return y, h, dx, db

    lib_opt("gemm_tile", "128")
    ref = run()
    lib_opt("gemm_tile", tile)
    got = run()
    for a_, b_, name in zip(got[:3], ref[:3], ("y", "preact", "dx")):
        assert torch.equal(a_, b_), (tile, name, (a_.float() - b_.float()).abs().max().item())
    # the bias gradient sums per-row-tile partials: a different row-tile height re-associates
    assert _rel(got[3], ref[3]) < 1e-5



@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(1, 1024, 1024), (5, 3072, 1024), (40, 5049, 1024), (17, 1024, 3072),
                                   (64, 100, 264), (33, 17, 8), (47, 256, 512), (12, 300, 3072)])
def test_skinny_linear(dev, dtype, M, N, K):
    """Few-row linears (beam-search decoder steps) on the vector-ALU skinny kernel: vs fp64 with
    the bias / ReLU / residual epilogue; run-to-run bit-identical."""
    g = torch.Generator(device="cpu").manual_seed(M * 13 + N + K)
    x = torch.randn(M, K, generator=g).to(dev, dtype)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, dtype)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(M, N, generator=g).to(dev, dtype)
    y = ops.linear_fwd(x, W, b, act=L.ACT_RELU, res=r)
    ref = torch.relu(x.double() @ W.double().t() + b.double()) + r.double()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert _rel(y, ref) < tol
    y2 = ops.linear_fwd(x, W, b, act=L.ACT_RELU, res=r)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,K", [(1024, 4096), (1024, 1024), (4096, 1024), (5056, 1024), (256, 2048)])
def test_skinny_k_split_rows_independent(dev, N, K, dtype):
    """The few-row path with its K split (skinny_ws given: S = avsr_gemm_skinny_splits(dtype, N, K)
    workgroup rows, fp32 partials reduced in a fixed order): S depends on dtype, N and K only, so
    every row equals the same row launched alone, bit for bit (batched beam search == per-utterance
    search relies on it); split and unsplit both match fp64. bf16 (vector-ALU kernel): >= 512
    workgroups; fp32 (matrix-core kernel, 8 waves per workgroup): >= 256 workgroups with K chunks of
    256..1024."""
    S = ops.skinny_splits(N, K, dtype)
    if dtype == torch.float32:
        assert S == {(1024, 4096): 4, (1024, 1024): 4, (4096, 1024): 1, (5056, 1024): 1, (256, 2048): 8}[(N, K)], (N, K, S)
    else:
        # the decoder's output layer (5056 columns) has no room for a split in AVSR_SKINNY_WS
        assert S == (1 if N == 5056 else {4096: 2}.get(N, S)) and (S > 1 or N == 5056), (N, K, S)
    g = torch.Generator(device="cpu").manual_seed(N + K)
    x = torch.randn(40, K, generator=g).to(dev, dtype)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, dtype)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(40, N, generator=g).to(dev, dtype)
    y = ops.linear_fwd(x, W, b, act=L.ACT_RELU, res=r, skinny_split=True)
    y1 = ops.linear_fwd(x, W, b, act=L.ACT_RELU, res=r, skinny_split=False)
    for m in (0, 7, 39):
        one = ops.linear_fwd(x[m:m + 1].contiguous(), W, b, act=L.ACT_RELU, res=r[m:m + 1].contiguous(),
                             skinny_split=True)
        assert torch.equal(one[0], y[m]), m
    ref = torch.relu(x.double() @ W.double().t() + b.double()) + r.double()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert _rel(y, ref) < tol and _rel(y1, ref) < tol
    assert _rel(y, y1.double()) < (1e-6 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("M,N,K,off", [(40, 3072, 1024, 3.0), (10, 1024, 1024, 3.0), (64, 4096, 1024, 3.0),
                                       (1, 256, 256, 3.0), (17, 100, 512, 3.0), (40, 1024, 1000 - 1000 % 16, 3.0),
                                       (40, 1024, 1024, 100.0), (5, 256, 256, -300.0)])
def test_skinny_layernorm_prologue(dev, M, N, K, off):
    """LayerNorm folded into the following fp32 few-row linear (ops.fold_layernorm + the kernel's
    LayerNorm prologue; the decoder's norm1/2/3 at decode time): vs LayerNorm then Linear in fp64,
    inputs with a common offset up to 150x their spread (the cancellation case of
    rstd * (x W'^T - mean * c1), removed by the kernel's per-row shift); a row equals the same
    row launched alone, bit for bit."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g) * 2 + off).to(dev)
    gam = (torch.rand(K, generator=g) + 0.5).to(dev)
    bet = (torch.randn(K, generator=g) * 0.1).to(dev)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    r = torch.randn(M, N, generator=g).to(dev)
    Wg, bb, c1 = ops.fold_layernorm(W, b, gam, bet)
    y = ops.linear_fwd(x, Wg, bb, act=L.ACT_RELU, res=r, ln=(c1, 1e-12))
    y1 = ops.linear_fwd(x, Wg, bb, act=L.ACT_RELU, res=r, ln=(c1, 1e-12), skinny_split=False)
    xd = x.double()
    ln = (xd - xd.mean(1, keepdim=True)) / torch.sqrt(xd.var(1, unbiased=False, keepdim=True) + 1e-12)
    ref = torch.relu((ln * gam.double() + bet.double()) @ W.double().t() + b.double()) + r.double()
    assert _rel(y, ref) < 2e-6 and _rel(y1, ref) < 2e-6      # split (chunk statistics combined) / unsplit
    for m in (0, M - 1):
        one = ops.linear_fwd(x[m:m + 1].contiguous(), Wg, bb, act=L.ACT_RELU, res=r[m:m + 1].contiguous(),
                             ln=(c1, 1e-12))
        assert torch.equal(one[0], y[m]), m


@pytest.mark.parametrize("ln", [False, True])
def test_skinny_kv_cache_append(dev, ln):
    """fused QKV projection of a decode step (kv=...): the Q third goes to the output, the K / V
    thirds to the caches at rows pos * rows + m (pos read on the device), nothing else written;
    equal bit for bit to the projection followed by the copy (avsr_beam_kv_put)."""
    g = torch.Generator(device="cpu").manual_seed(11 + ln)
    M, D, K, rows, Lmax = 40, 256, 512, 40, 6
    x = (torch.randn(M, K, generator=g) + 1).to(dev)
    W = (torch.randn(3 * D, K, generator=g) * K ** -0.5).to(dev)
    b = torch.randn(3 * D, generator=g).to(dev)
    lnarg = None
    if ln:
        W, b, c1 = ops.fold_layernorm(W, b, (torch.rand(K, generator=g) + 0.5).to(dev),
                                      (torch.randn(K, generator=g) * 0.1).to(dev))
        lnarg = (c1, 1e-12)
    pos = torch.tensor([3], dtype=torch.int32, device=dev)
    kc = torch.full((Lmax * rows, D), float("nan"), device=dev)
    vc = torch.full((Lmax * rows, D), float("nan"), device=dev)
    q = torch.full((M, 3 * D), float("nan"), device=dev)
    ops.linear_fwd(x, W, b, out=q, ln=lnarg, kv=(kc, vc, pos, rows))
    full = ops.linear_fwd(x, W, b, ln=lnarg)
    kr, vr = torch.full_like(kc, float("nan")), torch.full_like(vc, float("nan"))
    ops.beam_kv_put(full, kr, vr, pos, rows, D)
    assert torch.equal(q[:, :D], full[:, :D])
    assert torch.isnan(q[:, D:]).all()
    assert torch.equal(kc[3 * rows:3 * rows + M], kr[3 * rows:3 * rows + M])
    assert torch.equal(vc[3 * rows:3 * rows + M], vr[3 * rows:3 * rows + M])
    assert torch.isnan(kc[:3 * rows]).all() and torch.isnan(kc[3 * rows + M:]).all()


@pytest.mark.parametrize("M,N,K", [(20, 768, 256), (40, 1024, 1024), (17, 256, 512)])
def test_skinny_layernorm_prologue_every_row_alone(dev, M, N, K):
    """batch invariance of the folded-LayerNorm few-row linear for EVERY row: each row of an
    M-row launch (row tiles of 16: the row's lane position differs between the launches) equals
    the same row launched alone, bit for bit, with and without the fused K/V-cache append"""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    x = (torch.randn(M, K, generator=g) * 1.5 + torch.randn(M, 1, generator=g) * 4).to(dev)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    Wg, bb, c1 = ops.fold_layernorm(W, b, (torch.rand(K, generator=g) + 0.5).to(dev),
                                    (torch.randn(K, generator=g) * 0.1).to(dev))
    y = ops.linear_fwd(x, Wg, bb, ln=(c1, 1e-12))
    for m in range(M):
        one = ops.linear_fwd(x[m:m + 1].contiguous(), Wg, bb, ln=(c1, 1e-12))
        assert torch.equal(one[0], y[m]), m
    if N % 3 == 0:
        D = N // 3
        pos = torch.tensor([1], dtype=torch.int32, device=dev)
        kc = torch.zeros(2 * M, D, device=dev); vc = torch.zeros(2 * M, D, device=dev)
        q = ops.linear_fwd(x, Wg, bb, ln=(c1, 1e-12), kv=(kc, vc, pos, M))
        for m in range(M):
            k1 = torch.zeros(2, D, device=dev); v1 = torch.zeros(2, D, device=dev)
            q1 = ops.linear_fwd(x[m:m + 1].contiguous(), Wg, bb, ln=(c1, 1e-12), kv=(k1, v1, pos, 1))
            assert torch.equal(q1[0, :D], q[m, :D]) and torch.equal(k1[1], kc[M + m]) and torch.equal(v1[1], vc[M + m]), m


@pytest.mark.parametrize("M,N,K", [(20, 768, 256), (40, 1024, 1024), (17, 256, 512)])
def test_skinny_every_row_alone(dev, M, N, K):
    """the plain fp32 few-row linear (no LayerNorm prologue): every row of an M-row launch equals
    the same row launched alone, bit for bit"""
    g = torch.Generator(device="cpu").manual_seed(M * 5 + N + K)
    x = (torch.randn(M, K, generator=g) + 3).to(dev)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    y = ops.linear_fwd(x, W, b)
    for m in range(M):
        one = ops.linear_fwd(x[m:m + 1].contiguous(), W, b)
        assert torch.equal(one[0], y[m]), m
