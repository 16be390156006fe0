"""Thin tensor-level wrappers over the C-ABI (include/avsr_hip.h).

Each function validates shapes/dtypes on the host, then launches on the caller's current
stream. Nothing here computes on the CPU; a missing library raises (no fallback).
"""
import ctypes
import os

import torch

from . import _lib as L

_DT = {torch.float32: L.AVSR_F32, torch.bfloat16: L.AVSR_BF16}

# optional launch probes (bench.py): {"gemm": {"match": fn(M, N, K, ak, bk, dtype) -> bool,
# "stamps": int64 device tensor [2 * max launches] initialised to {-1, 0} pairs (the kernel's
# in-kernel first-start / last-end s_memrealtime stamps, 100 MHz), "events": [(start, end)]}}
# — HIP events recorded on the launching (current) stream beside them
PROBE = {}

SLAB_PAD = 1088   # AVSR_GEMM_SLAB_PAD


def slab_ws(batch, splitk, M, N):
    """fp32 floats of a split-K slab workspace (AVSR_GEMM_SLAB_WS)"""
    return batch * splitk * (M * N + SLAB_PAD)


def dtype_code(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise L.AvsrLibError(f"unsupported dtype {t.dtype}")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_SKINNY_WS = {}
SKINNY_WS = 1 << 19        # AVSR_SKINNY_WS (fp32 partials), followed by
SKINNY_CNT = 4096          # AVSR_SKINNY_CNT zeroed uint32 arrival counters
# few-row (decoder step) linears: split K over more workgroups (gemm(skinny_split=None) default;
# C4 / C5 decode 84 -> 93 / 15.0 -> 16.4 utt/s, profiles/r04_decode_split_ab.json)
SKINNY_SPLIT = True
# split-K weight-gradients reduce their slabs inside the GEMM (last-arriving split per tile)
SLAB_FUSED_REDUCE = True


def skinny_splits(N, K, dtype=torch.float32):
    """the K-split count the few-row path uses for an (N, K) weight of `dtype` when split (avsr_hip.h)"""
    code = L.AVSR_BF16 if dtype == torch.bfloat16 else L.AVSR_F32
    return int(L.load().avsr_gemm_skinny_splits(code, int(N), int(K)))


def _norm_dev(device):
    """workspace-cache key of a device: always with its index"""
    device = torch.device(device)
    return device if device.index is not None else torch.device(device.type, torch.cuda.current_device())


def _skinny_ws(device):
    """per (device, stream) partial-sum workspace of the few-row GEMM path: launches on one
    stream run in order, so one buffer per stream is never read and written at once. Its
    arrival counters must start at zero: a stream that will be captured into a graph gets its
    workspace from reserve_stream_workspaces() BEFORE the capture (a zero-fill recorded inside
    a capture only runs when that graph is replayed)."""
    device = _norm_dev(device)
    key = (device, L.stream_ptr().value)
    ws = _SKINNY_WS.get(key)
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            raise L.AvsrLibError("few-row GEMM workspace first requested inside a graph capture: call "
                                 "ops.reserve_stream_workspaces() on the capture stream before capturing")
        ws = _SKINNY_WS[key] = torch.zeros(SKINNY_WS + SKINNY_CNT, device=device, dtype=torch.float32)
    return ws


_SLAB_CNT = {}
SLAB_CNT = 4096            # AVSR_SLAB_CNT


def _slab_cnt(device):
    """per (device, stream) zeroed arrival counters of the slab split-K weight-gradients (every
    launch leaves them zero; launches on one stream run in order)"""
    key = (_norm_dev(device), L.stream_ptr().value)
    c = _SLAB_CNT.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            raise L.AvsrLibError("slab counters first requested inside a graph capture")
        c = _SLAB_CNT[key] = torch.zeros(SLAB_CNT, device=key[0], dtype=torch.int32)
    return c


def reserve_stream_workspaces(device, dec_attn_floats=0):
    """create (zeroed) the current stream's few-row GEMM workspace and slab split-K counters and
    size its dec_attn partial buffer to at least `dec_attn_floats`, eagerly — call outside any
    graph capture, on the stream that will be captured"""
    assert not torch.cuda.is_current_stream_capturing()
    device = _norm_dev(device)
    _skinny_ws(device)
    _slab_cnt(device)
    key = (device, L.stream_ptr().value)
    ws = _DA_WS.get(key)
    if dec_attn_floats and (ws is None or ws.numel() < dec_attn_floats):
        _DA_WS[key] = torch.empty(dec_attn_floats, device=device, dtype=torch.float32)


def gemm(A, B, C, *, M, N, K, a_kmajor, b_kmajor, lda, ldb, ldc, batch=1,
         strideA=0, strideB=0, strideC=0, alpha=1.0, beta=0.0, bias=None, act=L.ACT_NONE,
         epi_bwd=False, preact=None, res=None, ldr=None, strideR=0, gate=None, drop_p=0.0, seed=0,
         splitk=1, ws=None, db=None, db_ws=None, skinny_split=None, ln_c1=None, ln_eps=0.0, kv=None):
    """Raw GEMM launch: C[b,m,n] = epi(alpha * sum_k A(b,m,k) B(b,n,k)). See avsr_hip.h.
    skinny_split: few-row launches (M <= 64) split K over skinny_splits(N, K) workgroup rows
    (None: the module default SKINNY_SPLIT). ln_c1 / ln_eps: LayerNorm prologue of the fp32
    few-row kernel (A = LayerNorm input, B = gamma o W, ln_c1 = B's row sums)."""
    lib = L.load()
    assert A.is_cuda and B.is_cuda and C.is_cuda
    assert A.dtype == B.dtype, "A/B dtype mismatch"
    dt = dtype_code(A)
    c_f32 = 1 if (C.dtype == torch.float32 and dt == L.AVSR_BF16) else 0
    if not c_f32:
        assert C.dtype == A.dtype
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    for t in (res, preact, gate):
        if t is not None:
            assert t.dtype == A.dtype
    p = L.GemmParams()
    p.M, p.N, p.K, p.batch = M, N, K, batch
    p.dtype, p.a_kmajor, p.b_kmajor, p.c_f32 = dt, int(a_kmajor), int(b_kmajor), c_f32
    p.A, p.lda, p.strideA = A.data_ptr(), lda, strideA
    p.B, p.ldb, p.strideB = B.data_ptr(), ldb, strideB
    p.C, p.ldc, p.strideC = C.data_ptr(), ldc, strideC
    p.alpha, p.beta = alpha, beta
    p.bias = None if bias is None else bias.data_ptr()
    p.act, p.epi_bwd = act, int(epi_bwd)
    p.preact = None if preact is None else preact.data_ptr()
    p.res = None if res is None else res.data_ptr()
    p.ldr = ldc if ldr is None else ldr
    p.strideR = strideR
    p.gate = None if gate is None else gate.data_ptr()
    p.drop_p, p.seed = float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF
    p.splitk = int(splitk)
    if ws is not None:
        assert ws.dtype == torch.float32 and ws.numel() >= slab_ws(batch, splitk, M, N)
        p.ws = ws.data_ptr()
    if (SKINNY_SPLIT if skinny_split is None else skinny_split) and M <= 64 and splitk <= 1:
        p.skinny_ws = _skinny_ws(A.device).data_ptr()   # K-split partials of the few-row vector-ALU path
    elif ws is not None and splitk > 1 and SLAB_FUSED_REDUCE:
        p.slab_cnt = _slab_cnt(A.device).data_ptr()     # arrival counters: in-kernel slab reduction
    if ln_c1 is not None:
        assert ln_c1.dtype == torch.float32 and ln_c1.numel() >= N and dt == L.AVSR_F32
        p.ln_c1, p.ln_eps = ln_c1.data_ptr(), float(ln_eps)
    if kv is not None:           # (k cache, v cache, device position, rows per step)
        kc, vc, pos, rows = kv
        assert kc.dtype == vc.dtype == torch.float32 and pos.dtype == torch.int32 and dt == L.AVSR_F32
        p.kv_k, p.kv_v, p.kv_pos, p.kv_rows = kc.data_ptr(), vc.data_ptr(), pos.data_ptr(), int(rows)
    if db is not None:
        assert db.dtype == torch.float32 and db.numel() >= N and db_ws is not None and db_ws.dtype == torch.float32
        assert db_ws.numel() >= ((M + 63) // 64) * N
        p.db, p.db_ws = db.data_ptr(), db_ws.data_ptr()
    probe = PROBE.get("gemm")
    if probe is not None and probe["match"](M, N, K, a_kmajor, b_kmajor, dt):
        # in-kernel {first start, last end} stamps of this launch (s_memrealtime, 100 MHz) in
        # a preallocated int64 buffer; plus HIP events on the launching stream for comparison
        i = len(probe["events"])
        st = probe["stamps"]
        assert 2 * i + 2 <= st.numel(), "probe stamp buffer full"
        p.stamp = st[2 * i:].data_ptr()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        L.check(lib.avsr_gemm(ctypes.byref(p), L.stream_ptr()), "avsr_gemm")
        e.record()
        probe["events"].append((s, e))
        return C
    L.check(lib.avsr_gemm(ctypes.byref(p), L.stream_ptr()), "avsr_gemm")
    return C


def wgrad_group(problems):
    """several weight-gradients dW (fp32, [N][K]) += alpha * dy^T x (dy [M][N], x [M][K], bf16)
    in one launch (avsr_gemm_wgrad_group): problems = [(dy, x, dW, alpha), ...], at most 4"""
    lib = L.load()
    arr = (L.GemmParams * len(problems))()
    for p, (dy, x, dW, alpha) in zip(arr, problems):
        assert dy.dtype == x.dtype == torch.bfloat16 and dW.dtype == torch.float32
        M, N = dy.shape
        K = x.shape[1]
        p.M, p.N, p.K, p.batch = N, K, M, 1
        p.dtype, p.a_kmajor, p.b_kmajor, p.c_f32 = L.AVSR_BF16, 0, 0, 1
        p.A, p.lda = dy.data_ptr(), dy.stride(0)
        p.B, p.ldb = x.data_ptr(), x.stride(0)
        p.C, p.ldc = dW.data_ptr(), dW.stride(0)
        p.alpha, p.beta = float(alpha), 1.0
        p.ldr, p.splitk = dW.stride(0), 1
    L.check(lib.avsr_gemm_wgrad_group(arr, len(problems), L.stream_ptr()), "avsr_gemm_wgrad_group")


# ---------------------------------------------------------------------------------------
# Linear layer building blocks (x: (M, K) row-major, W: (N, K) = torch.nn.Linear.weight)
# ---------------------------------------------------------------------------------------

def linear_fwd(x, W, bias=None, *, act=L.ACT_NONE, preact=None, res=None, drop_p=0.0, seed=0, out=None,
               skinny_split=None, ln=None, kv=None):
    """y = dropout(act(x W^T + b)) + res ; optionally stores h = x W^T + b into `preact`.
    ln = (c1, eps): x is the input of a LayerNorm folded into this linear (fold_layernorm):
    y = act(LayerNorm(x) W0^T + b0) + res with W = gamma o W0, b = W0 beta + b0.
    kv = (k_cache, v_cache, pos, rows): fused QKV projection whose K / V thirds are appended to the
    caches at rows pos * rows + m (only the Q third is written to `out`)."""
    M, K = x.shape
    N = W.shape[0]
    assert W.shape[1] == K and x.stride(1) == 1 and W.stride(1) == 1
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    gemm(x, W, out, M=M, N=N, K=K, a_kmajor=True, b_kmajor=True, lda=x.stride(0), ldb=W.stride(0),
         ldc=out.stride(0), bias=bias, act=act, preact=preact, res=res,
         ldr=None if res is None else res.stride(0), drop_p=drop_p, seed=seed, skinny_split=skinny_split,
         ln_c1=None if ln is None else ln[0], ln_eps=0.0 if ln is None else ln[1], kv=kv)
    return out


def fold_layernorm(W, b, gamma, beta):
    """weights of LayerNorm(gamma, beta) followed by Linear(W, b) for linear_fwd(ln=...):
    (gamma o W, W beta + b, row sums of gamma o W); the sums in fp64 (one-time weight preparation)"""
    Wg = (W * gamma.unsqueeze(0)).contiguous()
    bb = (W.double() @ beta.double() + (0 if b is None else b.double())).float()
    c1 = Wg.double().sum(1).float()
    return Wg, bb, c1


def linear_dgrad(dy, W, *, gate=None, act=L.ACT_NONE, drop_p=0.0, seed=0, out=None, beta=0.0, db=None):
    """dx = (dy W) [* dropout mask][* act'(gate)]  — gradient w.r.t. the layer input.
    db (fp32 [K]): += column sums of dx (the bias gradient of the layer dx is the output
    gradient of), reduced in the GEMM epilogue."""
    M, N = dy.shape
    K = W.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=dy.dtype)
    # the epilogue reduction needs the LDS-DMA bf16 core (avsr_gemm: glds_ok) and 8-column vectors
    fused = (db is not None and dy.dtype == torch.bfloat16 and M >= 128 and K >= 128 and K % 8 == 0
             and out.stride(0) % 8 == 0)
    ws = _colsum_ws(((M + 63) // 64) * K, dy.device) if fused else None   # AVSR_GEMM_COLSUM_WS
    gemm(dy, W, out, M=M, N=K, K=N, a_kmajor=True, b_kmajor=False, lda=dy.stride(0), ldb=W.stride(0),
         ldc=out.stride(0), epi_bwd=True, gate=gate, act=act, drop_p=drop_p, seed=seed, beta=beta,
         db=db if fused else None, db_ws=ws)
    if db is not None and not fused:
        ew_bwd(out, db=db)
    return out


def linear_wgrad(dy, x, dW, *, beta=0.0):
    """dW (fp32, (N, K)) = beta*dW + dy^T x."""
    M, N = dy.shape
    K = x.shape[1]
    assert dW.shape == (N, K) and dW.dtype == torch.float32
    gemm(dy, x, dW, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=dy.stride(0), ldb=x.stride(0),
         ldc=dW.stride(0), beta=beta)
    return dW


# ---------------------------------------------------------------------------------------
# Implicit-GEMM convolution (NHWC activations, weights [cout][kh][kw][cin])
# ---------------------------------------------------------------------------------------

class ConvGeom:
    """Geometry of one (grouped) 2-D convolution over NHWC tensors."""

    def __init__(self, nimg, hin, win, cin, cout, kh, kw, stride=(1, 1), pad=(0, 0), groups=1,
                 hout=None, wout=None, ldx=None, ldy=None):
        self.nimg, self.hin, self.win, self.cin, self.cout = nimg, hin, win, cin, cout
        self.kh, self.kw = kh, kw
        self.sh, self.sw = stride
        self.ph, self.pw = pad
        self.groups = groups
        self.hout = hout if hout is not None else (hin + 2 * self.ph - kh) // self.sh + 1
        self.wout = wout if wout is not None else (win + 2 * self.pw - kw) // self.sw + 1
        self.ldx = ldx if ldx is not None else groups * cin
        self.ldy = ldy if ldy is not None else groups * cout

    def params(self, dtype):
        p = L.ConvParams()
        p.dtype = dtype
        p.nimg, p.hin, p.win, p.cin = self.nimg, self.hin, self.win, self.cin
        p.hout, p.wout, p.cout = self.hout, self.wout, self.cout
        p.kh, p.kw, p.sh, p.sw, p.ph, p.pw = self.kh, self.kw, self.sh, self.sw, self.ph, self.pw
        p.groups, p.ldx, p.ldy = self.groups, self.ldx, self.ldy
        p.alpha, p.beta = 1.0, 0.0
        return p

    @property
    def out_pixels(self):
        return self.nimg * self.hout * self.wout

    @property
    def in_pixels(self):
        return self.nimg * self.hin * self.win


def conv_stat_tiles(g, dtype):
    """output row tiles of conv_fwd(g, x of dtype code `dtype`, ..., stats): the tile height (hence
    the partial-statistics count) depends on the path the dtype takes"""
    p = g.params(dtype)
    return L.load().avsr_conv_stat_tiles(ctypes.byref(p))


def conv_fwd(g, x, w, y, stats=None, bias=None, act=L.ACT_NONE, preact=None, res=None):
    """y[pix, co] = act(conv(x, w) + bias) + res; stats: fp32 [cout, tiles, 3] BN partials."""
    p = g.params(dtype_code(x))
    assert x.dtype == w.dtype == y.dtype and x.is_cuda
    if stats is not None:
        # the kernel writes one (count, mean, M2) per output row tile of the launched tile height
        tiles = L.load().avsr_conv_stat_tiles(ctypes.byref(p))
        if stats.dtype != torch.float32 or stats.numel() < g.groups * g.cout * tiles * 3 or not stats.is_contiguous():
            raise ValueError(f"conv_fwd stats: need fp32 [{g.cout}, {tiles}, 3], got {tuple(stats.shape)}")
    p.x, p.w, p.y = x.data_ptr(), w.data_ptr(), y.data_ptr()
    p.stats = None if stats is None else stats.data_ptr()
    p.bias = None if bias is None else bias.data_ptr()
    p.act = act
    p.preact = None if preact is None else preact.data_ptr()
    p.res = None if res is None else res.data_ptr()
    p._keep = [t for t in (x, w, y, stats, bias, preact, res) if t is not None]
    L.check(L.load().avsr_conv_fwd(ctypes.byref(p), L.stream_ptr()), "avsr_conv_fwd")
    return y


def conv_bwd_data(g, dy, w, dx, alpha=1.0, beta=0.0):
    p = g.params(dtype_code(dy))
    assert dy.dtype == w.dtype == dx.dtype
    p.dy, p.w, p.dx = dy.data_ptr(), w.data_ptr(), dx.data_ptr()
    p.alpha, p.beta = alpha, beta
    L.check(L.load().avsr_conv_bwd_data(ctypes.byref(p), L.stream_ptr()), "avsr_conv_bwd_data")
    return dx


def bn_fin_ws(tiles, C):
    """floats of a BN-backward partials workspace (AVSR_BN_FIN_WS)"""
    return (tiles + ((tiles + 15) // 16 if tiles > 256 else 0)) * 4 * C


def conv_bwd_data_bnr(g, dy, w, dx, h, st, prelu, *, res=None, st2=None, alpha=1.0, beta=0.0):
    """data-grad whose epilogue runs the BatchNorm+PReLU backward reduction of the layer that
    produced the conv input: dx <- dz = prelu'(z) * (alpha*conv^T(dy) + beta*dx); returns the
    partial sums (ws, tiles) for bn_bwd_finalize (bf16 only)."""
    p = g.params(dtype_code(dy))
    assert dy.dtype == w.dtype == dx.dtype == h.dtype == torch.bfloat16
    lib = L.load()
    tiles = lib.avsr_conv_bnr_tiles(ctypes.byref(p))
    ws = torch.empty(bn_fin_ws(tiles, g.cin), device=dx.device)
    p.dy, p.w, p.dx = dy.data_ptr(), w.data_ptr(), dx.data_ptr()
    p.alpha, p.beta = alpha, beta
    p.bnr_h, p.bnr_res = h.data_ptr(), None if res is None else res.data_ptr()
    p.bnr_scale, p.bnr_shift, p.bnr_prelu = st.scale.data_ptr(), st.shift.data_ptr(), prelu.data_ptr()
    p.bnr_mean, p.bnr_invstd = st.mean.data_ptr(), st.invstd.data_ptr()
    if st2 is not None:
        p.bnr_scale2, p.bnr_shift2 = st2.scale.data_ptr(), st2.shift.data_ptr()
        p.bnr_mean2, p.bnr_invstd2 = st2.mean.data_ptr(), st2.invstd.data_ptr()
    p.bnr_ws = ws.data_ptr()
    L.check(lib.avsr_conv_bwd_data(ctypes.byref(p), L.stream_ptr()), "avsr_conv_bwd_data(bnr)")
    return ws, tiles


_WGRAD_SLAB = True      # conv weight-grad split-K through slabs (deterministic; fp32 atomics only by request)


def conv_bwd_weight(g, x, dy, dw, splitk=0, slab=None):
    """dw (fp32, [groups*cout, kh, kw, cin]) += wgrad(x, dy). The split-K partials go to an
    fp32 slab workspace from the caching allocator (slab=False: fp32 atomics instead)."""
    p = g.params(dtype_code(x))
    assert x.dtype == dy.dtype and dw.dtype == torch.float32
    p.x, p.dy, p.dw = x.data_ptr(), dy.data_ptr(), dw.data_ptr()
    p.splitk = splitk
    lib = L.load()
    ws = None
    if _WGRAD_SLAB if slab is None else slab:
        n = lib.avsr_conv_wgrad_ws(ctypes.byref(p))
        if n > 0:
            ws = torch.empty(n, device=dw.device, dtype=torch.float32)
            p.ws = ws.data_ptr()
    L.check(lib.avsr_conv_bwd_weight(ctypes.byref(p), L.stream_ptr()), "avsr_conv_bwd_weight")
    return dw


def _call(name, params):
    L.check(getattr(L.load(), name)(ctypes.byref(params), L.stream_ptr()), name)


# ---------------------------------------------------------------------------------------
# LayerNorm
# ---------------------------------------------------------------------------------------

def layernorm_fwd(x, gamma, beta, eps, y=None, mean=None, rstd=None):
    rows, N = x.shape
    y = torch.empty_like(x) if y is None else y
    mean = torch.empty(rows, device=x.device) if mean is None else mean
    rstd = torch.empty(rows, device=x.device) if rstd is None else rstd
    _call("avsr_layernorm_fwd", L.fill(L.LayerNormParams, dtype=dtype_code(x), rows=rows, N=N, eps=eps,
                                        x=x, ldx=x.stride(0), y=y, ldy=y.stride(0), gamma=gamma, beta=beta,
                                        mean=mean, rstd=rstd))
    return y, mean, rstd


def layernorm_bwd(dy, x, gamma, mean, rstd, dx=None, dres=None, dgamma=None, dbeta=None, g=None, drop_p=0.0, seed=0,
                  db=None):
    """dx = dres + LN-backward(dy); dgamma/dbeta (fp32) accumulate. With g: the following
    ew_bwd(dx, out=g, drop_p, seed, db) fused in (g = dropout-backward of dx as stored,
    db += column sums of g)."""
    rows, N = x.shape
    dx = torch.empty_like(x) if dx is None else dx
    if db is not None:
        assert g is not None and dgamma is not None
    ws = None if dgamma is None else _colsum_ws(256 * (3 if db is not None else 2) * N, x.device)   # AVSR_LN_WS(3)
    _call("avsr_layernorm_bwd", L.fill(L.LayerNormParams, dtype=dtype_code(x), rows=rows, N=N, eps=0.0,
                                        x=x, ldx=x.stride(0), ldy=N, gamma=gamma, mean=mean, rstd=rstd,
                                        dy=dy, lddy=dy.stride(0), dx=dx, lddx=dx.stride(0),
                                        dres=dres, lddres=0 if dres is None else dres.stride(0),
                                        dgamma=dgamma, dbeta=dbeta, ws=ws, g=g, ldg=0 if g is None else g.stride(0),
                                        drop_p=float(drop_p), seed=int(seed) & (2 ** 64 - 1), db=db))
    return dx


# ---------------------------------------------------------------------------------------
# BatchNorm (+PReLU, +residual) over NHWC rows
# ---------------------------------------------------------------------------------------

class BnState:
    """Per-step statistics of one BatchNorm: mean / invstd / folded scale / shift (fp32 [C])."""

    def __init__(self, C, device):
        buf = torch.empty(4, C, device=device)
        self.mean, self.invstd, self.scale, self.shift = buf[0], buf[1], buf[2], buf[3]


def bn_finalize(st, gamma, beta, running_mean, running_var, *, partials=None, training=True,
                momentum=0.1, eps=1e-5):
    C = gamma.shape[0]
    tiles = 0 if partials is None else partials.shape[1]
    _call("avsr_bn_finalize", L.fill(L.BnFinalizeParams, tiles=tiles, C=C, partials=partials, gamma=gamma,
                                      beta=beta, running_mean=running_mean, running_var=running_var,
                                      momentum=momentum, eps=eps, training=int(training), mean=st.mean,
                                      invstd=st.invstd, scale=st.scale, shift=st.shift))
    return st


def bn_act_fwd(h, st, prelu, y, res=None, st2=None):
    M, C = h.shape
    _call("avsr_bn_act_fwd", L.fill(L.BnActParams, dtype=dtype_code(h), M=M, C=C, h=h, scale=st.scale,
                                     shift=st.shift, res=res, scale2=None if st2 is None else st2.scale,
                                     shift2=None if st2 is None else st2.shift, prelu=prelu, y=y))
    return y


def _bn_params(h, st, *, M=None, res=None, st2=None, **kw):
    M = h.shape[0] if M is None else M
    C = h.shape[-1]
    return L.fill(L.BnActParams, dtype=dtype_code(h), M=M, C=C, h=h, scale=st.scale, shift=st.shift, res=res,
                  scale2=None if st2 is None else st2.scale, shift2=None if st2 is None else st2.shift,
                  mean=st.mean, invstd=st.invstd, mean2=None if st2 is None else st2.mean,
                  invstd2=None if st2 is None else st2.invstd, **kw)


def bn_act_bwd_reduce(dy, h, st, prelu, *, res=None, st2=None, dz=None, sums=None, dprelu=None, dgamma=None,
                      dbeta=None, dgamma2=None, dbeta2=None):
    """dz = prelu'(z) * dy (z recomputed) and the BN sums [C][3]; accumulates the PReLU / BN
    parameter gradients. Returns (dz, sums)."""
    C = h.shape[-1]
    dz = torch.empty_like(h) if dz is None else dz
    sums = torch.empty(C, 3, device=h.device) if sums is None else sums
    ws = torch.empty(bn_fin_ws(2048, C), device=h.device)
    _call("avsr_bn_act_bwd_reduce", _bn_params(h, st, res=res, st2=st2, ws=ws, prelu=prelu, dy=dy, dz=dz, sums=sums,
                                               dprelu=dprelu, dgamma=dgamma, dbeta=dbeta, dgamma2=dgamma2,
                                               dbeta2=dbeta2))
    return dz, sums


def bn_bwd_finalize(ws, tiles, C, *, sums=None, dprelu=None, dgamma=None, dbeta=None, dgamma2=None, dbeta2=None):
    """sums [C][3] + parameter gradients from the partials of a data-grad BN epilogue."""
    sums = torch.empty(C, 3, device=ws.device) if sums is None else sums
    p = L.fill(L.BnActParams, C=C, ws=ws, sums=sums, dprelu=dprelu, dgamma=dgamma, dbeta=dbeta, dgamma2=dgamma2,
               dbeta2=dbeta2)
    L.check(L.load().avsr_bn_bwd_finalize(ctypes.byref(p), tiles, L.stream_ptr()), "avsr_bn_bwd_finalize")
    return sums


def bn_bwd_apply(dz, h, st, sums, dh, *, res=None, st2=None, dh2=None, beta_acc=0.0):
    """dh = scale*(dz - S0/M - xhat*S1/M) (+ beta_acc*dh); dh2 likewise for the downsample BN."""
    _call("avsr_bn_bwd_apply", _bn_params(h, st, res=res, st2=st2, dz=dz, sums=sums, dh=dh, dh2=dh2,
                                          beta_acc=beta_acc))
    return dh


def bn_act_bwd(dy, h, st, prelu, dh, *, res=None, st2=None, dh2=None, dz=None, sums=None,
               dprelu=None, dgamma=None, dbeta=None, dgamma2=None, dbeta2=None, beta_acc=0.0):
    """Backward of y = prelu(bn(h) + [bn2(res) | res]): returns dz (grad of the residual
    input when identity) and writes dh (and dh2 for the downsample BN)."""
    dz, sums = bn_act_bwd_reduce(dy, h, st, prelu, res=res, st2=st2, dz=dz, sums=sums, dprelu=dprelu,
                                 dgamma=dgamma, dbeta=dbeta, dgamma2=dgamma2, dbeta2=dbeta2)
    bn_bwd_apply(dz, h, st, sums, dh, res=res, st2=st2, dh2=dh2, beta_acc=beta_acc)
    return dz


def stem_pool_fwd(h, nimg, H, W, st, prelu, y, argmax, hmax=None):
    """y = maxpool3x3s2(prelu(bn(h))) with the argmax window index and (hmax) h at the argmax"""
    C = h.shape[-1]
    _call("avsr_stem_pool_fwd", L.fill(L.StemPoolParams, dtype=dtype_code(h), nimg=nimg, H=H, W=W, C=C,
                                        Ho=(H + 1) // 2, Wo=(W + 1) // 2, h=h, scale=st.scale, shift=st.shift,
                                        prelu=prelu, y=y, argmax=argmax, hmax=hmax))
    return y


def stem_pool_bwd(dy, argmax, hmax, h, nimg, H, W, st, prelu, dh, *, dzp=None, sums=None, dprelu=None,
                  dgamma=None, dbeta=None, reduced=None):
    """Backward through max-pool, PReLU and BN of the stem: writes dh (grad of the conv output).
    The BN/PReLU reduction runs on the pooled grid (h = hmax); `reduced` = (ws, tiles) when a
    data-grad BN epilogue already stored the pooled dz in dy and wrote the partials."""
    dzp, sums = stem_pool_bwd_reduce(dy, hmax, nimg, H, W, st, prelu, dzp=dzp, sums=sums, dprelu=dprelu,
                                     dgamma=dgamma, dbeta=dbeta, reduced=reduced)
    return stem_pool_bwd_apply(dzp, argmax, h, nimg, H, W, st, sums, dh)


def stem_pool_bwd_reduce(dy, hmax, nimg, H, W, st, prelu, *, dzp=None, sums=None, dprelu=None, dgamma=None,
                         dbeta=None, reduced=None):
    """the stem's BN/PReLU backward reduction over the pooled grid: (pooled dz, sums)"""
    C = hmax.shape[-1]
    Mo = nimg * ((H + 1) // 2) * ((W + 1) // 2)
    if reduced is None:
        return bn_act_bwd_reduce(dy.view(Mo, C), hmax.view(Mo, C), st, prelu, dz=dzp, sums=sums,
                                 dprelu=dprelu, dgamma=dgamma, dbeta=dbeta)
    return dy, bn_bwd_finalize(reduced[0], reduced[1], C, sums=sums, dprelu=dprelu, dgamma=dgamma, dbeta=dbeta)


def stem_pool_bwd_apply(dzp, argmax, h, nimg, H, W, st, sums, dh, m_total=0):
    """dh of `nimg` images from their pooled dz / argmax (views starting at the first of them);
    m_total: the pixel count the BN statistics cover when this is a range of the batch"""
    C = h.shape[-1]
    _call("avsr_stem_pool_bwd_apply", L.fill(L.StemPoolParams, dtype=dtype_code(h), nimg=nimg, H=H, W=W, C=C,
                                              Ho=(H + 1) // 2, Wo=(W + 1) // 2, h=h, scale=st.scale, argmax=argmax,
                                              dz=dzp, mean=st.mean, invstd=st.invstd, sums=sums, dh=dh,
                                              m_total=int(m_total)))
    return dh


def avgpool_fwd(x, nimg, P, C, y):
    L.check(L.load().avsr_avgpool_fwd(dtype_code(x), nimg, P, C, x.data_ptr(), y.data_ptr(), L.stream_ptr()),
            "avsr_avgpool_fwd")
    return y


def avgpool_bwd(dy, nimg, P, C, dx):
    L.check(L.load().avsr_avgpool_bwd(dtype_code(dy), nimg, P, C, dy.data_ptr(), dx.data_ptr(), L.stream_ptr()),
            "avsr_avgpool_bwd")
    return dx


# ---------------------------------------------------------------------------------------
# Fused attention (head dim 64). q/k/v/o are 2-D row views (rows = batch*len, head h at
# columns h*64..h*64+63); they may be column slices of a fused QKV buffer.
# ---------------------------------------------------------------------------------------

def _attn_params(q, k, v, o, B, H, Lq, Lk, lse, klen, causal, scale, drop_p, seed):
    return L.fill(L.AttnParams, dtype=dtype_code(q), B=B, H=H, Lq=Lq, Lk=Lk, scale=scale,
                  q=q, ldq=q.stride(0), k=k, ldk=k.stride(0), v=v, ldv=v.stride(0), o=o, ldo=o.stride(0),
                  lse=lse, klen=klen, causal=int(causal), drop_p=float(drop_p), seed=int(seed) & (2 ** 64 - 1))


def attn_mask_words(B, H, Lq, Lk):
    """AVSR_ATTN_MASK_WORDS: 64-bit words of one attention call's stored dropout keep mask"""
    return B * H * ((Lq + 31) // 32) * (2 * ((Lk + 63) // 64)) * 16


def attn_dropmask(mask, *, B, H, Lq, Lk, drop_p, seed):
    """the keep decisions of the attention dropout (drop_p, seed) for (B, H, Lq, Lk) into mask
    (int64, attn_mask_words(...) elements); data-independent, so it may run on any stream ahead
    of the forward. Pass the same mask to attn_fwd / attn_bwd."""
    assert mask.dtype == torch.int64 and mask.is_contiguous() and mask.numel() >= attn_mask_words(B, H, Lq, Lk)
    p = L.fill(L.AttnParams, dtype=L.AVSR_BF16, B=B, H=H, Lq=Lq, Lk=Lk, drop_p=float(drop_p),
               seed=int(seed) & (2 ** 64 - 1), drop_mask=mask)
    _call("avsr_attn_dropmask", p)
    return mask


def attn_fwd(q, k, v, o, lse, *, B, H, Lq, Lk, klen=None, causal=False, scale=0.125, drop_p=0.0, seed=0, mask=None):
    """mask: a keep mask from attn_dropmask for the same (B, H, Lq, Lk, drop_p, seed), or None
    (the kernels hash the dropout per element; same result)"""
    p = _attn_params(q, k, v, o, B, H, Lq, Lk, lse, klen, causal, scale, drop_p, seed)
    if mask is not None:
        p.drop_mask = mask.data_ptr()
    _call("avsr_attn_fwd", p)
    return o


def attn_bwd(dout, q, k, v, o, lse, dq32, dk, dv, delta, *, B, H, Lq, Lk, klen=None, causal=False,
             scale=0.125, drop_p=0.0, seed=0, dq=None, db=None, mask=None):
    """dq32: fp32 accumulator (zeroed by the caller), or None with dq (bf16 only): dQ written
    straight into dq in the activation dtype. dk/dv in the activation dtype. db (fp32, 3*H*64):
    += the column sums of the stored dQ | dK | dV (the fused q/k/v bias gradients), finalised
    through the column-sum path (deferred within a training step's backward). mask: as attn_fwd."""
    p = _attn_params(q, k, v, o, B, H, Lq, Lk, lse, klen, causal, scale, drop_p, seed)
    if mask is not None:
        p.drop_mask = mask.data_ptr()
    p.dout, p.lddo = dout.data_ptr(), dout.stride(0)
    p.delta = delta.data_ptr()
    if dq is not None:
        assert q.dtype == torch.bfloat16 and dq.dtype == torch.bfloat16, "dq output path is bf16 only"
        p.dq_out, p.lddq_out = dq.data_ptr(), dq.stride(0)
    else:
        p.dq, p.lddq = dq32.data_ptr(), dq32.stride(0)
    p.dk, p.lddk = dk.data_ptr(), dk.stride(0)
    p.dv, p.lddv = dv.data_ptr(), dv.stride(0)
    ws = None
    if db is not None:
        assert db.dtype == torch.float32 and db.is_contiguous() and db.numel() == 3 * H * 64
        ws = _colsum_ws(B * 3 * H * 64, dk.device)                  # AVSR_ATTN_DB_WS(B, H)
        p.db, p.db_ws = db.data_ptr(), ws.data_ptr()
    _call("avsr_attn_bwd_prep", p)
    _call("avsr_attn_bwd", p)


# ---------------------------------------------------------------------------------------
# Losses
# ---------------------------------------------------------------------------------------

def _p(t):
    return None if t is None else t.data_ptr()


def row_lse(x, V, lse):
    _call("avsr_row_lse", L.fill(L.XentParams, dtype=dtype_code(x), rows=x.shape[0], V=V, x=x,
                                  ldx=x.stride(0), lse=lse))
    return lse


def lsm_fwd(x, V, target, smoothing, lse, row_loss, row_correct):
    _call("avsr_lsm_fwd", L.fill(L.XentParams, dtype=dtype_code(x), rows=x.shape[0], V=V, x=x, ldx=x.stride(0),
                                  target=target, smoothing=smoothing, lse=lse, row_loss=row_loss,
                                  row_correct=row_correct))


def lsm_bwd(x, V, target, smoothing, lse, dloss, coef, dx):
    _call("avsr_lsm_bwd", L.fill(L.XentParams, dtype=dtype_code(x), rows=x.shape[0], V=V, x=x, ldx=x.stride(0),
                                  target=target, smoothing=smoothing, lse=lse, dloss=dloss, coef=coef,
                                  dx=dx, lddx=dx.stride(0)))
    return dx


def ctc_params(x, B, T, V, labels, label_len, in_len, lse, alpha, gamma, nll):
    return L.fill(L.CtcParams, dtype=dtype_code(x), B=B, T=T, V=V, Lmax=labels.shape[1], x=x, ldx=x.stride(0),
                  lse=lse, labels=labels, label_len=label_len, in_len=in_len, alpha=alpha, gamma=gamma, nll=nll)


def ctc_fwd(p):
    _call("avsr_ctc_fwd", p)


def ctc_bwd(p, dloss, coef, dx):
    p.dloss, p.coef, p.dx, p.lddx = dloss.data_ptr(), coef, dx.data_ptr(), dx.stride(0)
    _call("avsr_ctc_bwd", p)
    return dx


def loss_finalize(B, nll, row_loss, row_correct, mtlalpha, out, att_per_token=False):
    """att_per_token: the attention loss divides by the number of target tokens
    (transformer_length_normalized_loss) instead of B"""
    L.check(L.load().avsr_loss_finalize(B, nll.data_ptr(), row_loss.shape[0], row_loss.data_ptr(),
                                        _p(row_correct), mtlalpha, int(bool(att_per_token)), out.data_ptr(),
                                        L.stream_ptr()),
            "avsr_loss_finalize")
    return out


# ---------------------------------------------------------------------------------------
# Elementwise / data movement
# ---------------------------------------------------------------------------------------

# deferred column-sum finalisation (avsr_colsum_defer / avsr_colsum_flush): the partial
# workspaces of the queued passes stay referenced here until the flush has been enqueued
_COLSUM = {"on": False, "keep": []}


def _colsum_ws(n, device):
    ws = torch.empty(n, device=device)
    if _COLSUM["on"]:
        _COLSUM["keep"].append(ws)
    return ws


def colsum_defer(on):
    """queue (True) or run at once (False) the finalise passes of bias / LayerNorm parameter
    gradients; returns the previous setting"""
    prev = _COLSUM["on"]
    L.load().avsr_colsum_defer(int(bool(on)))
    _COLSUM["on"] = bool(on)
    if not on:      # the C side drops passes still queued (an aborted step): so do we
        _COLSUM["keep"].clear()
    return prev


def colsum_flush():
    """one batched launch for every queued finalise pass (current stream)"""
    if _COLSUM["on"] or _COLSUM["keep"]:
        L.check(L.load().avsr_colsum_flush(L.stream_ptr()), "avsr_colsum_flush")
        _COLSUM["keep"].clear()


def ew_bwd(dy, *, out=None, gate=None, act=L.ACT_NONE, drop_p=0.0, seed=0, alpha=1.0, db=None, inline=False):
    """elementwise backward (dropout / activation gate) and/or bias gradient db += alpha * column
    sums; inline=True finalises the column sums at once on the current stream even while the
    finalise passes are deferred (a bias gradient issued on the weight-grad side stream)"""
    rows, N = dy.shape
    lib = L.load()
    if inline and db is not None:
        ws = torch.empty(256 * N, device=dy.device)       # consumed by the inline finalise
        prev = lib.avsr_colsum_inline(1)
    else:
        ws = None if db is None else _colsum_ws(256 * N, dy.device)   # AVSR_EW_WS
    try:
        _call("avsr_ew_bwd", L.fill(L.EwParams, dtype=dtype_code(dy), rows=rows, N=N, dy=dy, lddy=dy.stride(0),
                                     ws=ws, out=out, ldout=0 if out is None else out.stride(0), gate=gate,
                                     ldgate=0 if gate is None else gate.stride(0), act=act, drop_p=float(drop_p),
                                     seed=int(seed) & (2 ** 64 - 1), alpha=alpha, db=db))
    finally:
        if inline and db is not None:
            lib.avsr_colsum_inline(prev)
    return out


def dropout_fwd(x, out, p, seed):
    rows, N = x.shape
    _call("avsr_dropout_fwd", L.fill(L.EwParams, dtype=dtype_code(x), rows=rows, N=N, dy=x, lddy=x.stride(0),
                                      out=out, ldout=out.stride(0), drop_p=float(p),
                                      seed=int(seed) & (2 ** 64 - 1), alpha=1.0))
    return out


def mask_rows(x, B, T, lengths):
    L.check(L.load().avsr_mask_rows(dtype_code(x), B, T, x.shape[1], x.data_ptr(), x.stride(0),
                                    lengths.data_ptr(), L.stream_ptr()), "avsr_mask_rows")
    return x


def embed_fwd(tok, table, pe, scale, y, L_, drop_p=0.0, seed=0, pe_row=None):
    """pe_row: optional device int32 [1]: every row adds pe[pe_row[0]] (a beam-search step's
    position kept on the device)"""
    _call("avsr_embed_fwd", L.fill(L.EmbedParams, dtype=dtype_code(table), rows=tok.shape[0], L=L_,
                                    D=table.shape[1], tok=tok, table=table, pe=pe, scale=scale, y=y,
                                    drop_p=float(drop_p), seed=int(seed) & (2 ** 64 - 1), pe_row=pe_row))
    return y


def embed_bwd(tok, dy, scale, dtable, L_, drop_p=0.0, seed=0):
    _call("avsr_embed_bwd", L.fill(L.EmbedParams, dtype=dtype_code(dy), rows=tok.shape[0], L=L_,
                                    D=dy.shape[1], tok=tok, scale=scale, dy=dy, dtable=dtable,
                                    drop_p=float(drop_p), seed=int(seed) & (2 ** 64 - 1)))


def cast(src, dst, alpha=1.0, beta=0.0):
    rows, cols = src.shape
    assert dst.shape == src.shape
    L.check(L.load().avsr_cast(dtype_code(src), dtype_code(dst), rows, cols, src.data_ptr(), src.stride(0),
                               dst.data_ptr(), dst.stride(0), alpha, beta, L.stream_ptr()), "avsr_cast")
    return dst


def cast_flat(src, dst):
    """dst = src over two contiguous buffers of the same length (any dtype pair)."""
    assert src.is_contiguous() and dst.is_contiguous() and src.numel() == dst.numel()
    L.check(L.load().avsr_cast_flat(dtype_code(src), dtype_code(dst), src.numel(), src.data_ptr(), dst.data_ptr(),
                                    L.stream_ptr()), "avsr_cast_flat")
    return dst


def stem_pack(videos, out):
    B, _, T = videos.shape[:3]
    assert videos.dtype == torch.float32 and videos.is_contiguous()
    L.check(L.load().avsr_stem_pack(dtype_code(out), B, T, videos.data_ptr(), out.data_ptr(), L.stream_ptr()),
            "avsr_stem_pack")
    return out


def stem_wpack(w, wp):
    L.check(L.load().avsr_stem_wpack(dtype_code(wp), w.data_ptr(), wp.data_ptr(), L.stream_ptr()), "avsr_stem_wpack")
    return wp


STEM_K = 288     # packed stem weight row (avsr_stem_wpack2)
STEM_DIRECT_MAX_BYTES = 0x7fffffff   # avsr_stem_conv_fwd: fp32 video bytes must stay below this


def stem_wpack2(w, wk):
    """Conv3d stem weight (64,1,5,7,7) fp32 -> [64][288] bf16 (k = (dt*7 + kh)*8 + kw)"""
    assert w.dtype == torch.float32 and w.numel() == 64 * 245 and w.is_contiguous()
    assert wk.dtype == torch.bfloat16 and wk.numel() == 64 * STEM_K
    L.check(L.load().avsr_stem_wpack2(w.data_ptr(), wk.data_ptr(), L.stream_ptr()), "avsr_stem_wpack2")
    return wk


def stem_conv_tiles(B, T):
    """BN partial-statistics tiles of stem_conv_fwd (one per persistent block)"""
    return L.load().avsr_stem_conv_tiles(int(B), int(T))


def stem_conv_fwd(videos, wk, h, stats=None):
    """stem Conv3d straight from the videos (B,1,T,88,88) fp32 -> h [B*T*44*44][64] bf16 (+ BN
    partial statistics [64][stem_conv_tiles(B*T)][3])"""
    B, _, T = videos.shape[:3]
    assert videos.dtype == torch.float32 and videos.is_contiguous() and tuple(videos.shape[3:]) == (88, 88)
    assert h.dtype == torch.bfloat16 and h.numel() == B * T * 44 * 44 * 64 and h.is_contiguous()
    if stats is not None:
        assert stats.dtype == torch.float32 and stats.numel() >= 64 * stem_conv_tiles(B, T) * 3
    L.check(L.load().avsr_stem_conv_fwd(B, T, videos.data_ptr(), wk.data_ptr(), h.data_ptr(),
                                        None if stats is None else stats.data_ptr(), L.stream_ptr()),
            "avsr_stem_conv_fwd")
    return h


def stem_wgrad_unpack(gp, gw):
    L.check(L.load().avsr_stem_wgrad_unpack(gp.data_ptr(), gw.data_ptr(), L.stream_ptr()), "avsr_stem_wgrad_unpack")


def audio_pack(audios, out):
    B, F, T = audios.shape
    assert audios.dtype == torch.float32 and audios.is_contiguous()
    L.check(L.load().avsr_audio_pack(dtype_code(out), B, F, T, audios.data_ptr(), out.data_ptr(), L.stream_ptr()),
            "avsr_audio_pack")
    return out


def weightnorm_fwd(v, g, norm, w):
    O, K, C = v.shape
    L.check(L.load().avsr_weightnorm_fwd(dtype_code(w), O, K, C, v.data_ptr(), g.data_ptr(), norm.data_ptr(),
                                         w.data_ptr(), L.stream_ptr()), "avsr_weightnorm_fwd")


def weightnorm_bwd(v, g, norm, dw, dv, dg, scratch):
    O, K, C = v.shape
    L.check(L.load().avsr_weightnorm_bwd(O, K, C, v.data_ptr(), g.data_ptr(), norm.data_ptr(), dw.data_ptr(),
                                         dv.data_ptr(), dg.data_ptr(), scratch.data_ptr(), L.stream_ptr()),
            "avsr_weightnorm_bwd")


SUMSQ_WS = 1024   # AVSR_SUMSQ_WS


def sumsq(x, out, ws=None):
    """out += sum(x^2) in a fixed summation order (two passes through ws, no atomics)"""
    if ws is None:
        ws = torch.empty(SUMSQ_WS, device=x.device)
    assert ws.dtype == torch.float32 and ws.numel() >= SUMSQ_WS
    L.check(L.load().avsr_sumsq(x.data_ptr(), x.numel(), out.data_ptr(), ws.data_ptr(), L.stream_ptr()),
            "avsr_sumsq")
    return out


def adamw(param, grad, exp_avg, exp_avg_sq, *, lr, beta1, beta2, eps, weight_decay, step, shadow=None,
          sumsq_buf=None, max_norm=1.0, grad_scale=1.0, max_blocks=0, clear_grad=False):
    _call("avsr_adamw", L.fill(L.AdamWParams, n=param.numel(), param=param, grad=grad, exp_avg=exp_avg,
                                exp_avg_sq=exp_avg_sq, shadow=shadow,
                                shadow_dtype=L.AVSR_BF16 if shadow is None else dtype_code(shadow),
                                lr=lr, beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay,
                                bias_corr1=1 - beta1 ** step, bias_corr2=1 - beta2 ** step,
                                sumsq=sumsq_buf, max_norm=max_norm, grad_scale=grad_scale, max_blocks=max_blocks,
                                grad_clear=grad if clear_grad else None))


# ---------------------------------------------------------------------------------------
# Beam-search decode (decode.hip)
# ---------------------------------------------------------------------------------------

def log_softmax_rows(x, V, out):
    L.check(L.load().avsr_log_softmax_rows(dtype_code(x), x.shape[0], V, x.data_ptr(), x.stride(0), out.data_ptr(),
                                           out.stride(0), L.stream_ptr()), "avsr_log_softmax_rows")
    return out


_DA_WS = {}
DA_WAVES = 8               # waves per dec_attn workgroup (decode.hip)


def dec_attn_group_fits(klen_max, group):
    """the grouped dec_attn keeps [group][klen_max rounded to 4] scores plus [8][group][64]
    partials in 64 KiB of LDS (decode.hip avsr_dec_attn); beyond that the kernel refuses"""
    kpad = (int(klen_max) + 3) & ~3
    return (group * kpad + DA_WAVES * group * 64) * 4 <= 64 * 1024


def dec_attn_ws_floats(n, H, group, ksplit):
    """fp32 partials the key-split dec_attn needs for n hypotheses in runs of `group`"""
    G = max(1, group)
    return (n + G - 1) // G * H * ksplit * G * 66 if ksplit > 1 else 0


def dec_attn(q, k, v, o, *, n, H, klen_max, k_bstride, v_bstride, klen=None, scale=0.125, kidx=None, kmap=None,
             group=1, ksplit=1):
    """one query per hypothesis: q/o rows i (ld = stride(0)), keys j of hypothesis i at
    k[b*k_bstride + j*k.stride(-2)] with b = kidx[i] (kidx None: b = i; bstride 0: shared keys);
    kmap (int32 [n][ldmap]): key j of hypothesis i is row kmap[i][j] of k instead; group: runs of
    `group` hypotheses share their key block and klen (one read of each row for all of them);
    ksplit: up to ksplit workgroups per (group, head) over the keys, merged by the last to arrive
    (per-stream partial buffer; the arrival counters of the few-row GEMM workspace)."""
    ws = cnt = None
    if group > 1 and not dec_attn_group_fits(klen_max, group):
        group = 1          # the grouped kernel's [group][klen] scores would not fit its 64 KiB of LDS
    if ksplit > 1:
        G = max(1, group)
        slots = (n + G - 1) // G * H
        assert slots <= SKINNY_CNT
        key = (_norm_dev(q.device), L.stream_ptr().value)
        need = dec_attn_ws_floats(n, H, group, ksplit)
        ws = _DA_WS.get(key)
        if ws is None or ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise L.AvsrLibError("dec_attn workspace first sized inside a graph capture: call "
                                     "ops.reserve_stream_workspaces() on the capture stream before capturing")
            ws = _DA_WS[key] = torch.empty(need, device=q.device, dtype=torch.float32)
        cnt = _skinny_ws(q.device)[SKINNY_WS:]
    _call("avsr_dec_attn", L.fill(L.DecAttnParams, dtype=dtype_code(q), n=n, H=H, klen_max=klen_max, scale=scale,
                                   q=q, ldq=q.stride(0), k=k, ldk=k.stride(-2), k_bstride=k_bstride, v=v,
                                   ldv=v.stride(-2), v_bstride=v_bstride, klen=klen, o=o, ldo=o.stride(0),
                                   kidx=kidx, kmap=kmap, ldmap=0 if kmap is None else kmap.stride(0), group=group,
                                   ksplit=ksplit, ws=ws, cnt=cnt))
    return o


def row_topk(x, V, K, ids):
    _call("avsr_row_topk", L.fill(L.TopkParams, rows=x.shape[0], V=V, K=K, x=x, ldx=x.stride(0), ids=ids))
    return ids


def log_softmax_topk(x, V, out, K, ids):
    """log_softmax_rows(x, V, out) and row_topk(out, V, K, ids) in one pass (identical results)"""
    L.check(L.load().avsr_log_softmax_topk(dtype_code(x), x.shape[0], V, x.data_ptr(), x.stride(0), out.data_ptr(),
                                           out.stride(0), K, ids.data_ptr(), L.stream_ptr()),
            "avsr_log_softmax_topk")
    return out


def ctc_prefix(logp, r_prev, last, ids, r_new, psi, *, n, out_len, blank, eos, uidx=None, tlen=None,
               out_len_dev=None):
    """logp (T, V) of one utterance, or (U, Tmax, V) with uidx (per-hypothesis utterance) and
    tlen (per-utterance frames) for batched decoding; out_len_dev: device int32 [1] overriding
    out_len (graph-captured steps)"""
    T, V = logp.shape[-2:]
    _call("avsr_ctc_prefix", L.fill(L.CtcPrefixParams, n=n, T=T, V=V, P=ids.shape[1], blank=blank, eos=eos,
                                     out_len=out_len, logp=logp, r_prev=r_prev, last=last, ids=ids, r_new=r_new,
                                     psi=psi, uidx=uidx, logp_ustride=T * V if uidx is not None else 0,
                                     tlen=tlen, out_len_dev=out_len_dev))


def beam_select(dec, V, ids, psi, s_prev, score, out, *, n, beam, blank, eos, w_dec, w_ctc, seg=None):
    """out: dict of device tensors prev/tok/col (int32) and score/dec/ctc/s (fp32), [beam] —
    or, with seg (int32 [U+1] row offsets of U utterances), one selection per utterance into
    out[*][u*beam + r]"""
    _call("avsr_beam_select", L.fill(L.BeamSelectParams, n=n, V=V, P=ids.shape[1], beam=beam, blank=blank, eos=eos,
                                      w_dec=w_dec, w_ctc=w_ctc, dec=dec, ld=dec.stride(0), ids=ids, psi=psi,
                                      s_prev=s_prev, score=score, out_prev=out["prev"], out_tok=out["tok"],
                                      out_col=out["col"], out_score=out["score"], out_dec=out["dec"],
                                      out_ctc=out["ctc"], out_s=out["s"],
                                      nseg=0 if seg is None else seg.numel() - 1, seg=seg))


def gather_rows(src, dst, idx, *, groups, n, row_bytes, src_gstride, src_rstride, dst_gstride, dst_rstride):
    """dst[g][i] = src[g][idx[i]] (strides in bytes)"""
    L.check(L.load().avsr_gather_rows(groups, n, row_bytes, src.data_ptr(), src_gstride, src_rstride, dst.data_ptr(),
                                      dst_gstride, dst_rstride, idx.data_ptr(), L.stream_ptr()), "avsr_gather_rows")


def beam_step_prep(R, pos, anc, klen):
    """anc[r][pos] = pos*R + r, klen[r] = pos + 1 (pos: device int32 [1]); avsr_hip.h"""
    L.check(L.load().avsr_beam_step_prep(R, anc.shape[1], pos.data_ptr(), anc.data_ptr(), klen.data_ptr(),
                                         L.stream_ptr()), "avsr_beam_step_prep")


def beam_kv_put(qkv, cache_k, cache_v, pos, R, D):
    """this step's self-attention K / V rows -> cache rows pos*R + r"""
    L.check(L.load().avsr_beam_kv_put(dtype_code(qkv), R, D, qkv.data_ptr(), qkv.stride(0), cache_k.data_ptr(),
                                      cache_v.data_ptr(), pos.data_ptr(), L.stream_ptr()), "avsr_beam_kv_put")


def beam_post(**kw):
    """device-side bookkeeping after avsr_beam_select (avsr_hip.h avsr_beam_post)"""
    _call("avsr_beam_post", L.fill(L.BeamPostParams, **kw))
