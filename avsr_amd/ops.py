"""Thin tensor-level wrappers over the C-ABI (include/avsr_hip.h).

Each function validates shapes/dtypes on the host, then launches on the caller's current
stream. Nothing here computes on the CPU; a missing library raises (no fallback).
"""
import ctypes

import torch

from . import _lib as L

_DT = {torch.float32: L.AVSR_F32, torch.bfloat16: L.AVSR_BF16}


def dtype_code(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise L.AvsrLibError(f"unsupported dtype {t.dtype}")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def gemm(A, B, C, *, M, N, K, a_kmajor, b_kmajor, lda, ldb, ldc, batch=1,
         strideA=0, strideB=0, strideC=0, alpha=1.0, beta=0.0, bias=None, act=L.ACT_NONE,
         epi_bwd=False, preact=None, res=None, ldr=None, strideR=0, gate=None, drop_p=0.0, seed=0,
         splitk=1):
    """Raw GEMM launch: C[b,m,n] = epi(alpha * sum_k A(b,m,k) B(b,n,k)). See avsr_hip.h."""
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
    L.check(lib.avsr_gemm(ctypes.byref(p), L.stream_ptr()), "avsr_gemm")
    return C


# ---------------------------------------------------------------------------------------
# Linear layer building blocks (x: (M, K) row-major, W: (N, K) = torch.nn.Linear.weight)
# ---------------------------------------------------------------------------------------

def linear_fwd(x, W, bias=None, *, act=L.ACT_NONE, preact=None, res=None, drop_p=0.0, seed=0, out=None):
    """y = dropout(act(x W^T + b)) + res ; optionally stores h = x W^T + b into `preact`."""
    M, K = x.shape
    N = W.shape[0]
    assert W.shape[1] == K and x.stride(1) == 1 and W.stride(1) == 1
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    gemm(x, W, out, M=M, N=N, K=K, a_kmajor=True, b_kmajor=True, lda=x.stride(0), ldb=W.stride(0),
         ldc=out.stride(0), bias=bias, act=act, preact=preact, res=res,
         ldr=None if res is None else res.stride(0), drop_p=drop_p, seed=seed)
    return out


def linear_dgrad(dy, W, *, gate=None, act=L.ACT_NONE, drop_p=0.0, seed=0, out=None, beta=0.0):
    """dx = (dy W) [* dropout mask][* act'(gate)]  — gradient w.r.t. the layer input."""
    M, N = dy.shape
    K = W.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=dy.dtype)
    gemm(dy, W, out, M=M, N=K, K=N, a_kmajor=True, b_kmajor=False, lda=dy.stride(0), ldb=W.stride(0),
         ldc=out.stride(0), epi_bwd=True, gate=gate, act=act, drop_p=drop_p, seed=seed, beta=beta)
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


def conv_stat_tiles(g, dtype=L.AVSR_BF16):
    p = g.params(dtype)
    return L.load().avsr_conv_stat_tiles(ctypes.byref(p))


def conv_fwd(g, x, w, y, stats=None):
    """y[pix, co] = conv(x, w); stats: fp32 [tiles, cout, 3] BN partials (groups == 1)."""
    p = g.params(dtype_code(x))
    assert x.dtype == w.dtype == y.dtype and x.is_cuda
    p.x, p.w, p.y = x.data_ptr(), w.data_ptr(), y.data_ptr()
    p.stats = None if stats is None else stats.data_ptr()
    L.check(L.load().avsr_conv_fwd(ctypes.byref(p), L.stream_ptr()), "avsr_conv_fwd")
    return y


def conv_bwd_data(g, dy, w, dx, alpha=1.0, beta=0.0):
    p = g.params(dtype_code(dy))
    assert dy.dtype == w.dtype == dx.dtype
    p.dy, p.w, p.dx = dy.data_ptr(), w.data_ptr(), dx.data_ptr()
    p.alpha, p.beta = alpha, beta
    L.check(L.load().avsr_conv_bwd_data(ctypes.byref(p), L.stream_ptr()), "avsr_conv_bwd_data")
    return dx


def conv_bwd_weight(g, x, dy, dw, splitk=0):
    """dw (fp32, [groups*cout, kh, kw, cin]) += wgrad(x, dy)."""
    p = g.params(dtype_code(x))
    assert x.dtype == dy.dtype and dw.dtype == torch.float32
    p.x, p.dy, p.dw = x.data_ptr(), dy.data_ptr(), dw.data_ptr()
    p.splitk = splitk
    L.check(L.load().avsr_conv_bwd_weight(ctypes.byref(p), L.stream_ptr()), "avsr_conv_bwd_weight")
    return dw
