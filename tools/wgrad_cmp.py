"""ResNet conv weight-grads at C2 (6000 images) vs a dense GEMM of the same M x N x K (both
operands r-contiguous, same split count): isolates the cost of the im2col B loader.
usage: python tools/wgrad_cmp.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from avsr_amd import ops, _lib as L  # noqa: E402

dev = torch.device("cuda")
NIMG = 6000
SHAPES = [  # hw_in, cin, cout, k, stride
    (22, 64, 64, 3, 1), (22, 64, 128, 3, 2), (11, 128, 128, 3, 1), (11, 128, 256, 3, 2),
    (6, 256, 256, 3, 1), (6, 256, 512, 3, 2), (3, 512, 512, 3, 1)]


def timed(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for hw, cin, cout, k, s in SHAPES:
    g = ops.ConvGeom(NIMG, hw, hw, cin, cout, k, k, stride=(s, s), pad=(k // 2, k // 2))
    x = torch.randn(g.in_pixels, cin, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(g.out_pixels, cout, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(cout, k, k, cin, device=dev)
    p = g.params(ops.dtype_code(x))
    M, N, K = cout, k * k * cin, g.out_pixels
    fl = 2.0 * M * N * K
    tc = timed(lambda: ops.conv_bwd_weight(g, x, dy, dw))
    # dense stand-in: B = [K][N] r-contiguous (an explicit im2col matrix of the same size)
    Bm = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    C = torch.zeros(M, N, device=dev)
    res = []
    for sk in (1, 2, 4, 8):
        ws = torch.empty(ops.slab_ws(1, sk, M, N), device=dev) if sk > 1 else None
        t = timed(lambda: ops.gemm(dy, Bm, C, M=M, N=N, K=K, a_kmajor=False, b_kmajor=False, lda=cout, ldb=N,
                                   ldc=N, beta=1.0, splitk=sk, ws=ws, ))
        res.append(f"sk{sk} {t:7.1f}us/{fl / t / 1e6:5.0f}")
    print(f"wgrad {hw}x{hw} {cin}->{cout} k{k} s{s} M{M} N{N} K{K}: conv {tc:7.1f}us/{fl / tc / 1e6:5.0f} TF/s | dense "
          + "  ".join(res), flush=True)
    del x, dy, dw, Bm, C
