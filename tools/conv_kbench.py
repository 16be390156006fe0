"""Isolated ResNet-frontend kernels at C2 (6000 images), HIP-event timed, median of reps:
stem conv (general path: pack + 7x7 implicit GEMM, vs stem.hip straight from the video) and
the stage-1 3x3 convolutions (forward, fused BN-backward data-grad, weight-grad) with the
patch-resident kernel on / off. usage: python tools/conv_kbench.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import _lib as L, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
bf = torch.bfloat16
g = torch.Generator().manual_seed(0)
B, T = 16, 375
N = B * T


def timed(fn):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) * 1e3)
    return round(sorted(out)[len(out) // 2], 1)


res = {}
video = torch.randn(B, 1, T, 88, 88, generator=g).to(dev)
w5 = (torch.randn(64, 1, 5, 7, 7, generator=g) * 0.05).to(dev)
h0 = torch.empty(N * 44 * 44, 64, device=dev, dtype=bf)
xp = torch.empty(N, 88, 88, 8, device=dev, dtype=bf)
wp = torch.empty(64, 7, 7, 8, device=dev, dtype=bf)
gs = ops.ConvGeom(N, 88, 88, 8, 64, 7, 7, (2, 2), (3, 3))
part = torch.empty(64, ops.conv_stat_tiles(gs, ops.dtype_code(xp)), 3, device=dev)
ops.stem_wpack(w5, wp)


def stem_old():
    ops.stem_pack(video, xp)
    ops.conv_fwd(gs, xp, wp, h0, part)


wk = torch.empty(64, ops.STEM_K, device=dev, dtype=bf)
ops.stem_wpack2(w5, wk)
part2 = torch.empty(64, ops.stem_conv_tiles(B, T), 3, device=dev)
res["stem_pack"] = timed(lambda: ops.stem_pack(video, xp))
res["stem_conv_general"] = timed(lambda: ops.conv_fwd(gs, xp, wp, h0, part))
res["stem_conv_direct"] = timed(lambda: ops.stem_conv_fwd(video, wk, h0, part2))
del xp

# stage 1: 22 x 22 x 64, 3x3 stride 1
geom = ops.ConvGeom(N, 22, 22, 64, 64, 3, 3, (1, 1), (1, 1))
M = N * 484
x = torch.randn(M, 64, generator=g).to(dev, bf)
w = (torch.randn(64, 3, 3, 64, generator=g) * 0.04).to(dev, bf)
y = torch.empty(M, 64, device=dev, dtype=bf)
dy = torch.randn(M, 64, generator=g).to(dev, bf)
hh = torch.randn(M, 64, generator=g).to(dev, bf)
dx = torch.zeros(M, 64, device=dev, dtype=bf)
st = ops.BnState(64, dev)
st.mean.zero_(); st.invstd.fill_(1.0); st.scale.fill_(1.0); st.shift.zero_()
a = torch.full((64,), 0.25, device=dev)
dw = torch.zeros(64, 3, 3, 64, device=dev)
p1 = torch.empty(64, ops.conv_stat_tiles(geom, ops.dtype_code(x)), 3, device=dev)
for flag in ("0", "1"):
    L.set_option("conv_patch", int(flag))
    res[f"s1_fwd_patch{flag}"] = timed(lambda: ops.conv_fwd(geom, x, w, y, p1))
    res[f"s1_dgrad_bnr_patch{flag}"] = timed(lambda: ops.conv_bwd_data_bnr(geom, dy, w, dx, hh, st, a, beta=0.0))
    res[f"s1_dgrad_bnr_id_patch{flag}"] = timed(lambda: ops.conv_bwd_data_bnr(geom, dy, w, dx, hh, st, a, res=x,
                                                                             beta=1.0))
for flag in ("0", "1"):
    L.set_option("conv_wpatch", int(flag))
    res[f"s1_wgrad_wpatch{flag}"] = timed(lambda: ops.conv_bwd_weight(geom, x, dy, dw))
# stage 2: 11 x 11 x 128, 3x3 stride 1
geom2 = ops.ConvGeom(N, 11, 11, 128, 128, 3, 3, (1, 1), (1, 1))
M2 = N * 121
x2 = torch.randn(M2, 128, generator=g).to(dev, bf)
dy2 = torch.randn(M2, 128, generator=g).to(dev, bf)
dw2 = torch.zeros(128, 3, 3, 128, device=dev)
for flag in ("0", "1"):
    L.set_option("conv_wpatch", int(flag))
    res[f"s2_wgrad_wpatch{flag}"] = timed(lambda: ops.conv_bwd_weight(geom2, x2, dy2, dw2))
# stage-2 forward / data-grad (general implicit-GEMM kernels), for the fwd vs dgrad gap
w2 = (torch.randn(128, 3, 3, 128, generator=g) * 0.03).to(dev, bf)
y2 = torch.empty(M2, 128, device=dev, dtype=bf)
dx2 = torch.zeros(M2, 128, device=dev, dtype=bf)
hh2 = torch.randn(M2, 128, generator=g).to(dev, bf)
st2 = ops.BnState(128, dev)
st2.mean.zero_(); st2.invstd.fill_(1.0); st2.scale.fill_(1.0); st2.shift.zero_()
a2 = torch.full((128,), 0.25, device=dev)
p2 = torch.empty(128, ops.conv_stat_tiles(geom2, ops.dtype_code(x2)), 3, device=dev)
res["s2_fwd"] = timed(lambda: ops.conv_fwd(geom2, x2, w2, y2, p2))
res["s2_dgrad"] = timed(lambda: ops.conv_bwd_data(geom2, dy2, w2, dx2))
res["s2_dgrad_bnr"] = timed(lambda: ops.conv_bwd_data_bnr(geom2, dy2, w2, dx2, hh2, st2, a2, beta=0.0))
res["s2_gflop"] = round(2.0 * M2 * 128 * 1152 / 1e9, 1)
fl = 2.0 * M * 64 * 576
res["s1_gflop"] = round(fl / 1e9, 1)
res["stem_gflop_direct_k288"] = round(2.0 * N * 1936 * 64 * 288 / 1e9, 1)
res["unit"] = "us (median of %d)" % reps
print(json.dumps(res))
