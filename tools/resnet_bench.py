"""ResNet-18 lip frontend fwd / bwd device time at C2 (16 x 375 frames = 6000 images of 88x88),
bf16, with the BatchNorm-backward reductions fused into the data-grad epilogues (engine
default) vs separate reduce passes (AVSR_BN_FUSE=0), interleaved in one process.
usage: python tools/resnet_bench.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import _lib as L, engine as E  # noqa: E402
from avsr_amd.avhubert_avsr_model import AVHubertAVSR  # noqa: E402
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig  # noqa: E402
from bench import synthetic_batch  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
torch.manual_seed(0)
m = AVHubertAVSR(AVHubertAVSRConfig(odim=5049, num_hidden_layers=1)).train()
m.setup_engine(dev, torch.bfloat16)
eng = m.avsr.engine()
v = synthetic_batch(16, 375, 40)[0].to(dev)
dfeat = None


def once(fuse):
    global dfeat
    E._BN_FUSE = fuse
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    feat, ctx = eng.video_fwd(v, True, True)
    ev[1].record()
    if dfeat is None:
        dfeat = torch.randn(feat.shape, device=dev).to(feat.dtype)
    eng.video_bwd(ctx, dfeat)
    eng.join_side()
    ev[2].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])


# variants: (label, BN fusion, library option conv_s2phase)
mode = sys.argv[2] if len(sys.argv) > 2 else "fuse"
variants = [("fuse=1", True, "1"), ("fuse=0", False, "1")] if mode == "fuse" else \
    [("c192=1", True, "1", "1"), ("c192=0", True, "1", "0")] if mode == "c192" else \
    [("patch=1", True, "1", "1", "1"), ("patch=0", True, "1", "1", "0")] if mode == "patch" else \
    [("new", True, "1", "1", "1", True), ("old", True, "1", "1", "0", False)] if mode == "new" else \
    [("s2phase=1", True, "1"), ("s2phase=0", True, "0")]


def run(var):
    L.set_option("conv_s2phase", int(var[2]))
    L.set_option("conv_192", int(var[3]) if len(var) > 3 else 1)
    L.set_option("conv_patch", int(var[4]) if len(var) > 4 else 1)
    E._STEM_DIRECT = var[5] if len(var) > 5 else True
    return once(var[1])


for var in variants:
    run(var)
res = {var[0]: [] for var in variants}
for _ in range(reps):
    for var in variants:
        res[var[0]].append(run(var))
for var in variants:
    r = res[var[0]]
    fw = sorted(x[0] for x in r)[len(r) // 2]
    bw = sorted(x[1] for x in r)[len(r) // 2]
    print(f"{var[0]}: video fwd {fw:.3f} ms  bwd {bw:.3f} ms (median of {reps})", flush=True)
