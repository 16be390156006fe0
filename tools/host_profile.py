"""cProfile of the host side of the C2 train step (bench.py's step, 4 steps after warm-up):
where the ~20 ms of per-step Python / launch time goes. usage: python tools/host_profile.py"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from avsr_amd.avhubert_avsr_model import AVHubertAVSR  # noqa: E402
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig  # noqa: E402
from avsr_amd.optim import FusedAdamW  # noqa: E402
from bench import synthetic_batch  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
cfg = AVHubertAVSRConfig(odim=5049)
model = AVHubertAVSR(cfg).train()
model.setup_engine(dev, torch.bfloat16)
eng = model.avsr.engine()
opt = FusedAdamW(eng.arena, lr=1e-4, weight_decay=0.005, max_grad_norm=1.0)
v, a, lens, lab = synthetic_batch(16, 375, 40)
v, a = v.to(dev), a.to(dev)
d_ctc = torch.full((1,), cfg.mtlalpha, device=dev)
d_att = torch.full((1,), 1.0 - cfg.mtlalpha, device=dev)
np.random.seed(5)


def step(i):
    eng.arena.zero_grad()
    out, ctx = eng.forward(v, a, lens, lab, train=True, need_grad=True, seed=100 + i)
    eng.backward(ctx, d_ctc, d_att)
    opt.step()


for i in range(3):
    step(i)
torch.cuda.synchronize()
# enqueue time of one step with the GPU idle at its start (no profiler) vs its completion
import time  # noqa: E402
for i in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(20 + i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {i} ({eng.last_modality}): host enqueue {1e3 * (t1 - t0):.1f} ms, GPU done at {1e3 * (t2 - t0):.1f} ms",
          flush=True)
pr = cProfile.Profile()
pr.enable()
for i in range(4):
    step(10 + i)
    torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(30)
