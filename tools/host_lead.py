"""Host lead over the GPU through the C2 train step (bench.py's loop, no syncs): at a few points
of each step the host time of issue vs the GPU time the step stream reaches it (events), and
every host call that blocks for more than 1 ms (library launches, event / stream waits,
allocations) with where it came from. usage: python tools/host_lead.py [steps]"""
import os
import sys
import time
import traceback
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from avsr_amd import engine as E, ops  # noqa: E402
from avsr_amd import _lib as L  # noqa: E402
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
E.prioritize_step_stream(dev)
opt = FusedAdamW(eng.arena, lr=1e-4, weight_decay=0.005, max_grad_norm=1.0)
eng.pre_video_grads = opt.early_sumsq
v, a, lens, lab = synthetic_batch(16, 375, 40)
v, a = v.to(dev), a.to(dev)
d_ctc = torch.full((1,), cfg.mtlalpha, device=dev)
d_att = torch.full((1,), 1.0 - cfg.mtlalpha, device=dev)
np.random.seed(5)
eng.force_modality = (None,)

marks = []          # (label, host t, event)
t_ref = [0.0]


def mark(label):
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    marks.append((label, time.perf_counter(), ev))


def wrap(obj, name, label):
    f = getattr(obj, name)

    def g(*args, **kw):
        mark(label + ">")
        r = f(*args, **kw)
        mark(label + "<")
        return r
    setattr(obj, name, g)


for n in ("encoder_fwd", "decoder_fwd", "decoder_bwd", "encoder_bwd", "video_bwd"):
    wrap(eng, n, n)

blocks = defaultdict(lambda: [0, 0.0, None])
armed = [False]


def timed(fn, label):
    def g(*args, **kw):
        t0 = time.perf_counter()
        r = fn(*args, **kw)
        dt = time.perf_counter() - t0
        if armed[0] and dt > 1e-3:
            where = "".join(f"{os.path.basename(f.filename)}:{f.lineno} " for f in traceback.extract_stack()[-6:-1])
            key = (label, where)
            b = blocks[key]
            b[0] += 1
            b[1] += dt
        return r
    return g


ops._call = timed(ops._call, "lib")
torch.cuda.Event.synchronize = timed(torch.cuda.Event.synchronize, "event.sync")
torch.cuda.Stream.wait_event = timed(torch.cuda.Stream.wait_event, "wait_event")
_empty = torch.empty
torch.empty = timed(_empty, "torch.empty")


def step():
    eng.zero_grad_async()
    mark("step>")
    out4, ctx = eng.forward(v, a, lens, lab, train=True, need_grad=True, seed=7)
    eng.backward(ctx, d_ctc, d_att)
    mark("opt>")
    opt.step()
    mark("step<")
    return out4


n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for _ in range(4):
    step()
torch.cuda.synchronize()
marks.clear()
armed[0] = True
ev0 = torch.cuda.Event(enable_timing=True)
ev0.record()
h0 = time.perf_counter()
for _ in range(n):
    step()
torch.cuda.synchronize()
armed[0] = False
print("label               host_ms   gpu_ms   lead_ms   (per timed step; lead = GPU reaches the point - host issues it)")
for lab_, ht, ev in marks[-40:]:
    g = ev0.elapsed_time(ev)
    h = (ht - h0) * 1e3
    print(f"{lab_:18s} {h:9.2f} {g:9.2f} {g - h:9.2f}")
print("host calls blocking > 1 ms (count, total ms, call site):")
for (lab_, where), (c, t, _) in sorted(blocks.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"  {lab_:11s} n={c:4d} {t * 1e3:9.2f} ms  {where}")
