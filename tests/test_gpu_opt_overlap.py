"""Overlapped optimizer step (FusedAdamW(overlap=True), optim.ParamGate): the AdamW update runs
on its own stream in forward-ordered chunks while the next forward waits per stage only for
the chunk it reads, and the gradients are cleared behind the update. The update is
elementwise, so three bench-style steps (bf16 production path, dropouts on, modality draws
seeded) must leave the parameters, the bf16 shadow, the AdamW moments and the losses
bit-identical to the serial step."""
import numpy as np
import pytest
import torch

from avsr_amd.avhubert_avsr_model import AVHubertAVSR
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from avsr_amd.optim import FusedAdamW
from oracle.weights import TINY_CONFIG
from tests.oracle_util import golden_batch, golden_state, load_golden

pytestmark = pytest.mark.gpu


def _run(overlap, steps=3):
    g = load_golden()
    dev = torch.device("cuda:0")
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG)).train()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
    m.setup_engine(dev, torch.bfloat16)
    eng = m.avsr.engine()
    arena = eng.arena
    opt = FusedAdamW(arena, lr=1e-3, weight_decay=0.005, max_grad_norm=1.0, overlap=overlap,
                     stage_bounds=eng.param_stage_bounds())
    b = {k: torch.from_numpy(v) for k, v in golden_batch(g).items()}
    v, a = b["videos"].to(dev), b["audios"].to(dev)
    d_ctc = torch.full((1,), 0.1, device=dev)
    d_att = torch.full((1,), 0.9, device=dev)
    np.random.seed(5)
    arena.zero_grad()
    losses = []
    for i in range(steps):
        if not overlap:
            arena.zero_grad()
        out4, ctx = eng.forward(v, a, b["video_lengths"], b["labels"], train=True, need_grad=True, seed=100 + i)
        losses.append(out4.clone())
        eng.backward(ctx, d_ctc, d_att)
        opt.step(zero_grad=overlap)
    opt.sync()
    torch.cuda.synchronize()
    return (torch.stack(losses).cpu(), arena.data.cpu(), arena.shadow.cpu(), arena.exp_avg.cpu(),
            arena.exp_avg_sq.cpu(), arena.grad.cpu())


def test_overlapped_update_bit_identical_to_serial():
    ser = _run(False)
    ovl = _run(True)
    for name, x, y in zip(("losses", "params", "shadow", "exp_avg", "exp_avg_sq"), ser[:5], ovl[:5]):
        assert torch.equal(x, y), (name, (x.float() - y.float()).abs().max().item())
    # the overlapped step clears the gradients behind the update
    assert not ovl[5].any()


def test_stage_bounds_follow_forward_order():
    g = load_golden()
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG)).train()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
    m.setup_engine(torch.device("cuda:0"), torch.bfloat16)
    eng = m.avsr.engine()
    b = eng.param_stage_bounds()
    d0, d1 = eng.arena.segments["decay"]
    assert len(b) == eng.nl + 1 and b == sorted(b) and d0 < b[0] and b[-1] <= d1
    meta = eng.arena.meta
    for i in range(eng.nl):     # every decay parameter of layer i lies in [b[i], b[i+1])
        offs = [mm["off"] for n, mm in meta.items() if n.startswith(f"encoder.encoder.layers.{i}.") and d0 <= mm["off"] < d1]
        assert b[i] <= min(offs) and max(offs) < b[i + 1]


def test_cu_masked_side_stream_bit_identical(monkeypatch):
    """AVSR_SIDE_CUS confines the weight-gradient side stream to a subset of the CUs
    (avsr_stream_create_cumask); where a kernel runs does not change what it computes"""
    monkeypatch.delenv("AVSR_SIDE_CUS", raising=False)
    ref = _run(False, steps=2)
    monkeypatch.setenv("AVSR_SIDE_CUS", "1/2")
    got = _run(False, steps=2)
    for name, x, y in zip(("losses", "params", "shadow", "exp_avg", "exp_avg_sq"), ref[:5], got[:5]):
        assert torch.equal(x, y), name
