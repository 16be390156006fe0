"""Three reference config options on the HIP engine against the reference's own outputs
(tests/golden/make_golden_cfgvar.py -> avsr_cfgvar.npz; tiny config, fp32 parity mode, dropouts
0): modality_fuse='add' (avhubert.py:225-233,486-489), transformer_length_normalized_loss
(label_smoothing_loss.py:61) and layerdrop (avhubert.py:709-712, with the optimizer skipping a
dropped layer's parameters as torch.optim.AdamW skips parameters whose grad is None)."""
import io

import pytest
import torch

from avsr_amd.avhubert_avsr_model import AVHubertAVSR
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from avsr_amd.optim import ArenaAdamW, FusedAdamW
from oracle import avsr_oracle as O
from oracle.weights import NO_DROPOUT, TINY_CONFIG
from tests.oracle_util import (CFGVAR, LDROP_SEED, cfgvar_oracle_cfg, cfgvar_state, golden_batch, load_cfgvar,
                               load_golden, rel, zero_grad_by_symmetry)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gv():
    return load_cfgvar()


@pytest.fixture(scope="module")
def batch():
    return {k: torch.from_numpy(v) for k, v in golden_batch(load_golden()).items()}


def _model(gv, name, dtype=torch.float32):
    cfg = AVHubertAVSRConfig(**{**TINY_CONFIG, **NO_DROPOUT, **CFGVAR[name]})
    m = AVHubertAVSR(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in cfgvar_state(gv, name).items()}, strict=True)
    m.setup_engine("cuda", dtype)
    return m


def test_modality_fuse_add_eval(gv, batch):
    m = _model(gv, "add").eval()
    assert not any("post_extract_proj" in k for k, _ in m.named_parameters())
    x = m.avsr.encoder(input_features=batch["audios"].cuda(), video=batch["videos"].cuda()).last_hidden_state
    assert rel(x.cpu(), gv["add_enc_eval"]) < 2e-4


@pytest.mark.parametrize("name", ["add", "lnorm", "ldrop"])
def test_train_step(gv, batch, name):
    m = _model(gv, name).train()
    eng = m.avsr.engine()
    eng.capture = {}
    if name == "ldrop":
        torch.manual_seed(LDROP_SEED)
    out = m(**batch)
    out.loss.backward()
    ref = gv[f"{name}_loss"]
    for got, want in zip((out.loss.item(), out.loss_ctc.item(), out.loss_att.item()), ref[:3]):
        assert abs(got - want) <= 2e-4 * abs(want), (name, got, want)
    assert rel(eng.capture["enc"].float().cpu().view(gv[f"{name}_enc_train"].shape), gv[f"{name}_enc_train"]) < 2e-4
    params = dict(m.named_parameters())
    keys = set(gv[f"{name}_grad_keys"].tolist())
    for k, n in zip(gv[f"{name}_grad_keys"], gv[f"{name}_grad_norm"]):
        got = params[k].grad.double().norm().item()
        if zero_grad_by_symmetry(k):
            continue
        assert abs(got - n) <= 5e-3 * n + 1e-6, (name, k, got, n)
    for k, p in params.items():          # no gradient in the reference (dropped layer, frozen): zero here
        if k not in keys and p.grad is not None:
            assert p.grad.abs().max().item() == 0.0, (name, k)
    if name == "ldrop":
        assert not any(".layers.1." in k for k in keys)


def _arena_opt(eng):
    return ArenaAdamW(eng.arena, lr=1e-3, eps=1e-3, weight_decay=0.05)


def _resume(opt, eng):
    """the HF Trainer checkpoint path: the optimizer state dict through torch.save /
    torch.load(weights_only=True), loaded into a fresh ArenaAdamW whose moments were cleared"""
    buf = io.BytesIO()
    torch.save(opt.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    eng.arena.exp_avg.zero_()
    eng.arena.exp_avg_sq.zero_()
    new = _arena_opt(eng)
    new.load_state_dict(sd)
    return new


@pytest.mark.parametrize("kind", ["fused", "arena_resume"])
def test_layerdrop_optimizer_skips_dropped_layers(gv, batch, kind):
    """two AdamW steps with LayerDrop: step 1 drops layer 1 (draws 0.758 / 0.279), step 2 drops
    layer 0 (seed 0: 0.496 / 0.768). torch.optim.AdamW on the oracle with zero_grad(set_to_none)
    skips the dropped layer's parameters (grad None): no decay, no moment update, and its own
    step count for the bias correction. The arena optimizer must land on the same parameters —
    also (kind arena_resume) when the Trainer's ArenaAdamW is checkpointed after step 1 and a
    fresh one resumes from that checkpoint: the per-layer step counts travel in its state dict."""
    m = _model(gv, "ldrop").train()
    eng = m.avsr.engine()
    # eps 1e-3: Adam's normalisation would turn round-off-level gradient differences (signs of
    # near-zero elements) into +-lr updates; with this eps an update follows its gradient
    if kind == "fused":
        opt = FusedAdamW(eng.arena, lr=1e-3, eps=1e-3, weight_decay=0.05, max_grad_norm=0.0)
    else:
        opt = _arena_opt(eng)
    sd = O.to_torch_state(cfgvar_state(gv, "ldrop"), requires_grad=True)
    ocfg = cfgvar_oracle_cfg("ldrop")
    names = [k for k, _ in m.named_parameters()]
    a = eng.arena
    seg = {}
    for k in names:          # the arena's weight-decay segments (biases / norms: no decay; frozen)
        off = a.meta[k[len("avsr."):]]["off"]
        seg[k] = next(s for s, (lo, hi) in a.segments.items() if lo <= off < hi)
    ref_opt = torch.optim.AdamW([{"params": [sd[k] for k in names if seg[k] == "decay"], "weight_decay": 0.05},
                                 {"params": [sd[k] for k in names if seg[k] == "no_decay"], "weight_decay": 0.0}],
                                lr=1e-3, eps=1e-3)
    b = batch
    l1 = {k: p.detach().clone() for k, p in m.named_parameters() if ".layers.1." in k}
    for seed in (LDROP_SEED, 0):
        eng.arena.zero_grad()
        ref_opt.zero_grad(set_to_none=True)
        torch.manual_seed(seed)
        out = m(**b)
        out.loss.backward()
        torch.manual_seed(seed)
        loss, *_ = O.e2e_forward(sd, ocfg, b["videos"], b["audios"], b["video_lengths"], b["labels"], True)
        loss.backward()
        assert abs(out.loss.item() - loss.item()) <= 2e-4 * abs(loss.item()), seed
        opt.step()
        ref_opt.step()
        if seed == LDROP_SEED:       # layer 1 dropped: untouched, not even decayed
            for k, v in l1.items():
                assert torch.equal(dict(m.named_parameters())[k].detach(), v), k
            if kind == "arena_resume":
                opt = _resume(opt, eng)
                assert opt.fused.layer_steps == [1, 0]
    params = dict(m.named_parameters())
    for k in names:
        if zero_grad_by_symmetry(k):     # round-off gradients: Adam normalises their noise to +-lr
            continue
        r = sd[k].detach()
        d = (params[k].detach().cpu() - r).abs().max().item() / max(1e-3, r.abs().max().item())
        # ResNet: parity-mode gradients there differ by up to ~5e-3 (train-mode BatchNorm backward,
        # as in test_gpu_surface.py), which an Adam step passes on element by element
        assert d < (1e-2 if ".resnet." in k else 2e-3), (k, d)
    assert (opt.layer_steps if kind == "fused" else opt.fused.layer_steps) == [1, 1]


def test_early_gradient_norm_matches_full(gv, batch):
    """FusedAdamW.early_sumsq on the engine's side stream before the ResNet backward plus the
    ResNet ranges at step time == the one-pass gradient norm (fp32 sums, tolerance 1e-6)"""
    m = _model(gv, "add").train()
    eng = m.avsr.engine()
    opt = FusedAdamW(eng.arena, max_grad_norm=1.0)
    eng.pre_video_grads = opt.early_sumsq
    eng.arena.zero_grad()
    out = m(**batch)
    out.loss.backward()
    assert opt._early
    split = opt.grad_sumsq().item()
    full = opt.grad_sumsq().item()
    assert not opt._early and full > 0
    assert abs(split - full) <= 1e-6 * full, (split, full)
