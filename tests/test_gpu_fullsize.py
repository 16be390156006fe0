"""Full-size parity (BASELINE configs' model: AVHubertAVSRConfig(odim=5049), 24 encoder layers,
428 M parameters) of the HIP engine in fp32 parity mode against the CPU oracle on the same
deterministic weights (SURVEY c6 recipe) and a seeded 2-clip batch (one padded row):
eval-encoder output and CTC logits within the north-star 1e-3 relative bound, train-step
losses, and gradient norms across the model. Dropouts off (random streams cannot be matched)."""
import numpy as np
import pytest
import torch

from avsr_amd import ops
from avsr_amd.avhubert_avsr_model import AVHubertAVSR
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from oracle import avsr_oracle as O
from oracle.weights import NO_DROPOUT, collate, make_inputs, make_state_dict
from tests.oracle_util import rel

pytestmark = pytest.mark.gpu

# fp32 storage = parity mode (north_star: logits within 1e-3 relative); bf16 = throughput mode
TOL = {torch.float32: dict(logits=1e-3, loss=1e-4, grad=2e-3),
       torch.bfloat16: dict(logits=6e-2, loss=3e-2, grad=1e-1)}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_full_size_model_parity(dev, dtype):
    TOL_LOGITS, TOL_LOSS, TOL_GRAD = TOL[dtype]["logits"], TOL[dtype]["loss"], TOL[dtype]["grad"]
    torch.set_num_threads(16)
    m = AVHubertAVSR(AVHubertAVSRConfig(odim=5049, **NO_DROPOUT))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    state = make_state_dict(shapes)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()}, strict=True)
    m.setup_engine(dev, dtype)
    T = 50
    frames, feats, lengths, _ = make_inputs(B=2, T=T, lengths=(T, 41), seed=4321)
    labels = ((12, 7, 4001, 33, 5047, 1, 250), (9, 88, 1234, 3))
    b = {k: torch.from_numpy(v) for k, v in collate(frames, feats, lengths, labels).items()}
    cfg = O.OracleConfig()
    sd = O.to_torch_state(state, requires_grad=True)

    # eval encoder (script/evaluation.py call form, no mask) + CTC logits
    m.eval()
    eng = m.avsr.engine()
    enc = eng.encode(b["audios"], b["videos"])
    with torch.no_grad():
        ref_enc = O.encoder_forward(sd, cfg, b["audios"], b["videos"], None, train=False)
    e_enc = rel(enc.float().cpu(), ref_enc)
    assert e_enc < TOL_LOGITS
    W = m.avsr.ctc.ctc_lo.weight.detach().to(dev, dtype)
    bias = m.avsr.ctc.ctc_lo.bias.detach().to(dev, torch.float32)
    logits = ops.linear_fwd(enc.reshape(-1, enc.shape[-1]).contiguous(), W.contiguous(), bias)
    ref_logits = ref_enc.reshape(-1, ref_enc.shape[-1]) @ sd["avsr.ctc.ctc_lo.weight"].detach().t() + \
        sd["avsr.ctc.ctc_lo.bias"].detach()
    e_log = rel(logits.float().cpu(), ref_logits)
    assert e_log < TOL_LOGITS

    # train step: losses and gradients
    m.train()
    out = m(**b)
    out.loss.backward()
    torch.cuda.synchronize()
    loss, lc, la, acc, _ = O.e2e_forward(sd, cfg, b["videos"], b["audios"], b["video_lengths"], b["labels"], True)
    loss.backward()
    for got, ref in ((out.loss, loss), (out.loss_ctc, lc), (out.loss_att, la)):
        assert abs(got.item() - ref.item()) / abs(ref.item()) < TOL_LOSS, (got.item(), ref.item())
    e_loss = max(abs(g.item() - r.item()) / abs(r.item()) for g, r in ((out.loss, loss), (out.loss_ctc, lc),
                                                                        (out.loss_att, la)))
    params = dict(m.named_parameters())
    keys = [k for k in sd if sd[k].grad is not None]
    bad, worst = [], 0.0
    for k in keys[:: max(1, len(keys) // 48)]:
        ref = sd[k].grad.double().norm().item()
        got = params[k].grad.double().norm().item()
        if abs(ref) > 1e-3:
            worst = max(worst, abs(got - ref) / abs(ref))
        if abs(got - ref) > TOL_GRAD * abs(ref) + TOL_GRAD * 1e-3:
            bad.append((k, got, ref))
    print(f"full-size parity ({dtype}): encoder {e_enc:.2e}, CTC logits {e_log:.2e}, losses {e_loss:.2e}, "
          f"grad norms (worst of {len(keys[:: max(1, len(keys) // 48)])}) {worst:.2e}")
    assert not bad, bad[:8]
