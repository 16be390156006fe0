"""Pin the CPU oracle at the BASELINE model size (AVHubertAVSRConfig(odim=5049), 428 M
parameters) to the full-size golden vectors the reference itself produced
(tests/golden/make_golden_full.py): C1 eval encoder (8 x 1 s), greedy / beam 3 / beam 5
decoding, and a T=375 train step (B=2, one padded row). CPU only (≈ 1 min, ≈ 15 GB RAM)."""
import numpy as np
import pytest
import torch

from oracle import avsr_oracle as O
from oracle import decode_oracle as D
from tests.golden.full_inputs import DEC_ROWS, ENC_ROWS
from tests.oracle_util import full_c1_batch, full_state, full_train_batch, load_golden_full, rel


@pytest.fixture(scope="module")
def g():
    return load_golden_full()


@pytest.fixture(scope="module")
def sd(g):
    return O.to_torch_state(full_state(g))


def test_c1_encoder_eval(g, sd):
    torch.set_num_threads(8)
    b = full_c1_batch(g)
    with torch.no_grad():
        x = O.encoder_forward(sd, O.OracleConfig(), torch.from_numpy(b["audios"]), torch.from_numpy(b["videos"]),
                              None, False)
    assert rel(x, g["c1_enc"]) < 1e-4


@pytest.mark.parametrize("beam", [1, 3, 5])
def test_c1_decode(g, sd, beam):
    """greedy / beam 3 (C4) / beam 5 (C5) on the reference's own encoder output: exact
    token sequence, score to 1e-4 (clips 0 and 5 — the GPU tests cover all 8)."""
    torch.set_num_threads(8)
    cfg = O.OracleConfig()
    W, bias = sd["avsr.ctc.ctc_lo.weight"], sd["avsr.ctc.ctc_lo.bias"]
    for c in (0, 5):
        x = torch.from_numpy(g["c1_enc"][c])
        ctc_logp = torch.log_softmax(x @ W.t() + bias, -1)
        hyps = D.beam_search(sd, cfg, x, ctc_logp, beam, ctc_weight=0.1)
        assert hyps[0].yseq == g[f"c1_yseq_b{beam}_{c}"].tolist(), (c, beam)
        ref = float(g[f"c1_score_b{beam}_{c}"][0])
        assert abs(hyps[0].score - ref) <= 1e-4 * abs(ref)


def test_c1_batch_score(g, sd):
    x = torch.from_numpy(g["c1_enc"][:2])
    with torch.no_grad():
        logp = O.decoder_one_step(sd, O.OracleConfig(), torch.tensor([[5048, 5, 17, 301], [5048, 4000, 4000, 2]]), x)
        ctc = torch.log_softmax(x[:1] @ sd["avsr.ctc.ctc_lo.weight"].t() + sd["avsr.ctc.ctc_lo.bias"], -1)
    assert rel(logp, g["c1_batch_score"]) < 1e-5
    assert rel(ctc, g["c1_ctc_logp0"]) < 1e-5


def test_train_step_t375(g):
    torch.set_num_threads(8)
    sdg = O.to_torch_state(full_state(g), requires_grad=True)
    b = {k: torch.from_numpy(v) for k, v in full_train_batch(g).items()}
    loss, lc, la, acc, ex = O.e2e_forward(sdg, O.OracleConfig(), b["videos"], b["audios"], b["video_lengths"],
                                          b["labels"], True)
    loss.backward()
    ref = g["tr_loss"]
    for got, r in zip((loss.item(), lc.item(), la.item()), ref[:3]):
        assert abs(got - r) <= 1e-5 * abs(r)
    assert acc == pytest.approx(ref[3])
    rows = list(ENC_ROWS)
    assert rel(ex["enc"].detach()[:, rows], g["tr_enc_rows"]) < 1e-4
    assert rel(ex["ctc_logits"].detach().transpose(0, 1)[:, rows], g["tr_ctc_rows"]) < 1e-4
    assert rel(ex["dec_logits"].detach()[:, list(DEC_ROWS)], g["tr_dec_rows"]) < 1e-4
    for k, n in zip(g["grad_keys"], g["grad_norm"]):
        gr = sdg[k].grad
        assert gr is not None and torch.isfinite(gr).all(), k
        # k_proj.bias gradients are zero up to round-off (softmax shift invariance): absolute floor
        assert abs(gr.double().norm().item() - n) <= 1e-3 * abs(n) + 1e-6, (k, gr.double().norm().item(), n)
    for k, row in zip(g["bn_keys"], g["bn_after"]):
        got = sdg[k].detach().flatten()[:8].numpy()
        np.testing.assert_allclose(got, row[:len(got)], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("off", [4.0, 6.0, 8.0])
@pytest.mark.parametrize("beam", [3, 5])
def test_early_ending_beams(g, off, beam):
    """searches that end before maxlen (raised <eos> bias): end_detect and the ranking of
    hypotheses ended at different lengths reproduce the reference's full ended list"""
    from tests.golden.full_inputs import ENDBEAM
    from tests.oracle_util import endbeam_case, endbeam_state, load_golden_endbeam
    ge = load_golden_endbeam()
    torch.set_num_threads(8)
    sdb = O.to_torch_state(endbeam_state(g, off))
    cfg = O.OracleConfig()
    W, bias = sdb["avsr.ctc.ctc_lo.weight"], sdb["avsr.ctc.ctc_lo.bias"]
    c = ENDBEAM["clips"][-1]
    x = torch.from_numpy(g["c1_enc"][c])
    hyps = D.beam_search(sdb, cfg, x, torch.log_softmax(x @ W.t() + bias, -1), beam, ctc_weight=0.1)
    ref = endbeam_case(ge, off, beam, c)
    assert len(hyps) == len(ref)
    for h, r in zip(hyps, ref):
        assert h.yseq == r[0]
        assert abs(h.score - r[1]) <= 1e-4 * abs(r[1])
