"""Pin the CPU oracle (oracle/avsr_oracle.py) to the golden vectors the reference itself
produced (tests/golden/make_golden.py). CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import avsr_oracle as O
from tests.oracle_util import golden_batch, golden_state, load_golden, rel, tiny_cfg


@pytest.fixture(scope="module")
def g():
    return load_golden()


def test_encoder_eval(g):
    torch.set_num_threads(8)
    sd = O.to_torch_state(golden_state(g))
    b = golden_batch(g)
    with torch.no_grad():
        x = O.encoder_forward(sd, tiny_cfg(), torch.from_numpy(b["audios"]), torch.from_numpy(b["videos"]), None, False)
    assert rel(x, g["enc_eval"]) < 1e-4


@pytest.fixture(scope="module")
def train_run(g):
    torch.set_num_threads(8)
    sd = O.to_torch_state(golden_state(g), requires_grad=True)
    b = {k: torch.from_numpy(v) for k, v in golden_batch(g).items()}
    loss, lc, la, acc, ex = O.e2e_forward(sd, tiny_cfg(), b["videos"], b["audios"], b["video_lengths"], b["labels"], True)
    loss.backward()
    return sd, (loss, lc, la, acc), ex


def test_train_losses(g, train_run):
    _, (loss, lc, la, acc), ex = train_run
    ref = g["loss"]
    assert abs(loss.item() - ref[0]) / abs(ref[0]) < 1e-5
    assert abs(lc.item() - ref[1]) / abs(ref[1]) < 1e-5
    assert abs(la.item() - ref[2]) / abs(ref[2]) < 1e-5
    assert acc == pytest.approx(ref[3])
    assert rel(ex["enc"].detach(), g["enc_train"]) < 1e-4
    assert rel(ex["ctc_logits"].detach().transpose(0, 1), g["ctc_logits"]) < 1e-4
    assert rel(ex["dec_logits"].detach(), g["dec_logits"]) < 1e-4


def test_train_grads(g, train_run):
    sd, _, _ = train_run
    for k, n, head in zip(g["grad_keys"], g["grad_norm"], g["grad_head"]):
        gr = sd[k].grad
        assert gr is not None, k
        assert torch.isfinite(gr).all(), k
        assert abs(gr.double().norm().item() - n) <= 1e-4 * abs(n) + 1e-9, k
        h = gr.flatten()[:8].numpy()
        np.testing.assert_allclose(h, head[:len(h)], rtol=2e-3, atol=1e-6 * max(1.0, abs(n)))


def test_bn_running_stats(g, train_run):
    sd, _, _ = train_run
    for k, row in zip(g["bn_keys"], g["bn_after"]):
        np.testing.assert_allclose(sd[k].detach().flatten()[:8].numpy(), row, rtol=1e-5, atol=1e-6)


def test_decoder_one_step(g):
    sd = O.to_torch_state(golden_state(g))
    cfg = tiny_cfg()
    for b in range(2):
        x = torch.from_numpy(g[f"dec_enc_{b}"])
        with torch.no_grad():
            logp = O.decoder_one_step(sd, cfg, torch.tensor([[5048, 5, 17, 301]]), x.unsqueeze(0))
        assert rel(logp, g[f"onestep_{b}"]) < 1e-5


@pytest.mark.parametrize("b", [0, 1])
@pytest.mark.parametrize("beam", [1, 3])
def test_beam_search_oracle(g, b, beam):
    """oracle/decode_oracle.py (BatchBeamSearch + CTCPrefixScoreTH restated) reproduces the
    reference's best hypothesis (token sequence exactly, score to 1e-4) on the reference's
    own encoder output and CTC log-probs."""
    from oracle import decode_oracle as D
    sd = O.to_torch_state(golden_state(g))
    x = torch.from_numpy(g[f"dec_enc_{b}"])
    ctc_logp = torch.from_numpy(g[f"ctc_logp_{b}"])[0]
    hyps = D.beam_search(sd, tiny_cfg(), x, ctc_logp, beam, ctc_weight=0.1)
    assert hyps[0].yseq == g[f"yseq_b{beam}_{b}"].tolist()
    ref = float(g[f"score_b{beam}_{b}"][0])
    assert abs(hyps[0].score - ref) <= 1e-4 * abs(ref)


def _ctcw_hyps(c, key):
    """every hypothesis the reference returned for avsr_ctcw.npz entry `key`"""
    lens = c[key + "_len"]
    ys = np.split(c[key + "_yseq"], np.cumsum(lens)[:-1])
    return [y.tolist() for y in ys], c[key + "_score"]


@pytest.mark.parametrize("w", [0.0, 1.0])
@pytest.mark.parametrize("beam", [1, 3])
@pytest.mark.parametrize("b", [0, 1])
def test_beam_search_oracle_one_scorer(g, w, beam, b):
    """the oracle's decoder-only (ctc_weight 0) and CTC-only full-vocabulary (ctc_weight 1)
    searches return the reference's hypotheses (tests/golden/make_golden_ctcw.py): every token
    sequence in order, scores to 1e-5"""
    from oracle import decode_oracle as D
    c = np.load(os.path.join(os.path.dirname(__file__), "golden", "avsr_ctcw.npz"))
    sd = O.to_torch_state(golden_state(g))
    x = torch.from_numpy(g[f"dec_enc_{b}"])
    ctc_logp = torch.from_numpy(g[f"ctc_logp_{b}"])[0]
    hyps = D.beam_search(sd, tiny_cfg(), x, ctc_logp, beam, ctc_weight=w)
    ys, scores = _ctcw_hyps(c, f"w{w:g}_b{beam}_{b}")
    assert [h.yseq for h in hyps] == ys
    for h, s in zip(hyps, scores):
        assert abs(h.score - s) <= 1e-5 * abs(s)
    assert set(hyps[0].scores) == ({"decoder"} if w == 0.0 else {"ctc"})
