"""Full-size parity of the HIP engine against the golden vectors the REFERENCE itself produced
at the BASELINE model size (tests/golden/make_golden_full.py: AVHubertAVSRConfig(odim=5049),
428 M parameters, recipe weights):

  * C1 (8 x 1 s, eval): encoder output; greedy / beam 3 (C4) / beam 5 (C5) decoding of the
    reference's own encoder output (exact token sequences, scores to 1e-4); the decoder's
    batch_score and the CTC log-softmax through the reference's module API;
  * the reference's evaluation call sequence replayed verbatim (script/evaluation.py:89-108:
    from_pretrained -> .eval().cuda() -> model.avsr.encoder(input_features=, video=) ->
    get_beam_search_decoder(model.avsr, token_list, beam_size) -> yseq[1:]) for every clip and
    beam: token-identical in fp32 (the reference's evaluation precision); in bf16 the match
    rate is reported;
  * a C2-shaped train step at T=375 (B=2, one row padded to 300 frames, dropouts 0): losses,
    encoder / CTC / decoder logit rows within the north-star 1e-3 bound, every gradient norm,
    BatchNorm running statistics.

Tolerances (relative, ||a-b||_inf / ||b||_inf) are written per test below. Set AVSR_REPORT_DIR
to also write the measured errors as JSON."""
import json
import os

import numpy as np
import pytest
import torch

from avsr_amd.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from oracle.weights import NO_DROPOUT
from tests.golden.full_inputs import C1, DEC_ROWS, ENC_ROWS
from tests.oracle_util import (TOKENS, full_c1_batch, full_state, full_train_batch, load_golden_full, rel,
                               zero_grad_by_symmetry)

pytestmark = pytest.mark.gpu

REPORT = {}


def _report(key, value):
    REPORT[key] = value
    d = os.environ.get("AVSR_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "parity_fullsize.json"), "w") as f:
            json.dump(REPORT, f, indent=1, sort_keys=True)


@pytest.fixture(scope="module")
def g():
    return load_golden_full()


@pytest.fixture(scope="module")
def state(g):
    return {k: torch.from_numpy(v) for k, v in full_state(g).items()}


@pytest.fixture(scope="module")
def model(state):
    """one full-size model (built once: 428 M parameters); every test reloads the recipe
    state (parameters AND BatchNorm buffers) before it runs."""
    m = AVHubertAVSR(AVHubertAVSRConfig(odim=5049, **NO_DROPOUT))
    m.load_state_dict(state, strict=True)
    return m


def _fresh(model, state, dtype):
    model.setup_engine("cuda", dtype)
    model.load_state_dict(state, strict=True)
    model.zero_grad()
    return model


# ------------------------------------------------------------------------------- C1 eval
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 6e-2)])
def test_c1_encoder(g, model, state, dtype, tol):
    m = _fresh(model, state, dtype).eval()
    b = full_c1_batch(g)
    with torch.no_grad():
        x = m.avsr.encoder(input_features=torch.from_numpy(b["audios"]).cuda(),
                           video=torch.from_numpy(b["videos"]).cuda()).last_hidden_state
    err = rel(x.cpu(), g["c1_enc"])
    _report(f"c1_encoder_{str(dtype)[6:]}", err)
    assert x.dtype == torch.float32 and x.shape == (C1["B"], C1["T"], 1024)
    assert err < tol


@pytest.mark.parametrize("beam", [1, 3, 5])
def test_c1_decode_reference_encoder_output(g, model, state, beam):
    """the decoder + CTC prefix scorer, driven by the engine's beam search, on the
    reference's own encoder output: exact best token sequence, score within 1e-4."""
    m = _fresh(model, state, torch.float32).eval()
    bs = get_beam_search_decoder(m.avsr, TOKENS, ctc_weight=0.1, beam_size=beam)
    worst = 0.0
    for c in range(C1["B"]):
        x = torch.from_numpy(g["c1_enc"][c]).cuda()
        best = bs(x)[0].asdict()
        assert best["yseq"] == g[f"c1_yseq_b{beam}_{c}"].tolist(), (c, best["yseq"])
        ref = float(g[f"c1_score_b{beam}_{c}"][0])
        worst = max(worst, abs(best["score"] - ref) / abs(ref))
    _report(f"c1_decode_score_b{beam}", worst)
    assert worst <= 1e-4


@pytest.mark.parametrize("beam", [1, 3, 5])
def test_c1_decode_batched(g, model, state, beam):
    """the 8 C1 clips decoded together (BatchBeamSearch.decode_batch, one launch sequence for all
    utterances) reproduce the reference's per-utterance best hypotheses."""
    m = _fresh(model, state, torch.float32).eval()
    bs = get_beam_search_decoder(m.avsr, TOKENS, ctc_weight=0.1, beam_size=beam)
    hyps = bs.decode_batch([torch.from_numpy(g["c1_enc"][c]).cuda() for c in range(C1["B"])])
    for c in range(C1["B"]):
        best = hyps[c][0].asdict()
        assert best["yseq"] == g[f"c1_yseq_b{beam}_{c}"].tolist(), (c, best["yseq"])
        ref = float(g[f"c1_score_b{beam}_{c}"][0])
        assert abs(best["score"] - ref) <= 1e-4 * abs(ref)


def test_c1_module_api(g, model, state):
    """Decoder.batch_score (decoder.py:199-227) and CTC.log_softmax (ctc.py:163-170) as the
    reference's scorers call them."""
    m = _fresh(model, state, torch.float32).eval()
    x = torch.from_numpy(g["c1_enc"][:2]).cuda()
    ys = torch.tensor([[5048, 5, 17, 301], [5048, 4000, 4000, 2]]).cuda()
    logp, states = m.avsr.decoder.batch_score(ys, [None, None], x)
    e1 = rel(logp.cpu(), g["c1_batch_score"])
    e2 = rel(m.avsr.ctc.log_softmax(x[:1]).cpu(), g["c1_ctc_logp0"])
    _report("c1_batch_score", e1)
    _report("c1_ctc_log_softmax", e2)
    assert e1 < 1e-4 and e2 < 1e-4
    assert len(states) == 2 and len(states[0]) == 6 and states[0][0].shape == (4, 1024)


def _replay_evaluation(ckpt, audios, videos, beam, dtype):
    """script/evaluation.py:89-108, statement by statement (AVSRCocktailModel.load_model +
    inference), with this package's classes."""
    avsr_model = AVHubertAVSR.from_pretrained(ckpt)
    avsr_model.eval().cuda()
    if dtype != torch.float32:
        avsr_model.to(dtype=dtype)
    model = avsr_model.avsr
    beam_search = get_beam_search_decoder(model, TOKENS, beam_size=beam)
    out = []
    for a, v in zip(audios, videos):
        avhubert_features = model.encoder(input_features=a, video=v)
        audiovisual_feat = avhubert_features.last_hidden_state
        audiovisual_feat = audiovisual_feat.squeeze(0)
        nbest_hyps = beam_search(audiovisual_feat)
        nbest_hyps = [h.asdict() for h in nbest_hyps[:min(len(nbest_hyps), 1)]]
        out.append(list(map(int, nbest_hyps[0]["yseq"][1:])))
    return out


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_c1_evaluation_script_replay(g, model, state, tmp_path, dtype):
    """C1 / C4 / C5 decode configurations end to end through the reference's call forms:
    fp32 (the reference evaluates in fp32) must be token-identical for all 8 clips x beams
    1, 3, 5; bf16 reports its match rate (and must decode)."""
    m = _fresh(model, state, torch.float32)
    m.save_pretrained(tmp_path)
    b = full_c1_batch(g)
    audios = [torch.from_numpy(b["audios"][c:c + 1]).cuda() for c in range(C1["B"])]
    videos = [torch.from_numpy(b["videos"][c:c + 1]).cuda() for c in range(C1["B"])]
    match, total = 0, 0
    for beam in (1, 3, 5):
        got = _replay_evaluation(str(tmp_path), audios, videos, beam, dtype)
        for c in range(C1["B"]):
            want = g[f"c1_yseq_b{beam}_{c}"].tolist()[1:]
            total += 1
            match += int(got[c] == want)
            if dtype == torch.float32:
                assert got[c] == want, (beam, c)
            else:
                assert len(got[c]) > 0
    _report(f"c1_replay_match_{str(dtype)[6:]}", f"{match}/{total}")


# ---------------------------------------------------------------------- train step T=375
TR_TOL = {torch.float32: dict(loss=1e-4, rows=1e-3, grad=2e-3, bn=1e-4),
          torch.bfloat16: dict(loss=3e-2, rows=8e-2, grad=1.2e-1, bn=5e-2)}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_train_step_t375(g, model, state, dtype):
    tol = TR_TOL[dtype]
    m = _fresh(model, state, dtype).train()
    b = {k: torch.from_numpy(v).cuda() for k, v in full_train_batch(g).items()}
    eng = m.avsr.engine()
    eng.capture = {}
    out = m(**b)
    out.loss.backward()
    torch.cuda.synchronize()
    ctx, eng.capture = eng.capture, None
    ref = g["tr_loss"]
    e_loss = max(abs(float(x) - r) / abs(r) for x, r in zip((out.loss, out.loss_ctc, out.loss_att), ref[:3]))
    # encoder / CTC / decoder rows of this forward (train mode: batch statistics)
    enc = ctx["enc"].float().view(2, 375, -1)[:, list(ENC_ROWS)].cpu()
    ctc = ctx["clog"].float().view(2, 375, -1)[:, list(ENC_ROWS), :5049].cpu()
    L1 = ctx["bt"]["L1"]
    dec = ctx["dlog"].float().view(2, L1, -1)[:, list(DEC_ROWS), :5049].cpu()
    e_rows = max(rel(enc, g["tr_enc_rows"]), rel(ctc, g["tr_ctc_rows"]), rel(dec, g["tr_dec_rows"]))
    params = dict(m.named_parameters())
    worst, bad = 0.0, []
    for k, n in zip(g["grad_keys"], g["grad_norm"]):
        k = str(k)
        got = params[k].grad.double().norm().item()
        if zero_grad_by_symmetry(k):
            if got > 1e-2:
                bad.append((k, got, float(n)))
            continue
        if n > 1e-3:
            worst = max(worst, abs(got - n) / n)
        if abs(got - n) > tol["grad"] * abs(n) + 1e-6:
            bad.append((k, got, float(n)))
    sdm = m.state_dict()
    e_bn = 0.0
    for k, row in zip(g["bn_keys"], g["bn_after"]):
        got = sdm[str(k)].detach().flatten()[:8].cpu().numpy()
        e_bn = max(e_bn, float(np.abs(got - row[:len(got)]).max() / max(1e-6, np.abs(row).max())))
    key = str(dtype)[6:]
    _report(f"t375_{key}", dict(loss=e_loss, rows=e_rows, grad_norm_worst=worst, bn=e_bn,
                               acc=(float(out.acc), float(ref[3]))))
    assert e_loss < tol["loss"]
    assert e_rows < tol["rows"]
    assert not bad, bad[:8]
    assert e_bn < tol["bn"]
    assert len(params) and len(g["grad_keys"]) == sum(1 for p in m.parameters() if p.grad is not None)


# ------------------------------------------------------------- searches ending early
@pytest.mark.parametrize("off", [4.0, 6.0, 8.0])
@pytest.mark.parametrize("beam", [3, 5])
def test_early_ending_beam_search(g, model, state, off, beam):
    """tests/golden/avsr_endbeam.npz: the reference's searches with a raised <eos> bias stop
    before maxlen (end_detect, e2e_asr_common.py:18-48) and return hypotheses that ended at
    different lengths (beam_search.py:330-406). The engine's one-utterance search AND the
    batched search return the same ended list: token sequences identical, total / decoder /
    CTC scores within 1e-4 (fp32) of the reference, and batched == one-utterance bit for bit."""
    from tests.golden.full_inputs import ENDBEAM
    from tests.oracle_util import endbeam_case, endbeam_state, load_golden_endbeam
    ge = load_golden_endbeam()
    st = {k: torch.from_numpy(v) for k, v in endbeam_state(g, off).items()}
    m = _fresh(model, st, torch.float32).eval()
    bs = get_beam_search_decoder(m.avsr, TOKENS, ctc_weight=0.1, beam_size=beam)
    xs = [torch.from_numpy(g["c1_enc"][c]).cuda() for c in ENDBEAM["clips"]]
    batched = bs.decode_batch(xs)
    worst = 0.0
    for c, x, hb in zip(ENDBEAM["clips"], xs, batched):
        ref = endbeam_case(ge, off, beam, c)
        single = bs(x)
        for h1, h2 in zip((h.asdict() for h in single), (h.asdict() for h in hb)):
            assert h1["yseq"] == h2["yseq"] and float(h1["score"]) == float(h2["score"]), c
            assert all(float(h1["scores"][k]) == float(h2["scores"][k]) for k in h1["scores"]), c
        assert len(single) == len(hb)
        for hyps in (single, hb):
            got = [h.asdict() for h in hyps]
            assert [h["yseq"] for h in got] == [r[0] for r in ref], (c, [len(h["yseq"]) for h in got])
            for h, r in zip(got, ref):
                for a, b in ((h["score"], r[1]), (h["scores"]["decoder"], r[2]), (h["scores"]["ctc"], r[3])):
                    worst = max(worst, abs(a - b) / max(abs(b), 1e-3))
    _report(f"endbeam_{off:g}_b{beam}", worst)
    assert worst <= 1e-4
