"""CPU restatement of the reference's joint CTC/attention beam search (TEST INFRASTRUCTURE
ONLY: imported by tests/ and __graft_entry__.smoke(), never by the product path).

Follows, for the configuration `get_beam_search_decoder` builds
(src/avhubert_avsr/avhubert_avsr_model.py:12-36: weights decoder 1-ctc_weight, ctc
ctc_weight, length_bonus 0 and lm None => both dropped, pre_beam_score_key "decoder"):
  BatchBeamSearch.search / batch_beam / post_process   src/nets/batch_beam_search.py:102-349
  BeamSearch.forward (maxlenratio 0 => maxlen = T)     src/nets/beam_search.py:330-400
  end_detect (M=3, D_end=-10)                          src/nets/e2e_asr_common.py:18-48
  CTCPrefixScoreTH.__call__ (B=1, no windowing)        src/nets/ctc_prefix_score.py:65-187
  CTCPrefixScorer.select_state                         src/nets/scorers/ctc.py:40-63
  Decoder.batch_score / forward_one_step               src/nets/backend/transformer/decoder.py:153-227
The decoder is evaluated without a cache (full causal recompute of the prefix), which is
the same function of the prefix as the reference's output cache.
ctc_weight 0 / 1 are the one-scorer searches the reference builds (a scorer of weight 0 is
dropped, beam_search.py:69-73): the decoder alone (no partial scorer => no pre-beam,
:96-100), or the CTC prefix scorer alone over the full vocabulary (pre_beam_score_key None).
"""
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np
import torch

from .avsr_oracle import decoder_one_step

LOGZERO = -10000000000.0


@dataclass
class Hyp:
    yseq: List[int]
    score: float
    scores: Dict[str, float] = field(default_factory=dict)
    ctc_r: torch.Tensor = None      # (T, 2) CTC forward variables of the prefix
    ctc_s: float = 0.0              # CTC prefix score of the prefix

    def asdict(self):
        return {"yseq": list(self.yseq), "score": float(self.score),
                "scores": {k: float(v) for k, v in self.scores.items()}}


def ctc_prefix_scores(logp, yseqs, states, ids, blank, eos):
    """CTCPrefixScoreTH.__call__ for one utterance (batch 1), n hypotheses, scoring ids
    (n, P). logp: (T, V) CTC log-probs. states: per hyp (r (T,2), s) or None at the first
    step. Returns (log_psi - s_prev (n, V), r_new (T, 2, n, P), log_psi (n, V))."""
    T, V = logp.shape
    n, P = ids.shape
    output_length = len(yseqs[0]) - 1
    if states[0] is None:
        r_prev = torch.full((T, 2, n), LOGZERO, dtype=logp.dtype)
        r_prev[:, 1] = torch.cumsum(logp[:, blank], 0).unsqueeze(1)
        s_prev = torch.zeros(n, 1, dtype=logp.dtype)
    else:
        r_prev = torch.stack([st[0] for st in states], dim=2)              # (T, 2, n)
        s_prev = torch.tensor([[st[1]] for st in states], dtype=logp.dtype)  # (n, 1)
    x0 = logp[:, ids.reshape(-1)].view(T, n, P)                            # non-blank of id
    x1 = logp[:, blank].view(T, 1, 1).expand(T, n, P)                      # blank
    r = torch.full((T, 2, n, P), LOGZERO, dtype=logp.dtype)
    if output_length == 0:
        r[0, 0] = x0[0]
    r_sum = torch.logsumexp(r_prev, 1)                                     # (T, n)
    log_phi = r_sum.unsqueeze(2).repeat(1, 1, P)
    for h in range(n):
        last = yseqs[h][-1]
        for j in range(P):
            if int(ids[h, j]) == last:
                log_phi[:, h, j] = r_prev[:, 1, h]
    start = max(output_length, 1)
    for t in range(start, T):
        r[t, 0] = torch.logsumexp(torch.stack([r[t - 1, 0], log_phi[t - 1]]), 0) + x0[t]
        r[t, 1] = torch.logsumexp(torch.stack([r[t - 1, 0], r[t - 1, 1]]), 0) + x1[t]
    log_phi_x = torch.cat((log_phi[0].unsqueeze(0), log_phi[:-1]), dim=0) + x0
    log_psi_ = torch.logsumexp(torch.cat((log_phi_x[start:T], r[start - 1, 0].unsqueeze(0)), dim=0), dim=0)
    log_psi = torch.full((n, V), LOGZERO, dtype=logp.dtype)
    for h in range(n):
        log_psi[h, ids[h]] = log_psi_[h]
    log_psi[:, eos] = r_sum[T - 1]
    log_psi[:, blank] = LOGZERO
    return log_psi - s_prev, r, log_psi


def end_detect(ended, i, M=3, D_end=np.log(1 * np.exp(-10))):
    if len(ended) == 0:
        return False
    count = 0
    best = max(ended, key=lambda h: h.score)
    for m in range(M):
        same = [h for h in ended if len(h.yseq) == i - m]
        if same and max(same, key=lambda h: h.score).score - best.score < D_end:
            count += 1
    return count == M


def beam_search(sd, cfg, x, ctc_logp, beam_size, ctc_weight=0.1, maxlenratio=0.0):
    """BatchBeamSearch(x) for one encoded utterance x (T, D). Returns the ended hypotheses
    sorted by score (best first)."""
    V = cfg.odim
    sos = eos = V - 1
    blank = 0
    w_dec, w_ctc = 1.0 - ctc_weight, ctc_weight
    use_dec, use_ctc = w_dec != 0.0, w_ctc != 0.0
    pre_beam = int(1.5 * beam_size)
    T = x.shape[0]
    # beam_search.py:349-354
    maxlen = T if maxlenratio == 0 else (-int(maxlenratio) if maxlenratio < 0 else max(1, int(maxlenratio * T)))
    running = [Hyp([sos], 0.0, {k: 0.0 for k, u in (("decoder", use_dec), ("ctc", use_ctc)) if u}, None, 0.0)]
    ended = []
    for i in range(maxlen):
        n = len(running)
        ys = torch.tensor([h.yseq for h in running])
        weighted = torch.zeros(n, V, dtype=ctc_logp.dtype)
        if use_dec:
            with torch.no_grad():
                dec = decoder_one_step(sd, cfg, ys, x.unsqueeze(0).expand(n, -1, -1))   # (n, V)
            weighted = weighted + w_dec * dec
        if use_ctc:
            # pre-beam on the decoder score in the joint search; the full vocabulary without it
            ids = torch.topk(dec, pre_beam, dim=-1)[1] if use_dec else torch.arange(V).expand(n, V)
            states = [None if h.ctc_r is None else (h.ctc_r, h.ctc_s) for h in running]
            ctc_sc, r_new, log_psi = ctc_prefix_scores(ctc_logp, [h.yseq for h in running], states, ids, blank, eos)
            weighted = weighted + w_ctc * ctc_sc
        weighted = weighted + torch.tensor([h.score for h in running], dtype=weighted.dtype).unsqueeze(1)
        top = weighted.view(-1).topk(beam_size)[1]
        best = []
        for flat in top.tolist():
            p, tok = flat // V, flat % V
            h = running[p]
            sc = {}
            if use_dec:
                sc["decoder"] = h.scores["decoder"] + float(dec[p, tok])
            if not use_ctc:
                best.append(Hyp(h.yseq + [tok], float(weighted[p, tok]), sc, None, 0.0))
                continue
            pos = (ids[p] == tok).nonzero()
            col = int(pos[0, 0]) if len(pos) else P_LAST(ids)   # scoring_idmap -1 => index -1
            sc["ctc"] = h.scores["ctc"] + float(ctc_sc[p, tok])
            best.append(Hyp(h.yseq + [tok], float(weighted[p, tok]), sc, r_new[:, :, p, col].clone(),
                            float(log_psi[p, tok])))
        if i == maxlen - 1:
            best = [Hyp(h.yseq + [eos], h.score, h.scores, h.ctc_r, h.ctc_s) for h in best]
        running = []
        for h in best:
            (ended if h.yseq[-1] == eos else running).append(h)
        if maxlenratio == 0.0 and end_detect(ended, i):      # beam_search.py:369
            break
        if not running:
            break
    return sorted(ended, key=lambda h: h.score, reverse=True)


def P_LAST(ids):
    return ids.shape[1] - 1
