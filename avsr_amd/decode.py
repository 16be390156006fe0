"""Joint CTC / attention beam search on the HIP engine.

Drop-in for the decoder the reference builds with `get_beam_search_decoder`
(src/avhubert_avsr/avhubert_avsr_model.py:12-36): a `BatchBeamSearch` whose call
`bs(x)` on one encoded utterance x (T, d) returns the ended hypotheses sorted by score,
`Hypothesis.asdict()["yseq"]` starting with sos (script/evaluation.py:104-107).

Search semantics follow src/nets/batch_beam_search.py:102-349 and beam_search.py:330-456
(weights decoder 1-ctc_weight / ctc ctc_weight, length bonus and LM weight 0 => dropped,
pre-beam of int(1.5*beam) tokens on the decoder score, maxlen = T when maxlenratio = 0,
eos forced at the last step, end detection M=3, D_end=-10). Per step everything runs on
the device (decoder one-step with self-attention K/V caches and per-utterance cross-attention
K/V, pre-beam top-k, CTC prefix recursion, weighted flat top-beam, state reordering); the
host reads back only the beam's (previous hypothesis, token, scores) to manage ended
hypotheses — the reference synchronises per hypothesis instead.

Differences that do not change results: the cross-attention K/V of the memory are computed
once per utterance (the reference recomputes them every step), and the self-attention K/V
of earlier positions are cached instead of the layer outputs they are computed from.
"""
import math
from typing import Any, Dict, List, NamedTuple, Union

import numpy as np
import torch

from . import ops

LOGZERO = -10000000000.0


class Hypothesis(NamedTuple):
    """src/nets/beam_search.py:13-29"""
    yseq: torch.Tensor
    score: Union[float, torch.Tensor] = 0
    scores: Dict[str, Union[float, torch.Tensor]] = dict()
    states: Dict[str, Any] = dict()

    def asdict(self) -> dict:
        return self._replace(
            yseq=self.yseq.tolist(),
            score=float(self.score),
            scores={k: float(v) for k, v in self.scores.items()},
        )._asdict()


def end_detect(ended_hyps, i, M=3, D_end=np.log(1 * np.exp(-10))):
    """src/nets/e2e_asr_common.py:18-48"""
    if len(ended_hyps) == 0:
        return False
    count = 0
    best_hyp = sorted(ended_hyps, key=lambda x: x["score"], reverse=True)[0]
    for m in range(M):
        hyp_length = i - m
        same = [x for x in ended_hyps if len(x["yseq"]) == hyp_length]
        if len(same) > 0:
            best_same = sorted(same, key=lambda x: x["score"], reverse=True)[0]
            if best_same["score"] - best_hyp["score"] < D_end:
                count += 1
    return count == M


class BatchBeamSearch:
    """Beam search over one utterance with the decoder + CTC prefix scorers of an E2E model
    running on its HIP engine."""

    def __init__(self, e2e, beam_size: int, vocab_size: int, weights: Dict[str, float], sos: int, eos: int,
                 token_list: List[str] = None, pre_beam_ratio: float = 1.5, pre_beam_score_key: str = "decoder"):
        self.e2e = e2e
        self.beam_size = beam_size
        self.n_vocab = vocab_size
        self.weights = weights
        self.sos, self.eos = sos, eos
        self.blank = 0
        self.token_list = token_list
        self.pre_beam_size = int(pre_beam_ratio * beam_size)
        self.w_dec = float(weights.get("decoder", 0.0))
        self.w_ctc = float(weights.get("ctc", 0.0))
        if self.w_ctc == 0.0 or self.w_dec == 0.0:
            raise NotImplementedError("the HIP beam search implements the joint decoder+CTC configuration "
                                      "(0 < ctc_weight < 1) that get_beam_search_decoder builds")
        if pre_beam_score_key != "decoder" or not (self.pre_beam_size < vocab_size):
            raise NotImplementedError("pre-beam on the decoder score is the configuration the reference uses")

    def __call__(self, x, maxlenratio: float = 0.0, minlenratio: float = 0.0):
        return self.forward(x, maxlenratio, minlenratio)

    # ----------------------------------------------------------------------- per utterance
    def _prepare(self, eng, x):
        x = x.to(eng.device, eng.dtype).contiguous()
        T = x.shape[0]
        ar = eng.arena
        # CTC log-probs (ctc.py:153-160 log_softmax(ctc_lo(x)))
        cl = eng._e(T, eng.Vp)
        ops.linear_fwd(x, eng.w("ctc.ctc_lo.weight"), ar.master("ctc.ctc_lo.bias"), out=cl[:, :eng.V])
        logp = torch.empty(T, eng.V, device=eng.device, dtype=torch.float32)
        ops.log_softmax_rows(cl, eng.V, logp)
        # cross-attention K/V of the memory, once per utterance and layer
        mem = []
        for i in range(eng.dl):
            ca = f"decoder.decoders.{i}.src_attn."
            mem.append(ops.linear_fwd(x, ar.span([ca + "linear_k.weight", ca + "linear_v.weight"]),
                                      ar.span([ca + "linear_k.bias", ca + "linear_v.bias"], buf="master")))
        return x, logp, mem

    # ----------------------------------------------------------------------- decoder step
    def _decoder_step(self, eng, toks, pos, n, cache, mem, T, kidx=None, klen=None):
        """Decoder.forward_one_step for n prefixes whose last token (position pos) is toks:
        returns log-probs (n, V) fp32; appends this position's self-attention K/V to cache.
        Batched utterances: memory rows [U*T][2D], hypothesis i attends to block kidx[i] over
        klen[i] frames."""
        ar = eng.arena
        D, H = eng.dD, eng.dH
        x = eng._e(n, D)
        if eng._pe.shape[0] <= pos:
            from .engine import positional_encoding
            eng._pe = positional_encoding(2 * (pos + 1), D, eng.device)
        ops.embed_fwd(toks, eng.w("decoder.embed.0.weight"), eng._pe[pos:pos + 1], math.sqrt(D), x, 1)
        Lmax = cache.shape[3]
        for i in range(eng.dl):
            p = f"decoder.decoders.{i}."
            sa, ca, ff = p + "self_attn.", p + "src_attn.", p + "feed_forward."
            n1, _, _ = ops.layernorm_fwd(x, ar.master(p + "norm1.weight"), ar.master(p + "norm1.bias"), 1e-12)
            qkv = ops.linear_fwd(n1, ar.span([sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight"]),
                                 ar.span([sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias"], buf="master"))
            kc, vc = cache[i, 0, :n], cache[i, 1, :n]            # (n, Lmax, D)
            ops.cast(qkv[:, D:2 * D], kc[:, pos, :])
            ops.cast(qkv[:, 2 * D:], vc[:, pos, :])
            o1 = eng._e(n, D)
            ops.dec_attn(qkv[:, :D], kc, vc, o1, n=n, H=H, klen_max=pos + 1, k_bstride=Lmax * D,
                         v_bstride=Lmax * D)
            y1 = ops.linear_fwd(o1, eng.w(sa + "linear_out.weight"), ar.master(sa + "linear_out.bias"), res=x)
            n2, _, _ = ops.layernorm_fwd(y1, ar.master(p + "norm2.weight"), ar.master(p + "norm2.bias"), 1e-12)
            q2 = ops.linear_fwd(n2, eng.w(ca + "linear_q.weight"), ar.master(ca + "linear_q.bias"))
            o2 = eng._e(n, D)
            kv = mem[i]
            bs = 0 if kidx is None else T * kv.stride(0)
            ops.dec_attn(q2, kv[:, :D], kv[:, D:], o2, n=n, H=H, klen_max=T, k_bstride=bs, v_bstride=bs,
                         kidx=kidx, klen=klen)
            y2 = ops.linear_fwd(o2, eng.w(ca + "linear_out.weight"), ar.master(ca + "linear_out.bias"), res=y1)
            n3, _, _ = ops.layernorm_fwd(y2, ar.master(p + "norm3.weight"), ar.master(p + "norm3.bias"), 1e-12)
            a = ops.linear_fwd(n3, eng.w(ff + "w_1.weight"), ar.master(ff + "w_1.bias"), act=ops.L.ACT_RELU)
            x = ops.linear_fwd(a, eng.w(ff + "w_2.weight"), ar.master(ff + "w_2.bias"), res=y2)
        yn, _, _ = ops.layernorm_fwd(x, ar.master("decoder.after_norm.weight"), ar.master("decoder.after_norm.bias"),
                                     1e-12)
        logits = eng._e(n, eng.Vp)
        ops.linear_fwd(yn, eng.w("decoder.output_layer.weight"), ar.master("decoder.output_layer.bias"),
                       out=logits[:, :eng.V])
        logp = torch.empty(n, eng.V, device=eng.device, dtype=torch.float32)
        return ops.log_softmax_rows(logits, eng.V, logp)

    # ----------------------------------------------------------------------- search
    def forward(self, x, maxlenratio: float = 0.0, minlenratio: float = 0.0) -> List[Hypothesis]:
        eng = self.e2e.engine()
        dev = eng.device
        T = x.shape[0]
        if maxlenratio == 0:
            maxlen = T
        elif maxlenratio < 0:
            maxlen = -1 * int(maxlenratio)
        else:
            maxlen = max(1, int(maxlenratio * T))
        x, logp, mem = self._prepare(eng, x)
        V, P, beam = self.n_vocab, self.pre_beam_size, self.beam_size
        D = eng.dD
        Lmax = maxlen + 1
        cache = torch.empty(eng.dl, 2, beam, Lmax, D, device=dev, dtype=eng.dtype)
        cache2 = torch.empty_like(cache)
        ids = torch.empty(beam, P, device=dev, dtype=torch.int32)
        psi = torch.empty(beam, P + 1, device=dev, dtype=torch.float32)
        r_new = torch.empty(beam, P, T, 2, device=dev, dtype=torch.float32)
        r_prev = torch.empty(beam, T, 2, device=dev, dtype=torch.float32)
        r_prev2 = torch.empty_like(r_prev)
        out = {k: torch.empty(beam, device=dev, dtype=torch.int32) for k in ("prev", "tok", "col")}
        out.update({k: torch.empty(beam, device=dev, dtype=torch.float32) for k in ("score", "dec", "ctc", "s")})
        esz = cache.element_size()

        # running hypotheses (host side): token lists, scores; device side: caches, r_prev
        yseqs = [[self.sos]]
        score = [0.0]
        sc_dec, sc_ctc = [0.0], [0.0]
        s_prev = [0.0]
        first = True
        ended = []
        for i in range(maxlen):
            n = len(yseqs)
            pos = len(yseqs[0]) - 1
            toks = torch.tensor([y[-1] for y in yseqs], dtype=torch.int32).to(dev, non_blocking=True)
            dec = self._decoder_step(eng, toks, pos, n, cache, mem, T)
            ops.row_topk(dec, V, P, ids[:n])
            ops.ctc_prefix(logp, None if first else r_prev[:n], toks, ids[:n], r_new[:n], psi[:n], n=n,
                           out_len=pos, blank=self.blank, eos=self.eos)
            sp = torch.tensor(s_prev, dtype=torch.float32).to(dev, non_blocking=True)
            scv = torch.tensor(score, dtype=torch.float32).to(dev, non_blocking=True)
            nb = min(beam, n * V)
            ops.beam_select(dec, V, ids[:n], psi[:n], sp, scv, out, n=n, beam=nb, blank=self.blank, eos=self.eos,
                            w_dec=self.w_dec, w_ctc=self.w_ctc)
            res = {k: v[:nb].cpu() for k, v in out.items()}     # the one host sync per step
            prev, tok, col = res["prev"].tolist(), res["tok"].tolist(), res["col"].tolist()
            # new hypotheses (batch_beam_search.py:228-260)
            new = []
            for j in range(nb):
                h = prev[j]
                new.append(dict(yseq=yseqs[h] + [tok[j]], score=float(res["score"][j]),
                                dec=sc_dec[h] + float(res["dec"][j]), ctc=sc_ctc[h] + float(res["ctc"][j]),
                                s=float(res["s"][j]), src=h, col=col[j]))
            # post_process (batch_beam_search.py:262-349)
            if i == maxlen - 1:
                for hyp in new:
                    hyp["yseq"] = hyp["yseq"] + [self.eos]
            keep = []
            for hyp in new:
                if hyp["yseq"][-1] == self.eos:
                    ended.append(self._make_hyp(hyp))
                else:
                    keep.append(hyp)
            # beam_search.py:369: end detection only when the length limit is the input length
            if maxlenratio == 0.0 and end_detect([h.asdict() for h in ended], i):
                break
            if not keep:
                break
            # reorder the device state of the surviving hypotheses
            m = len(keep)
            src_idx = torch.tensor([hyp["src"] for hyp in keep], dtype=torch.int32).to(dev, non_blocking=True)
            rsel = torch.tensor([hyp["src"] * P + hyp["col"] for hyp in keep], dtype=torch.int32).to(dev, non_blocking=True)
            row = Lmax * D * esz
            ops.gather_rows(cache, cache2, src_idx, groups=eng.dl * 2, n=m, row_bytes=(pos + 1) * D * esz,
                            src_gstride=beam * row, src_rstride=row, dst_gstride=beam * row, dst_rstride=row)
            cache, cache2 = cache2, cache
            ops.gather_rows(r_new, r_prev2, rsel, groups=1, n=m, row_bytes=T * 2 * 4, src_gstride=0,
                            src_rstride=T * 2 * 4, dst_gstride=0, dst_rstride=T * 2 * 4)
            r_prev, r_prev2 = r_prev2, r_prev
            first = False
            yseqs = [hyp["yseq"] for hyp in keep]
            score = [hyp["score"] for hyp in keep]
            sc_dec = [hyp["dec"] for hyp in keep]
            sc_ctc = [hyp["ctc"] for hyp in keep]
            s_prev = [hyp["s"] for hyp in keep]
        nbest = sorted(ended, key=lambda h: float(h.score), reverse=True)
        if len(nbest) == 0:
            return [] if minlenratio < 0.1 else self.forward(x, maxlenratio, max(0.0, minlenratio - 0.1))
        return nbest

    # ----------------------------------------------------------------- batched utterances
    def decode_batch(self, xs, maxlenratio: float = 0.0, minlenratio: float = 0.0):
        """Beam search of several utterances at once: xs = list of encoded utterances (T_u, d).
        Every step runs the decoder, pre-beam, CTC prefix scoring and the per-utterance beam
        selection for all running hypotheses of all utterances in the same launches (the
        hypotheses of utterance u are rows [seg[u], seg[u+1])), with one host read-back per
        step. Per utterance the search is exactly `self(x)`: same scores, same stopping rules
        (maxlen = T_u, end detection, eos forced at the last step); an utterance that finishes
        leaves the batch. Returns one n-best list per utterance."""
        eng = self.e2e.engine()
        dev = eng.device
        U = len(xs)
        if U == 0:
            return []
        Ts = [int(x.shape[0]) for x in xs]
        Tm = max(Ts)
        maxlens = [T if maxlenratio == 0 else (-int(maxlenratio) if maxlenratio < 0 else max(1, int(maxlenratio * T)))
                   for T in Ts]
        D, V, P, beam = eng.dD, self.n_vocab, self.pre_beam_size, self.beam_size
        ar = eng.arena
        # padded memory [U][Tm][D] -> CTC log-probs [U][Tm][V] and per-layer cross K/V [U*Tm][2D]
        xp = torch.zeros(U, Tm, D, device=dev, dtype=eng.dtype)
        for u, x in enumerate(xs):      # (the cast kernel converts fp32 encoder outputs to bf16 if needed)
            ops.cast(x.to(dev).reshape(Ts[u], D).contiguous(), xp[u, :Ts[u]])
        x2 = xp.view(U * Tm, D)
        cl = eng._e(U * Tm, eng.Vp)
        ops.linear_fwd(x2, eng.w("ctc.ctc_lo.weight"), ar.master("ctc.ctc_lo.bias"), out=cl[:, :eng.V])
        logp = torch.empty(U, Tm, eng.V, device=dev, dtype=torch.float32)
        ops.log_softmax_rows(cl, eng.V, logp.view(U * Tm, eng.V))
        mem = []
        for i in range(eng.dl):
            ca = f"decoder.decoders.{i}.src_attn."
            mem.append(ops.linear_fwd(x2, ar.span([ca + "linear_k.weight", ca + "linear_v.weight"]),
                                      ar.span([ca + "linear_k.bias", ca + "linear_v.bias"], buf="master")))
        tlen = torch.tensor(Ts, dtype=torch.int32).to(dev)
        NM = U * beam
        Lmax = max(maxlens) + 1
        cache = torch.empty(eng.dl, 2, NM, Lmax, D, device=dev, dtype=eng.dtype)
        cache2 = torch.empty_like(cache)
        ids = torch.empty(NM, P, device=dev, dtype=torch.int32)
        psi = torch.empty(NM, P + 1, device=dev, dtype=torch.float32)
        r_new = torch.empty(NM, P, Tm, 2, device=dev, dtype=torch.float32)
        r_prev = torch.empty(NM, Tm, 2, device=dev, dtype=torch.float32)
        r_prev2 = torch.empty_like(r_prev)
        out = {k: torch.empty(NM, device=dev, dtype=torch.int32) for k in ("prev", "tok", "col")}
        out.update({k: torch.empty(NM, device=dev, dtype=torch.float32) for k in ("score", "dec", "ctc", "s")})
        esz = cache.element_size()
        # running hypotheses, grouped by utterance: host lists
        run = [[dict(yseq=[self.sos], score=0.0, dec=0.0, ctc=0.0, s=0.0)] for _ in range(U)]
        active = list(range(U))
        ended = [[] for _ in range(U)]
        first = True
        i = 0
        while active:
            hyps = [(u, h) for u in active for h in run[u]]
            n = len(hyps)
            pos = i
            seg_h = [0]
            for u in active:
                seg_h.append(seg_h[-1] + len(run[u]))
            host = torch.tensor([h["yseq"][-1] for _, h in hyps] + [u for u, _ in hyps] +
                                [Ts[u] for u, _ in hyps] + seg_h, dtype=torch.int32)
            dv = host.to(dev, non_blocking=True)
            toks, uidx, klen, seg = dv[:n], dv[n:2 * n], dv[2 * n:3 * n], dv[3 * n:]
            dec = self._decoder_step(eng, toks, pos, n, cache, mem, Tm, kidx=uidx, klen=klen)
            ops.row_topk(dec, V, P, ids[:n])
            ops.ctc_prefix(logp, None if first else r_prev[:n], toks, ids[:n], r_new[:n], psi[:n], n=n, out_len=pos,
                           blank=self.blank, eos=self.eos, uidx=uidx, tlen=tlen)
            fv = torch.tensor([h["s"] for _, h in hyps] + [h["score"] for _, h in hyps], dtype=torch.float32)
            fv = fv.to(dev, non_blocking=True)
            ops.beam_select(dec, V, ids[:n], psi[:n], fv[:n], fv[n:], out, n=n, beam=beam, blank=self.blank,
                            eos=self.eos, w_dec=self.w_dec, w_ctc=self.w_ctc, seg=seg)
            nsel = len(active) * beam
            res = {k: v[:nsel].cpu() for k, v in out.items()}     # the one host sync per step
            prev, tok, col = res["prev"].tolist(), res["tok"].tolist(), res["col"].tolist()
            keep_src, keep_col, still = [], [], []
            for a, u in enumerate(active):
                new = []
                for r in range(beam):
                    o = a * beam + r
                    g = prev[o]
                    h = hyps[g][1]
                    new.append(dict(yseq=h["yseq"] + [tok[o]], score=float(res["score"][o]),
                                    dec=h["dec"] + float(res["dec"][o]), ctc=h["ctc"] + float(res["ctc"][o]),
                                    s=float(res["s"][o]), src=g, col=col[o]))
                if i == maxlens[u] - 1:
                    for hyp in new:
                        hyp["yseq"] = hyp["yseq"] + [self.eos]
                keep = []
                for hyp in new:
                    if hyp["yseq"][-1] == self.eos:
                        ended[u].append(self._make_hyp(hyp))
                    else:
                        keep.append(hyp)
                done = (maxlenratio == 0.0 and end_detect([h.asdict() for h in ended[u]], i)) or not keep \
                    or i >= maxlens[u] - 1
                if done:
                    run[u] = []
                    continue
                run[u] = keep
                still.append(u)
                keep_src += [hyp["src"] for hyp in keep]
                keep_col += [hyp["src"] * P + hyp["col"] for hyp in keep]
            active = still
            if not active:
                break
            m = len(keep_src)
            idx = torch.tensor(keep_src + keep_col, dtype=torch.int32).to(dev, non_blocking=True)
            row = Lmax * D * esz
            ops.gather_rows(cache, cache2, idx[:m], groups=eng.dl * 2, n=m, row_bytes=(pos + 1) * D * esz,
                            src_gstride=NM * row, src_rstride=row, dst_gstride=NM * row, dst_rstride=row)
            cache, cache2 = cache2, cache
            ops.gather_rows(r_new, r_prev2, idx[m:], groups=1, n=m, row_bytes=Tm * 2 * 4, src_gstride=0,
                            src_rstride=Tm * 2 * 4, dst_gstride=0, dst_rstride=Tm * 2 * 4)
            r_prev, r_prev2 = r_prev2, r_prev
            first = False
            i += 1
        results = []
        for u in range(U):
            nbest = sorted(ended[u], key=lambda h: float(h.score), reverse=True)
            if not nbest and minlenratio >= 0.1:
                nbest = self.forward(xs[u], maxlenratio, max(0.0, minlenratio - 0.1))
            results.append(nbest)
        return results

    @staticmethod
    def _make_hyp(hyp):
        return Hypothesis(yseq=torch.tensor(hyp["yseq"], dtype=torch.int64),
                          score=torch.tensor(hyp["score"], dtype=torch.float32),
                          scores={"decoder": torch.tensor(hyp["dec"], dtype=torch.float32),
                                  "ctc": torch.tensor(hyp["ctc"], dtype=torch.float32)},
                          states={})


def get_beam_search_decoder(model, token_list, ctc_weight=0.1, beam_size=3):
    """src/avhubert_avsr/avhubert_avsr_model.py:12-36 — `model` is the E2E (`AVHubertAVSR.avsr`)."""
    weights = {"decoder": 1.0 - ctc_weight, "ctc": ctc_weight, "lm": 0.0, "length_bonus": 0.0}
    return BatchBeamSearch(model, beam_size=beam_size, vocab_size=len(token_list), weights=weights, sos=model.sos,
                           eos=model.eos, token_list=token_list,
                           pre_beam_score_key=None if ctc_weight == 1.0 else "decoder")
