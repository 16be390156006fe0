"""Joint CTC / attention beam search on the HIP engine.

Drop-in for the decoder the reference builds with `get_beam_search_decoder`
(src/avhubert_avsr/avhubert_avsr_model.py:12-36): a `BatchBeamSearch` whose call
`bs(x)` on one encoded utterance x (T, d) returns the ended hypotheses sorted by score,
`Hypothesis.asdict()["yseq"]` starting with sos (script/evaluation.py:104-107).

Search semantics follow src/nets/batch_beam_search.py:102-349 and beam_search.py:330-456
(weights decoder 1-ctc_weight / ctc ctc_weight, length bonus and LM weight 0 => dropped,
pre-beam of int(1.5*beam) tokens on the decoder score, maxlen = T when maxlenratio = 0,
eos forced at the last step, end detection M=3, D_end=-10). Everything runs on the device,
bookkeeping included (decoder one-step with an ancestry-indexed self-attention K/V cache and
per-utterance cross-attention K/V, pre-beam top-k, CTC prefix recursion, weighted flat
top-beam, running scores, back-pointers, ended-hypothesis records, end detection), and every
step after the first is one HIP-graph replay; the host reads a finished-utterance count every
8 steps and the history once at the end — the reference synchronises per hypothesis.

Differences that do not change results: the cross-attention K/V of the memory are computed
once per utterance (the reference recomputes them every step), the self-attention K/V of
earlier positions are cached instead of the layer outputs they are computed from (rows of
step j at cache row j*R + r, reached through each hypothesis's ancestry table instead of
being copied on every reorder), and finished hypotheses stay in the batch as dead rows.

The two ends of the CTC-weight range are the configurations the reference builds with one
scorer (a scorer of weight 0 is dropped, beam_search.py:69-73): ctc_weight = 0 searches on the
decoder alone (no partial scorer, so no pre-beam: every token of every row is a candidate);
ctc_weight = 1 on the CTC prefix scorer alone over the full vocabulary (pre_beam_score_key None,
no decoder step at all): psi of every token in chunks of 64, then the row's top int(1.5*beam)
tokens by psi (a superset of every token the flat top-beam can pick from that row, since the row
offset is common) get their CTC states.
"""
import math
from typing import Any, Dict, List, NamedTuple, Union

import numpy as np
import torch

from . import ops

LOGZERO = -10000000000.0
# fp32 decode: LayerNorms folded into the linears they feed (the few-row kernel's LN prologue)
FOLD_LN = True
D_END = np.log(1 * np.exp(-10))          # end_detect's threshold (e2e_asr_common.py:18)


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


def end_detect(ended_hyps, i, M=3, D_end=D_END):
    """src/nets/e2e_asr_common.py:18-48 (host form; the search evaluates it on the device,
    decode.hip beam_post_kernel, over the per-length best ended scores)"""
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


_CAPTURE_STREAMS = {}


def _capture_stream(dev):
    """one graph-capture stream per device for every search (its workspaces are reused)"""
    s = _CAPTURE_STREAMS.get(dev)
    if s is None:
        s = _CAPTURE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


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
        self.use_dec, self.use_ctc = self.w_dec != 0.0, self.w_ctc != 0.0
        if not (self.use_dec or self.use_ctc):
            raise NotImplementedError("no scorer with a non-zero weight")
        if self.use_ctc and pre_beam_score_key is not None and pre_beam_score_key != "decoder":
            raise NotImplementedError(f"pre-beam on {pre_beam_score_key!r}: the reference builds 'decoder' or None")
        if self.use_ctc and not self.use_dec and pre_beam_score_key == "decoder":
            raise KeyError("decoder is not a scorer (weight 0): pre_beam_score_key must be None")   # beam_search.py:92-97
        if self.use_ctc and self.use_dec and (pre_beam_score_key is None or not self.pre_beam_size < vocab_size):
            raise NotImplementedError("the joint search pre-beams on the decoder score, as the reference configures it")

    def __call__(self, x, maxlenratio: float = 0.0, minlenratio: float = 0.0):
        return self.forward(x, maxlenratio, minlenratio)

    def _cross_group(self, Tm):
        """hypotheses of one utterance per cross-attention workgroup: the beam, while its
        [beam][Tm] scores fit the grouped kernel's LDS (about 2.7 k frames at beam 5)"""
        G = self.beam_size if self.beam_size <= 8 else 1
        return G if ops.dec_attn_group_fits(Tm, G) else 1

    # ----------------------------------------------------------------------- decoder step
    def _decoder_step(self, eng, st):
        """Decoder.forward_one_step for the R rows of the search state `st` (position and
        tokens on the device): returns log-probs (R, V) fp32. This step's self-attention K / V
        go to cache rows pos*R + r; key j of row r is cache row anc[r][j] (its ancestry), the
        memory of row r is utterance r // beam over klen[r] frames."""
        ar = eng.arena
        D, H, R = eng.dD, eng.dH, st["R"]
        pos, cache, anc = st["pos"], st["cache"], st["anc_in"]
        x = eng._e(R, D)
        ops.embed_fwd(st["tok"], eng.w("decoder.embed.0.weight"), eng._pe, math.sqrt(D), x, 1, pe_row=pos)
        Tm = st["Tm"]
        fold = st.get("fold")
        for i in range(eng.dl):
            p = f"decoder.decoders.{i}."
            sa, ca, ff = p + "self_attn.", p + "src_attn.", p + "feed_forward."
            kc, vc = cache[i, 0], cache[i, 1]               # (Lmax * R, D): rows step * R + r
            if fold is not None:       # norm1 folded into the QKV linear, K / V appended to the cache (one launch)
                Wg, bb, c1 = fold[i]["qkv"]
                qkv = ops.linear_fwd(x, Wg, bb, ln=(c1, 1e-12), kv=(kc, vc, pos, R))
            else:
                n1, _, _ = ops.layernorm_fwd(x, ar.master(p + "norm1.weight"), ar.master(p + "norm1.bias"), 1e-12)
                qkv = ops.linear_fwd(n1, ar.span([sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight"]),
                                     ar.span([sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias"],
                                             buf="master"))
                ops.beam_kv_put(qkv, kc, vc, pos, R, D)
            o1 = eng._e(R, D)
            ops.dec_attn(qkv[:, :D], kc, vc, o1, n=R, H=H, klen_max=st["Lmax"], k_bstride=0, v_bstride=0,
                         klen=st["klen_self"], kmap=anc)
            y1 = ops.linear_fwd(o1, eng.w(sa + "linear_out.weight"), ar.master(sa + "linear_out.bias"), res=x)
            if fold is not None:
                Wg, bb, c1 = fold[i]["q2"]
                q2 = ops.linear_fwd(y1, Wg, bb, ln=(c1, 1e-12))
            else:
                n2, _, _ = ops.layernorm_fwd(y1, ar.master(p + "norm2.weight"), ar.master(p + "norm2.bias"), 1e-12)
                q2 = ops.linear_fwd(n2, eng.w(ca + "linear_q.weight"), ar.master(ca + "linear_q.bias"))
            o2 = eng._e(R, D)
            kv = st["mem"][i]
            ops.dec_attn(q2, kv[:, :D], kv[:, D:], o2, n=R, H=H, klen_max=Tm, k_bstride=Tm * kv.stride(0),
                         v_bstride=Tm * kv.stride(0), kidx=st["uidx"], klen=st["klen_mem"],
                         group=self._cross_group(Tm), ksplit=2)
            y2 = ops.linear_fwd(o2, eng.w(ca + "linear_out.weight"), ar.master(ca + "linear_out.bias"), res=y1)
            if fold is not None:
                Wg, bb, c1 = fold[i]["ff1"]
                a = ops.linear_fwd(y2, Wg, bb, act=ops.L.ACT_RELU, ln=(c1, 1e-12))
            else:
                n3, _, _ = ops.layernorm_fwd(y2, ar.master(p + "norm3.weight"), ar.master(p + "norm3.bias"), 1e-12)
                a = ops.linear_fwd(n3, eng.w(ff + "w_1.weight"), ar.master(ff + "w_1.bias"), act=ops.L.ACT_RELU)
            x = ops.linear_fwd(a, eng.w(ff + "w_2.weight"), ar.master(ff + "w_2.bias"), res=y2)
        yn, _, _ = ops.layernorm_fwd(x, ar.master("decoder.after_norm.weight"), ar.master("decoder.after_norm.bias"),
                                     1e-12)
        logits = eng._e(R, eng.Vp)
        ops.linear_fwd(yn, eng.w("decoder.output_layer.weight"), ar.master("decoder.output_layer.bias"),
                       out=logits[:, :eng.V])
        logp = torch.empty(R, eng.V, device=eng.device, dtype=torch.float32)
        # log-probs and the pre-beam (top-P decoder tokens per row) in one pass
        return ops.log_softmax_topk(logits, eng.V, logp, self.pre_beam_size, st["ids"])

    def _fold_layernorms(self, eng):
        """fp32 decode: each decoder layer's norm1 / norm2 / norm3 folded into the linear it feeds
        (QKV, cross-attention query, FFN w_1): ops.fold_layernorm weights for the few-row kernel's
        LayerNorm prologue (one launch instead of two per pair). Prepared per search (the weights may
        have changed since the last one); None where the prologue does not apply (bf16, D > 1024)."""
        if eng.dtype != torch.float32 or eng.dD > 1024 or eng.dD % 16:
            return None
        ar = eng.arena
        out = []
        for i in range(eng.dl):
            p = f"decoder.decoders.{i}."
            sa, ca, ff = p + "self_attn.", p + "src_attn.", p + "feed_forward."

            def f(W, b, n):
                return ops.fold_layernorm(W, b, ar.master(n + ".weight"), ar.master(n + ".bias"))
            out.append(dict(
                qkv=f(ar.span([sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight"]),
                      ar.span([sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias"], buf="master"),
                      p + "norm1"),
                q2=f(eng.w(ca + "linear_q.weight"), ar.master(ca + "linear_q.bias"), p + "norm2"),
                ff1=f(eng.w(ff + "w_1.weight"), ar.master(ff + "w_1.bias"), p + "norm3")))
        return out

    def _ctc_full_vocab(self, st, r_prev):
        """ctc_weight = 1: psi of every token (chunks of 64 ids through the prefix kernel), then
        the row's top-P tokens by psi into st["ids"] (the kernel's psi of a token does not depend
        on the other ids of its launch)"""
        R, V = st["R"], self.n_vocab
        kw = dict(n=R, out_len=0, out_len_dev=st["pos"], blank=self.blank, eos=self.eos, uidx=st["uidx"], tlen=st["tlen"])
        pf = st["psi_full"]
        for c in range(st["vchunks"].shape[0]):
            ops.ctc_prefix(st["logp"], r_prev, st["tok"], st["vchunks"][c], st["r_scr"], st["psi_c"], **kw)
            pf[:, c * 64:(c + 1) * 64].copy_(st["psi_c"][:, :64])
        ops.row_topk(pf, V, self.pre_beam_size, st["ids"])

    def _step(self, eng, st, first, k):
        """one search step on the device (no host sync): decoder, pre-beam, CTC prefix scores,
        per-utterance beam selection, bookkeeping, state reorder. k = 0 / 1 picks the ancestry
        and CTC-state ping-pong buffers (read k, write 1 - k)."""
        R, P, beam = st["R"], self.pre_beam_size, self.beam_size
        st["anc_in"] = st["anc"][k]
        ops.beam_step_prep(R, st["pos"], st["anc"][k], st["klen_self"])
        # decoder log-probs + the pre-beam ids; without a decoder scorer its score is 0
        dec = self._decoder_step(eng, st) if self.use_dec else st["dec0"]
        if self.use_ctc:
            r_prev = None if first else st["r_prev"][k]
            if not self.use_dec:
                self._ctc_full_vocab(st, r_prev)
            ops.ctc_prefix(st["logp"], r_prev, st["tok"], st["ids"], st["r_new"], st["psi"], n=R, out_len=0,
                           out_len_dev=st["pos"], blank=self.blank, eos=self.eos, uidx=st["uidx"], tlen=st["tlen"])
        out = st["out"]
        ops.beam_select(dec, self.n_vocab, st["ids"], st["psi"], st["s_prev"], st["score"], out, n=R, beam=beam,
                        blank=self.blank, eos=self.eos, w_dec=self.w_dec, w_ctc=self.w_ctc, seg=st["seg"])
        ops.beam_post(U=st["U"], beam=beam, P=P, R=R, Lmax=st["Lmax"], steps_cap=st["steps"], eos=self.eos,
                      end_detect=st["end_detect"], d_end=float(D_END), pos=st["pos"], maxlen=st["maxlen"],
                      sel_prev=out["prev"], sel_tok=out["tok"], sel_col=out["col"], sel_score=out["score"],
                      sel_dec=out["dec"], sel_ctc=out["ctc"], sel_s=out["s"], tok=st["tok"], score=st["score"],
                      sdec=st["sdec"], sctc=st["sctc"], s_prev=st["s_prev"], src=st["src"], bp_prev=st["bp_prev"],
                      bp_tok=st["bp_tok"], end_flag=st["end_flag"], end_score=st["end_score"], end_dec=st["end_dec"],
                      end_ctc=st["end_ctc"], best_len=st["best_len"], best_end=st["best_end"], done=st["done"])
        Lm, Tm = st["Lmax"], st["Tm"]
        ops.gather_rows(st["anc"][k], st["anc"][1 - k], st["src"][:R], groups=1, n=R, row_bytes=Lm * 4,
                        src_gstride=0, src_rstride=Lm * 4, dst_gstride=0, dst_rstride=Lm * 4)
        if self.use_ctc:
            ops.gather_rows(st["r_new"], st["r_prev"][1 - k], st["src"][R:], groups=1, n=R, row_bytes=Tm * 2 * 4,
                            src_gstride=0, src_rstride=Tm * 2 * 4, dst_gstride=0, dst_rstride=Tm * 2 * 4)

    # ----------------------------------------------------------------------- search
    def forward(self, x, maxlenratio: float = 0.0, minlenratio: float = 0.0) -> List[Hypothesis]:
        """the reference's call form bs(x) on one encoded utterance (T, d)"""
        return self.decode_batch([x], maxlenratio, minlenratio)[0]

    def decode_batch(self, xs, maxlenratio: float = 0.0, minlenratio: float = 0.0):
        """Beam search of U utterances at once: xs = list of encoded utterances (T_u, d). Per
        utterance the search is exactly `self(x)` of the reference (batch_beam_search.py:102-349,
        beam_search.py:330-456): same scores, same stopping rules (maxlen = T_u, end detection,
        eos forced at the last step). The whole search state lives on the device in a fixed
        geometry of U x beam rows (a finished hypothesis or utterance becomes a dead row with
        score -inf, which no selection picks — the same outcome as the reference removing it);
        the first step runs eagerly, every later step is ONE replay of a captured HIP graph (two
        graphs: the ancestry / CTC-state ping-pong buffers alternate), the host only reads the
        count of finished utterances every few steps and the history once at the end. Returns
        one n-best list per utterance."""
        eng = self.e2e.engine()
        dev = eng.device
        U = len(xs)
        if U == 0:
            return []
        Ts = [int(x.shape[0]) for x in xs]
        Tm = max(Ts)
        maxlens = [T if maxlenratio == 0 else (-int(maxlenratio) if maxlenratio < 0 else max(1, int(maxlenratio * T)))
                   for T in Ts]
        D, P, beam = eng.dD, self.pre_beam_size, self.beam_size
        ar = eng.arena
        # padded memory [U][Tm][D] -> CTC log-probs [U][Tm][V] and per-layer cross K/V [U*Tm][2D]
        xp = torch.zeros(U, Tm, D, device=dev, dtype=eng.dtype)
        for u, x in enumerate(xs):      # (the cast kernel converts fp32 encoder outputs to bf16 if needed)
            ops.cast(x.to(dev).reshape(Ts[u], D).contiguous(), xp[u, :Ts[u]])
        # the CTC head and the cross-attention K / V projections run per utterance (M = T_u rows,
        # as in the one-utterance call): the few-row and tiled GEMM cores round differently, so
        # one launch over all U * Tm rows would make an utterance's scores depend on the batch
        cl = torch.zeros(U * Tm, eng.Vp, device=dev, dtype=eng.dtype)
        mem = [torch.zeros(U * Tm, 2 * D, device=dev, dtype=eng.dtype) for _ in range(eng.dl)]
        for u in range(U):
            xu, r0 = xp[u, :Ts[u]], u * Tm
            ops.linear_fwd(xu, eng.w("ctc.ctc_lo.weight"), ar.master("ctc.ctc_lo.bias"), out=cl[r0:r0 + Ts[u], :eng.V])
            for i in range(eng.dl):
                ca = f"decoder.decoders.{i}.src_attn."
                ops.linear_fwd(xu, ar.span([ca + "linear_k.weight", ca + "linear_v.weight"]),
                               ar.span([ca + "linear_k.bias", ca + "linear_v.bias"], buf="master"),
                               out=mem[i][r0:r0 + Ts[u]])
        logp = torch.empty(U, Tm, eng.V, device=dev, dtype=torch.float32)
        ops.log_softmax_rows(cl, eng.V, logp.view(U * Tm, eng.V))
        steps = max(maxlens)
        Lmax = steps + 1
        eng.ensure_pe(Lmax)
        R = U * beam
        i32 = dict(device=dev, dtype=torch.int32)
        f32 = dict(device=dev, dtype=torch.float32)
        f64 = dict(device=dev, dtype=torch.float64)
        rows = torch.arange(R, dtype=torch.int32)
        score0 = torch.full((R,), float("-inf"))
        score0[::beam] = 0.0                  # one live hypothesis (sos) per utterance
        st = dict(
            U=U, R=R, Lmax=Lmax, Tm=Tm, steps=steps, end_detect=int(maxlenratio == 0.0), mem=mem, logp=logp,
            pos=torch.zeros(1, **i32), maxlen=torch.tensor(maxlens, dtype=torch.int32).to(dev),
            tok=torch.full((R,), self.sos, **i32), score=score0.to(dev),
            sdec=torch.zeros(R, **f64), sctc=torch.zeros(R, **f64), s_prev=torch.zeros(R, **f32),
            cache=torch.empty(eng.dl, 2, Lmax * R, D, device=dev, dtype=eng.dtype),
            anc=[torch.zeros(R, Lmax, **i32), torch.zeros(R, Lmax, **i32)], klen_self=torch.empty(R, **i32),
            uidx=(rows // beam).to(dev), klen_mem=torch.tensor(Ts, dtype=torch.int32)[rows // beam].to(dev),
            tlen=torch.tensor(Ts, dtype=torch.int32).to(dev),
            seg=(torch.arange(U + 1, dtype=torch.int32) * beam).to(dev),
            ids=torch.empty(R, P, **i32), psi=torch.empty(R, P + 1, **f32),
            r_new=torch.empty(R, P, Tm, 2, **f32), r_prev=[torch.empty(R, Tm, 2, **f32), torch.empty(R, Tm, 2, **f32)],
            out={**{k: torch.empty(R, **i32) for k in ("prev", "tok", "col")},
                 **{k: torch.empty(R, **f32) for k in ("score", "dec", "ctc", "s")}},
            src=torch.empty(2 * R, **i32),
            bp_prev=torch.zeros(steps, R, **i32), bp_tok=torch.zeros(steps, R, **i32),
            end_flag=torch.zeros(steps, R, **i32), end_score=torch.zeros(steps, R, **f32),
            end_dec=torch.zeros(steps, R, **f64), end_ctc=torch.zeros(steps, R, **f64),
            best_len=torch.full((U, Lmax + 3), float("-inf"), **f32), best_end=torch.full((U,), float("-inf"), **f32),
            done=torch.zeros(U + 1, **i32), fold=self._fold_layernorms(eng) if FOLD_LN and self.use_dec else None)
        if not self.use_ctc:
            st["psi"].zero_()                 # w_ctc = 0 multiplies it: keep it finite
        if not self.use_dec:
            st["dec0"] = torch.zeros(R, eng.V, **f32)
            nch = -(-self.n_vocab // 64)
            ids = torch.arange(nch * 64, dtype=torch.int32)
            ids[ids >= self.n_vocab] = self.blank          # padding ids: blank (psi = LOGZERO)
            st["vchunks"] = ids.view(nch, 1, 64).expand(nch, R, 64).contiguous().to(dev)
            st["psi_c"] = torch.empty(R, 65, **f32)
            st["r_scr"] = torch.empty(R, 64, Tm, 2, **f32)
            st["psi_full"] = torch.empty(R, nch * 64, **f32)
        self._step(eng, st, True, 0)           # step 0: CTC state from scratch; reads ancestry 0, writes 1
        if steps > 1:
            graphs = self._capture(eng, st)
            done_host = st["done"][U:]
            for i in range(1, steps):
                graphs[i & 1].replay()         # step i reads ping-pong buffer i & 1
                if i % 8 == 0 and int(done_host.item()) == U:
                    break
        torch.cuda.current_stream(dev).synchronize()
        return self._collect(st, xs, maxlenratio, minlenratio)

    def _capture(self, eng, st):
        """two graphs of the generic step (k = 0, 1): capture records, it does not run. The
        capture stream is one long-lived stream per device, and its workspaces (split-K arrival
        counters, which must start at zero, and the dec_attn partials) are created eagerly
        before the capture: a zero-fill recorded inside graph 0 would never run before graph 1's
        first replay."""
        dev = eng.device
        graphs = []
        s = _capture_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            ops.reserve_stream_workspaces(dev, ops.dec_attn_ws_floats(st["R"], eng.dH, self._cross_group(st["Tm"]), 2))
        for k in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._step(eng, st, False, k)
            graphs.append(g)
        torch.cuda.current_stream(dev).wait_stream(s)
        return graphs

    def _collect(self, st, xs, maxlenratio, minlenratio):
        """ended hypotheses from the device history, per utterance in the reference's order
        (step, then selection rank), yseq rebuilt from the back-pointers"""
        U, R, beam = st["U"], st["R"], self.beam_size
        n = min(int(st["pos"].item()), st["steps"])
        bp_prev = st["bp_prev"][:n].cpu().numpy()
        bp_tok = st["bp_tok"][:n].cpu().numpy()
        flag = st["end_flag"][:n].cpu().numpy()
        esc = st["end_score"][:n].cpu().numpy()
        edec = st["end_dec"][:n].cpu().numpy()
        ectc = st["end_ctc"][:n].cpu().numpy()
        ended = [[] for _ in range(U)]
        for i in range(n):
            for r in np.nonzero(flag[i])[0].tolist():
                toks = [int(bp_tok[i, r])]
                h = int(bp_prev[i, r])
                for j in range(i - 1, -1, -1):
                    toks.append(int(bp_tok[j, h]))
                    h = int(bp_prev[j, h])
                yseq = [self.sos] + toks[::-1] + ([self.eos] if flag[i, r] == 2 else [])
                ended[r // beam].append(self._make_hyp(dict(yseq=yseq, score=float(esc[i, r]), dec=float(edec[i, r]),
                                                            ctc=float(ectc[i, r])), self.use_dec, self.use_ctc))
        results = []
        for u in range(U):
            nbest = sorted(ended[u], key=lambda h: float(h.score), reverse=True)
            if not nbest and minlenratio >= 0.1:
                nbest = self.forward(xs[u], maxlenratio, max(0.0, minlenratio - 0.1))
            results.append(nbest)
        return results

    @staticmethod
    def _make_hyp(hyp, use_dec=True, use_ctc=True):
        """the reference's Hypothesis: scores of the scorers in the search only"""
        scores = {}
        if use_dec:
            scores["decoder"] = torch.tensor(hyp["dec"], dtype=torch.float32)
        if use_ctc:
            scores["ctc"] = torch.tensor(hyp["ctc"], dtype=torch.float32)
        return Hypothesis(yseq=torch.tensor(hyp["yseq"], dtype=torch.int64),
                          score=torch.tensor(hyp["score"], dtype=torch.float32), scores=scores, states={})


def get_beam_search_decoder(model, token_list, ctc_weight=0.1, beam_size=3):
    """src/avhubert_avsr/avhubert_avsr_model.py:12-36 — `model` is the E2E (`AVHubertAVSR.avsr`)."""
    weights = {"decoder": 1.0 - ctc_weight, "ctc": ctc_weight, "lm": 0.0, "length_bonus": 0.0}
    return BatchBeamSearch(model, beam_size=beam_size, vocab_size=len(token_list), weights=weights, sos=model.sos,
                           eos=model.eos, token_list=token_list,
                           pre_beam_score_key=None if ctc_weight == 1.0 else "decoder")
