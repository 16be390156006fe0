"""The reference's module-level call surface, run on the HIP engine.

Callers of the reference reach the model through three sub-modules of `AVHubertAVSR.avsr`
(script/evaluation.py:96-108, src/avhubert_avsr/avhubert_avsr_model.py:12-36):

  encoder(input_features, attention_mask=None, video=...) -> BaseModelOutput
        src/nets/backend/backbones/avhubert.py:546-561
  decoder.forward / forward_one_step / score / batch_score
        src/nets/backend/transformer/decoder.py:122-227
  ctc.forward / log_softmax / softmax / argmax
        src/nets/backend/ctc.py:83-180

The functions here implement those entry points on an `Engine` (avsr_amd.engine); the
parameter-holder modules of avsr_amd.nets.modules forward to them. Semantics follow the
reference, including its state format: the decoder cache / scorer state of one hypothesis is
the list of per-layer outputs (l, D) for every prefix position (decoder.py:166-180), so a
reference-style beam search can drive this decoder unchanged. (The engine's own beam search,
avsr_amd.decode, keeps self-attention K/V caches instead — faster, same numbers.)

The encoder is differentiable (train mode: dropouts, BatchNorm batch statistics, gradients
into the parameter arena). Decoder and CTC entry points are inference paths: they run without
building a graph (the training step reaches them through `E2E.forward`).
"""
import math

import torch

from . import ops

_RELU = ops.L.ACT_RELU


def to_engine(eng, t, dtype=None):
    """host or device tensor -> contiguous device tensor (`dtype`: converted by the cast
    kernel on the device)."""
    t = t.to(eng.device).contiguous()
    if dtype is not None and t.dtype != dtype:
        out = torch.empty(t.shape, device=eng.device, dtype=dtype)
        if t.numel():
            ops.cast(t.view(-1, t.shape[-1]), out.view(-1, t.shape[-1]))
        return out
    return t


def lengths_from_mask(mask, B, T):
    """(B, T) / (B, 1, T) bool padding mask (True = valid, a prefix per row) -> int64 lengths
    (host). The reference builds these masks with make_non_pad_mask (nets_utils.py:183)."""
    if mask is None:
        return torch.full((B,), T, dtype=torch.int64)
    m = mask.reshape(B, -1).detach().cpu().bool()
    lens = m.sum(-1)
    ref = torch.arange(m.shape[1]).unsqueeze(0) < lens.unsqueeze(1)
    if not torch.equal(ref, m):
        raise NotImplementedError("padding masks must be prefix masks (make_non_pad_mask layout)")
    return lens.to(torch.int64)


# ============================================================================== encoder
class _EncoderStep(torch.autograd.Function):
    """AVHubertModel.forward in train mode with gradients: forward = Engine.encoder_fwd,
    backward = Engine.encoder_bwd (weight gradients land in the arena)."""

    @staticmethod
    def forward(fctx, anchor, eng, audios, videos, bt, seeds, modality):
        if eng.before_forward is not None:      # DDP buffer broadcast (parallel.ArenaDDP)
            eng.before_forward()
        x, ctx = eng.encoder_fwd(audios, videos, bt, True, True, seeds, modality)
        fctx.eng, fctx.ctx = eng, ctx
        B, T = bt["B"], bt["T"]
        out = torch.empty(B, T, eng.D, device=eng.device, dtype=torch.float32)
        ops.cast(x, out.view(B * T, eng.D))
        return out

    @staticmethod
    def backward(fctx, dout):
        eng = fctx.eng
        eng.arena.attach_grads()
        B, T, D = dout.shape
        d = to_engine(eng, dout.reshape(B * T, D), eng.dtype)
        eng.encoder_backward(fctx.ctx, d)     # with the DDP reducer's begin / buckets / finish
        fctx.ctx = None
        return (None,) * 7


def encoder_forward(e2e, input_features, attention_mask=None, video=None, **kwargs):
    """AVHubertModel.forward (avhubert.py:546-561) -> BaseModelOutput(last_hidden_state (B,T,D) fp32)."""
    from transformers.modeling_outputs import BaseModelOutput
    if video is None or input_features is None:
        raise ValueError("AVHubertModel.forward needs both input_features (audio) and video")
    eng = e2e.engine()
    B, _, T = video.shape[:3]
    lens = lengths_from_mask(attention_mask, B, T)
    train = e2e.encoder.training
    if train and torch.is_grad_enabled():
        bt = eng.prepare(video, input_features, lens)
        x = _EncoderStep.apply(e2e._anchor, eng, input_features.to(eng.device), video.to(eng.device), bt,
                               eng.new_seeds(), eng.draw_modality(train=True))
    else:
        x = to_engine(eng, eng.encode(input_features, video, lens, train=train), torch.float32)
    return BaseModelOutput(last_hidden_state=x, hidden_states=None, attentions=None)


# ============================================================================== decoder
def _check_causal(tgt_mask, L):
    """the decoder kernels implement the causal self-attention mask the reference builds
    (target_mask with pad = eos never masks a key: e2e_asr_avhubert.py:141-142, mask.py:20-51)"""
    if tgt_mask is None:
        return
    m = tgt_mask.detach().cpu().bool().reshape(-1, L, L)
    causal = torch.tril(torch.ones(L, L, dtype=torch.bool))
    if not bool((m == causal).all()):
        raise NotImplementedError("decoder self-attention masks must be causal (subsequent_mask)")


def _teacher_forced(eng, tgt, memory, mlens):
    """Engine.decoder_fwd (eval) over token ids tgt (n, l) and memory (n, T, D):
    logits (n*l, Vp) in the engine dtype and the per-layer context."""
    n, l = tgt.shape
    T = memory.shape[1]
    mem = to_engine(eng, memory, eng.dtype).view(n * T, eng.dD)
    lens_host = mlens if mlens is not None else torch.full((n,), T, dtype=torch.int64)
    bt = {"B": n, "T": T, "L1": l, "lens_host": lens_host,
          "lens": lens_host.to(torch.int32).to(eng.device), "full": bool((lens_host == T).all()),
          "ys_in": tgt.reshape(-1).to(eng.device, torch.int32)}
    eng.ensure_pe(l)
    logits, ctx = eng.decoder_fwd(mem, bt, False, True, eng.new_seeds(0))
    return logits, ctx


def _log_softmax_positions(eng, logits, n, l, pos):
    """fp32 log-softmax over the vocabulary of position `pos` of each of n sequences."""
    rows = logits.view(n, l, eng.Vp)[:, pos]
    out = torch.empty(n, eng.V, device=eng.device, dtype=torch.float32)
    return ops.log_softmax_rows(rows, eng.V, out)


@torch.no_grad()
def decoder_forward(e2e, tgt, tgt_mask, memory, memory_mask):
    """Decoder.forward (decoder.py:122-151): logits (B, L, V) fp32 and tgt_mask."""
    eng = e2e.engine()
    n, l = tgt.shape
    _check_causal(tgt_mask, l)
    mlens = None if memory_mask is None else lengths_from_mask(memory_mask, n, memory.shape[1])
    logits, _ = _teacher_forced(eng, tgt, memory, mlens)
    out = torch.empty(n * l, eng.V, device=eng.device, dtype=torch.float32)
    ops.cast(logits[:, :eng.V], out)
    return out.view(n, l, eng.V), tgt_mask


def _stacked_cache(eng, c, n, rows):
    """a layer's cache as one (n, rows, D) engine-dtype tensor (accepts the batched tensor or a
    list of per-hypothesis (rows, D) tensors)."""
    D = eng.dD
    if torch.is_tensor(c):
        return to_engine(eng, c, eng.dtype).view(n, rows, D)
    out = eng._e(n, rows, D)
    for b, cb in enumerate(c):
        ops.cast(to_engine(eng, cb, eng.dtype).view(1, rows * D), out.view(n, rows * D)[b:b + 1])
    return out


@torch.no_grad()
def decoder_forward_one_step(e2e, tgt, tgt_mask, memory, memory_mask=None, cache=None):
    """Decoder.forward_one_step (decoder.py:153-187): log-probs of the next token for every
    prefix tgt (n, l), and the new cache (per layer: outputs (n, l, D) of all positions)."""
    eng = e2e.engine()
    ar = eng.arena
    n, l = tgt.shape
    D, H = eng.dD, eng.dH
    T = memory.shape[1]
    _check_causal(tgt_mask, l)
    mlens = None if memory_mask is None else lengths_from_mask(memory_mask, n, T)
    if cache is None:
        # every position is a query (decoder_layer.py:84-92 with cache=None): teacher forcing
        logits, ctx = _teacher_forced(eng, tgt, memory, mlens)
        outs = [lc["y"] for lc in ctx["layers"][1:]] + [ctx["y_last"]]
        return _log_softmax_positions(eng, logits, n, l, l - 1), [o.view(n, l, D) for o in outs]
    # cached: only the last position is a query; K/V of the self-attention come from the
    # layer input of every position (decoder_layer.py:84-92)
    mem = to_engine(eng, memory, eng.dtype).view(n * T, D)
    mlen = None if mlens is None else mlens.to(torch.int32).to(eng.device)
    eng.ensure_pe(l)
    x = eng._e(n * l, D)
    ops.embed_fwd(tgt.reshape(-1).to(eng.device, torch.int32), eng.w("decoder.embed.0.weight"), eng._pe[:l],
                  math.sqrt(D), x, l)
    new_cache = []
    for i in range(eng.dl):
        p = f"decoder.decoders.{i}."
        sa, ca, ff = p + "self_attn.", p + "src_attn.", p + "feed_forward."
        n1, _, _ = ops.layernorm_fwd(x, ar.master(p + "norm1.weight"), ar.master(p + "norm1.bias"), 1e-12)
        qkv = ops.linear_fwd(n1, ar.span([sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight"]),
                             ar.span([sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias"], buf="master"))
        q3 = qkv.view(n, l, 3 * D)
        o1 = eng._e(n, D)
        ops.dec_attn(q3[:, l - 1, :D], q3[:, :, D:2 * D], q3[:, :, 2 * D:], o1, n=n, H=H, klen_max=l,
                     k_bstride=l * 3 * D, v_bstride=l * 3 * D)
        y1 = ops.linear_fwd(o1, eng.w(sa + "linear_out.weight"), ar.master(sa + "linear_out.bias"),
                            res=x.view(n, l, D)[:, l - 1])
        n2, _, _ = ops.layernorm_fwd(y1, ar.master(p + "norm2.weight"), ar.master(p + "norm2.bias"), 1e-12)
        q2 = ops.linear_fwd(n2, eng.w(ca + "linear_q.weight"), ar.master(ca + "linear_q.bias"))
        kv = ops.linear_fwd(mem, ar.span([ca + "linear_k.weight", ca + "linear_v.weight"]),
                            ar.span([ca + "linear_k.bias", ca + "linear_v.bias"], buf="master"))
        o2 = eng._e(n, D)
        ops.dec_attn(q2, kv[:, :D], kv[:, D:], o2, n=n, H=H, klen_max=T, k_bstride=T * 2 * D, v_bstride=T * 2 * D,
                     klen=mlen)
        y2 = ops.linear_fwd(o2, eng.w(ca + "linear_out.weight"), ar.master(ca + "linear_out.bias"), res=y1)
        n3, _, _ = ops.layernorm_fwd(y2, ar.master(p + "norm3.weight"), ar.master(p + "norm3.bias"), 1e-12)
        a = ops.linear_fwd(n3, eng.w(ff + "w_1.weight"), ar.master(ff + "w_1.bias"), act=_RELU)
        out = eng._e(n, l, D)
        ops.linear_fwd(a, eng.w(ff + "w_2.weight"), ar.master(ff + "w_2.bias"), res=y2, out=out[:, l - 1])
        if l > 1:
            c = _stacked_cache(eng, cache[i], n, l - 1)
            ops.cast(c.view(n, (l - 1) * D), out.view(n, l * D)[:, :(l - 1) * D])
        new_cache.append(out)
        x = out.view(n * l, D)
    yn, _, _ = ops.layernorm_fwd(x.view(n, l, D)[:, l - 1], ar.master("decoder.after_norm.weight"),
                                 ar.master("decoder.after_norm.bias"), 1e-12)
    logits = eng._e(n, eng.Vp)
    ops.linear_fwd(yn, eng.w("decoder.output_layer.weight"), ar.master("decoder.output_layer.bias"),
                   out=logits[:, :eng.V])
    logp = torch.empty(n, eng.V, device=eng.device, dtype=torch.float32)
    return ops.log_softmax_rows(logits, eng.V, logp), new_cache


def decoder_score(e2e, ys, state, x):
    """Decoder.score (decoder.py:190-196): ys (l,), x (T, D) -> (logp (V,), state)."""
    logp, state = decoder_forward_one_step(e2e, ys.unsqueeze(0), None, x.unsqueeze(0), cache=state)
    return logp.squeeze(0), state


def decoder_batch_score(e2e, ys, states, xs):
    """Decoder.batch_score (decoder.py:199-227): ys (n, l), per-hypothesis states (a list of
    per-layer (l-1, D) tensors, or None), xs (n, T, D) -> (logp (n, V), new per-hyp states)."""
    n = len(ys)
    nl = e2e.engine().dl
    batch_state = None if states[0] is None else [[states[b][i] for b in range(n)] for i in range(nl)]
    logp, st = decoder_forward_one_step(e2e, ys, None, xs, cache=batch_state)
    return logp, [[st[i][b] for i in range(nl)] for b in range(n)]


# ============================================================================== CTC
def _ctc_logits(eng, hs):
    """ctc_lo over hs (B, T, D) -> logits (B*T, Vp) in the engine dtype."""
    B, T, D = hs.shape
    x = to_engine(eng, hs, eng.dtype).view(B * T, D)
    logits = eng._e(B * T, eng.Vp)
    ops.linear_fwd(x, eng.w("ctc.ctc_lo.weight"), eng.arena.master("ctc.ctc_lo.bias"), out=logits[:, :eng.V])
    return logits


@torch.no_grad()
def ctc_log_softmax(e2e, hs_pad):
    """CTC.log_softmax (ctc.py:163-170): (B, T, D) -> (B, T, V) fp32."""
    eng = e2e.engine()
    B, T, _ = hs_pad.shape
    out = torch.empty(B * T, eng.V, device=eng.device, dtype=torch.float32)
    ops.log_softmax_rows(_ctc_logits(eng, hs_pad), eng.V, out)
    return out.view(B, T, eng.V)


@torch.no_grad()
def ctc_argmax(e2e, hs_pad):
    """CTC.argmax (ctc.py:172-180): (B, T) int64."""
    eng = e2e.engine()
    B, T, _ = hs_pad.shape
    lp = ctc_log_softmax(e2e, hs_pad).view(B * T, eng.V)
    ids = torch.empty(B * T, 1, device=eng.device, dtype=torch.int32)
    ops.row_topk(lp, eng.V, 1, ids)
    return ids.view(B, T).long()


@torch.no_grad()
def ctc_forward(e2e, hs_pad, hlens, ys_pad):
    """CTC.forward (ctc.py:83-151): (loss = sum over utterances of the CTC NLL / B, with
    zero_infinity; ys_hat (T, B, V) logits). Eval path (dropout off, no graph)."""
    eng = e2e.engine()
    B, T, _ = hs_pad.shape
    logits = _ctc_logits(eng, hs_pad)
    lse = torch.empty(B * T, device=eng.device, dtype=torch.float32)
    ops.row_lse(logits, eng.V, lse)
    lab = ys_pad.detach().cpu()
    ys = [r[r != -1] for r in lab]
    Lmax = max(1, max(len(y) for y in ys))
    ctc_lab = torch.full((B, Lmax), -1, dtype=torch.int32)
    for i, y in enumerate(ys):
        ctc_lab[i, :len(y)] = y
    S = 2 * Lmax + 1
    alpha = torch.empty(B, T, S, device=eng.device)
    gamma = torch.empty(B, T, S, device=eng.device)
    nll = torch.empty(B, device=eng.device)
    cp = ops.ctc_params(logits, B, T, eng.V, ctc_lab.to(eng.device),
                        torch.tensor([len(y) for y in ys], dtype=torch.int32).to(eng.device),
                        torch.as_tensor(hlens).to(torch.int32).to(eng.device), lse, alpha, gamma, nll)
    ops.ctc_fwd(cp)
    out4 = torch.empty(4, device=eng.device)
    ops.loss_finalize(B, nll, torch.empty(0, device=eng.device), None, 1.0, out4)
    ys_hat = torch.empty(T, B, eng.V, device=eng.device, dtype=torch.float32)
    for b in range(B):                      # (B*T, V) rows -> (T, B, V) like ys_hat.transpose(0, 1)
        ops.cast(logits[b * T:(b + 1) * T, :eng.V], ys_hat[:, b, :])
    return out4[1], ys_hat
