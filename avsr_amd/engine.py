"""The AVSR hot path on MI355X: explicit forward and backward of E2E (encoder + CTC +
attention decoder + joint loss) as a sequence of libavsr_hip.so launches.

Reference semantics (quanpn90/avsr @ 2025-08-29):
  E2E.forward                  src/nets/backend/e2e_asr_avhubert.py:119-159
  AVHubertModel.forward_gen    src/nets/backend/backbones/avhubert.py:448-544
  ResEncoder                   src/nets/backend/backbones/resnet.py:126-164
  AVHubertEncoder(+Layer)      avhubert.py:668-768 (+ HF Wav2Vec2 modules)
  CTC                          src/nets/backend/ctc.py:64-151
  Decoder / DecoderLayer       src/nets/backend/transformer/decoder.py:122-151, decoder_layer.py:58-121
  LabelSmoothingLoss           src/nets/backend/transformer/label_smoothing_loss.py:41-63

Design (MI355X-first):
  * one process per GPU; all math in hand-written HIP kernels (ops.*); activations NHWC /
    row-major [tokens][features] in the compute dtype (bf16, or fp32 "parity mode");
  * no autograd graph inside the model: the forward saves exactly what the backward
    needs, the backward is written out layer by layer and accumulates fp32 weight
    gradients straight into the flat Arena buffer (fused bias/activation/dropout/residual
    epilogues, fused BatchNorm statistics, flash attention, fused loss gradients);
  * dropout masks are counter-based (seed, element index): recomputed in the backward,
    never stored; the loss and its gradient never leave the device (no host sync).
"""
import math
import os
import random

import numpy as np
import torch

from . import ops
from . import _lib as L
from .arena import Arena

GELU, RELU, NONE = L.ACT_GELU, L.ACT_RELU, L.ACT_NONE
# One configuration (the A/B switches of rounds 1-3 were removed; their measurements are in
# DESIGN.md §9 and the git history). Module constants, flipped only by parity tests:
# BatchNorm-backward reductions in the ResNet data-grad epilogues (bf16; fp32 uses separate passes)
_BN_FUSE = True
# bias gradients reduced in the epilogue of the data-grad GEMM that produces their operand
_DB_FUSE = True
# parameter-gradient column-sum finalise passes batched per flush (ops.colsum_defer)
_COLSUM_DEFER = True
# bias gradients of operands only the side stream's weight-grads read run on the side stream
_SIDE_BIAS = True
# encoder QKV and out-proj weight-gradients as one grouped launch (192 + 64 output tiles = one
# block per CU) instead of a 192-tile launch beside 64 idle CUs and a 64-tile x 4 split-K launch:
# 68.1 vs 66.7 + 30.2 us isolated, but 0.4-0.6 % slower in the step (its 256 long 128-KiB blocks
# hold every CU while the data-gradient chain waits; profiles/r06_wgrad_group_ab.txt): off
WGRAD_GROUP = False
# order of an encoder layer's side-stream batch (f2 / f1: FFN output / input weight-gradients,
# o: out-proj weight-gradient, c: q/k/v bias column sums, q: QKV weight-gradient). The batch of
# layer i runs beside layer i-1's data-gradient chain. "o,f2,f1,c,q" (the out-proj weight-gradient
# ahead of the FFN ones, its 8-wave blocks then beside the next layer's FFN data-gradients rather
# than the whole-CU dQ kernel) measured +0.3 % over the issue order "f2,f1,o,c,q"; o second
# -1.7 %, o last -0.7 % (profiles/r06_side_order_ab.txt). Results do not depend on it.
SIDE_ORDER = "o,f2,f1,c,q"
# encoder self-attention dropout from stored keep masks (avsr_attn_dropmask, generated for every
# layer on the side stream while the step stream runs the frontends) instead of a hash per score
# element in the forward, dK/dV and dQ kernels (same bits)
ATTN_MASK = True
# the CTC branch of the forward runs on the side stream beside the decoder forward
_CTC_SIDE = True
# bf16 stem conv straight from the video (stem.hip) instead of pack + general implicit GEMM
_STEM_DIRECT = True
# encoder residual-branch dropout backward (+ bias gradient) fused into the LayerNorm backward
# that produces its input gradient
_LN_EW_FUSE = True
# weight-gradients, the forward's CTC branch and the gradient clear on a second stream beside the
# data-gradient chain (off: in line on the step stream; 54.3 vs 51.0 ms per video-on step,
# profiles/r04_side_stream_ab.txt)
SIDE_STREAM = True
# single process: the optimizer's gradient-norm pass over everything but the ResNet frontend runs
# on the side stream beside the ResNet backward (bench.py wires Engine.pre_video_grads)
EARLY_NORM = True
# training loops that own their optimizer (bench.py) update everything past the frontends on an
# update stream beside the next step's frontend forward (FusedAdamW(overlap=True))
OPT_OVERLAP = True
# grid cap of the overlapped update launches (FusedAdamW.overlap_blocks; 0: the whole chip)
OPT_OVERLAP_BLOCKS = 128
# ... and those launches zero the gradients they read (the next step's gradient clear)
OPT_CLEAR_IN_UPDATE = True


_STEP_STREAMS = {}


def prioritize_step_stream(device):
    """Make a high-priority stream the current stream of `device` for the training step; the
    weight-gradient side stream keeps the default priority, so the data-gradient chain (which
    bounds the step) wins CU slots over it (bench A/B, profiles/r02_stream_priority_ab.txt:
    +1.5 %). Returns the stream (or None off the GPU)."""
    if device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _STEP_STREAMS.get(idx)
    if s is None:
        s = _STEP_STREAMS[idx] = torch.cuda.Stream(device=idx, priority=-1)
    # work already queued on the stream that was current (engine setup: arena copies, the
    # bf16 shadow cast) must finish before the step stream reads it: side streams created by
    # torch are non-blocking w.r.t. the legacy default stream
    prev = torch.cuda.current_stream(idx)
    if prev != s:
        s.wait_stream(prev)
    torch.cuda.set_stream(s)
    return s


def wgrad_splitk(M, N, K):
    """token-dimension split of a weight-gradient GEMM dW[N][K] += dy[M][N]^T x[M][K] over
    blocks. The library runs weight-gradients as 8-wave blocks that already split their K range
    between two wave groups (gemm.hip wgrad_dual_kernel, one block per CU), so the block grid is
    split only when the 128x128 tiles fill less than half the chip (out-proj 1024x1024: 64 tiles
    x 4), through a slab workspace (no atomics). With the library option wgrad_dual = 0 (A/B):
    the 4-wave core at two blocks per CU with its 512-block target."""
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    if ops.L.get_option("wgrad_dual") == 0:
        return 1 if tiles > 256 else max(1, min(16, 512 // max(tiles, 1), M // 512))
    return 1 if tiles >= 128 else max(1, min(16, 256 // max(tiles, 1), M // 1024))


def _pad8(n):
    return (n + 7) // 8 * 8


class _Seeds:
    """deterministic per-site dropout stream ids for one step"""

    def __init__(self, base):
        self.base = base & 0xFFFFFFFFFFFF
        self.i = 0

    def next(self):
        self.i += 1
        return self.peek(0)

    def peek(self, k):
        """the value next() returns k + 1 calls from now (k = 0: the last one drawn)"""
        return (self.base * 0x9E3779B97F4A7C15 + (self.i + k) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF


def positional_encoding(L_, d, device):
    """embedding.py:59-78 sinusoidal table (fp32)."""
    pe = torch.zeros(L_, d)
    pos = torch.arange(0, L_, dtype=torch.float32).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.to(device)


class Engine:
    RES_BLOCKS = [(1, 0, 64, 64, 1), (1, 1, 64, 64, 1), (2, 0, 64, 128, 2), (2, 1, 128, 128, 1),
                  (3, 0, 128, 256, 2), (3, 1, 256, 256, 1), (4, 0, 256, 512, 2), (4, 1, 512, 512, 1)]

    def __init__(self, shell, cfg, device, dtype=torch.bfloat16):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.D = cfg.hidden_size
        self.H = cfg.num_attention_heads
        self.F = cfg.intermediate_size
        self.nl = cfg.num_hidden_layers
        self.dD = cfg.ddim
        self.dH = cfg.dheads
        self.dF = cfg.dunits
        self.dl = cfg.dlayers
        self.V = cfg.odim
        self.Vp = _pad8(cfg.odim)
        self.G = cfg.num_conv_pos_embedding_groups
        self.PK = cfg.num_conv_pos_embeddings
        assert self.D // self.H == 64 and self.dD // self.dH == 64, "kernels use head dim 64"
        assert cfg.adim == self.D == self.dD, "proj_decoder (adim != ddim) not on the hot path"
        # configuration the reference reads but the engine does not implement: refuse loudly
        # LayerDrop (avhubert.py:709-712): training skips encoder layer i when its draw is below it
        self.layerdrop = float(getattr(cfg, "layerdrop", 0.0) or 0.0)
        # LabelSmoothingLoss(normalize_length) (label_smoothing_loss.py:61): / tokens instead of / B
        self.len_norm = bool(getattr(cfg, "transformer_length_normalized_loss", False))
        if getattr(cfg, "modality_fuse", "concat") not in ("concat", "add"):
            raise ValueError(f"unknown modality_fuse {cfg.modality_fuse!r}")
        self.fuse_add = getattr(cfg, "modality_fuse", "concat") == "add"
        if getattr(cfg, "modality", "av") not in ("av", "audio", "video"):
            raise ValueError(f"unknown modality {cfg.modality!r}")
        self.last_modality = None
        self.force_modality = None   # (modality,): skip the draw (bench warm-up of every variant)
        self.capture = None          # tests: a dict receives the last forward's enc / logits / batch
        self._pinned = [(None, None)] * 4
        self._pin_next = 0
        self._nbt = None
        self.side = (torch.cuda.Stream(device=self.device)
                     if self.device.type == "cuda" and SIDE_STREAM else None)
        # reused events: a stream wait binds the record that precedes it
        self._side_ev = [torch.cuda.Event() for _ in range(8)] if self.side is not None else []
        self._amask, self._amask_wait = None, False     # encoder attention dropout masks (ATTN_MASK)
        self._amask_ev = torch.cuda.Event() if self.side is not None else None
        self._side_i = 0
        # operands the side stream reads stay referenced until join_side() (instead of
        # record_stream, whose deferred frees keep the caching allocator growing for steps)
        self._side_keep = []
        self._side_defer = None      # list while a layer's handoffs are batched (_side_layer)
        E = "encoder.encoder.layers"
        groups = []
        for i in range(self.nl):
            a = f"{E}.{i}.attention."
            groups.append([a + "q_proj.weight", a + "k_proj.weight", a + "v_proj.weight"])
            groups.append([a + "q_proj.bias", a + "k_proj.bias", a + "v_proj.bias"])
        for i in range(self.dl):
            s = f"decoder.decoders.{i}.self_attn."
            groups.append([s + "linear_q.weight", s + "linear_k.weight", s + "linear_v.weight"])
            groups.append([s + "linear_q.bias", s + "linear_k.bias", s + "linear_v.bias"])
            c = f"decoder.decoders.{i}.src_attn."
            groups.append([c + "linear_k.weight", c + "linear_v.weight"])
            groups.append([c + "linear_k.bias", c + "linear_v.bias"])
        perms = {}
        for n, p in shell.named_parameters():
            if p.dim() == 4:
                perms[n] = (0, 2, 3, 1)
        self.pc = "encoder.encoder.pos_conv_embed.conv."
        perms[self.pc + "parametrizations.weight.original1"] = (0, 2, 1)
        pad_rows = {"decoder.output_layer.weight": self.Vp, "ctc.ctc_lo.weight": self.Vp,
                    "decoder.output_layer.bias": self.Vp, "ctc.ctc_lo.bias": self.Vp}
        frozen = ["encoder.mask_emb", "encoder.label_embs_concat"]
        # buffers to the device; the BatchNorm running statistics (fp32 running_mean / var)
        # are re-homed into ONE flat buffer so that DDP's per-forward buffer broadcast is a
        # single collective (parallel.ArenaDDP)
        stats = []
        for m in shell.modules():
            for k, b in list(m._buffers.items()):
                if b is not None:
                    m._buffers[k] = b.to(self.device)
                    if k in ("running_mean", "running_var") and b.dtype == torch.float32:
                        stats.append((m, k))
        self.bn_flat = torch.empty(sum(m._buffers[k].numel() for m, k in stats), device=self.device)
        o = 0
        for m, k in stats:
            b = m._buffers[k]
            view = self.bn_flat[o:o + b.numel()].view(b.shape)
            view.copy_(b)
            m._buffers[k] = view
            o += b.numel()
        self.arena = Arena(shell, self.device, dtype, fuse_groups=groups, pad_rows=pad_rows, perms=perms, frozen=frozen)
        # gradient-readiness hook for the overlapped all-reduce (parallel.GradReducer): after
        # encoder layer i's backward, the weight-decay segment is final from the first element of
        # layer i on (the arena keeps module order inside a segment; decoder / CTC head come later
        # and are done before the encoder).
        # data-parallel hooks (set by parallel.ArenaDDP / bench.py): before_forward() at the start
        # of a training forward, before_backward() / on_grad_ready(offset) / after_backward()
        # around the backward (offset: the decay segment is final from there on)
        self.on_grad_ready = None
        self.pre_video_grads = None   # callable: see _grads_before_video
        self.before_forward = None
        self.before_backward = None
        self.after_backward = None
        d0, d1 = self.arena.segments["decay"]
        self._layer_decay_off = []
        for i in range(self.nl):
            pre = f"encoder.encoder.layers.{i}."
            offs = [m["off"] for n, m in self.arena.meta.items() if n.startswith(pre) and d0 <= m["off"] < d1]
            self._layer_decay_off.append(min(offs) if offs else d1)
        if self.layerdrop > 0:      # the optimizer skips the layers no backward touched (grad None)
            self.arena.ld_ranges = [self.arena.ranges_of(f"encoder.encoder.layers.{i}.") for i in range(self.nl)]
        self.shell = shell
        self.step_count = 0
        self._pe = positional_encoding(max(512, 64), self.dD, self.device)
        self._stem_wp = None

    # ------------------------------------------------------------------------------ utils
    @staticmethod
    def new_seeds(seed=None):
        """per-step dropout stream ids (counter-based hash masks, recomputed in the backward)"""
        return _Seeds(random.getrandbits(48) if seed is None else seed)

    def draw_modality(self, train):
        """which frontend's features are zeroed (avhubert.py:471-482): cfg.modality 'audio' /
        'video' always zero the other stream; in training with 'av' the reference draws two
        numbers from numpy's global RNG per forward (np.random.random() twice, unconditionally)
        and drops a modality with probability modality_dropout. Same RNG, same draw order, so a
        seeded run makes the same decisions as the reference."""
        cfg = self.cfg
        mod = getattr(cfg, "modality", "av")
        if mod == "audio":
            return "video_off"
        if mod == "video":
            return "audio_off"
        if not train:
            return None
        p_modality, p_audio = np.random.random(), np.random.random()
        if p_modality < cfg.modality_dropout:
            return "audio_off" if p_audio < cfg.audio_dropout else "video_off"
        return None

    def ensure_pe(self, L_):
        if self._pe.shape[0] < L_:
            self._pe = positional_encoding(2 * L_, self.dD, self.device)

    def _e(self, *shape, dtype=None):
        return torch.empty(*shape, device=self.device, dtype=dtype or self.dtype)

    def _z(self, *shape, dtype=None):
        return torch.zeros(*shape, device=self.device, dtype=dtype or self.dtype)

    def _dq32(self, rows, D):
        """fp32 dQ accumulator for the fp32 (parity) attention backward; None in bf16, where
        the backward writes dQ straight into the activation-dtype gradient buffer."""
        return self._z(rows, D, dtype=torch.float32) if self.dtype == torch.float32 else None

    def w(self, n):
        return self.arena.w(n)

    def g(self, n):
        return self.arena.g(n)

    def _bn(self, prefix):
        """(module, gamma, beta master fp32 views) of a BatchNorm with the given key prefix."""
        mod = self.shell.get_submodule(prefix)
        return mod, self.arena.master(prefix + ".weight"), self.arena.master(prefix + ".bias")

    # weight gradients run on a side stream: nothing on the backward's critical path (the data-
    # gradient chain) waits for them, so they fill the CUs the chain's kernels leave idle (grid
    # tails, one-block-per-CU attention, small LayerNorm / bias kernels). Their inputs are kept
    # alive for the side stream (_side_keep) and never overwritten afterwards; gradient
    # consumers (all-reduce buckets, the optimizer) wait for the side stream first.
    def _on_side(self, fn, *keep):
        side = self.side
        if side is None:
            return fn()
        if self._side_defer is not None:        # batched: issued by _flush_side after one wait
            self._side_defer.append((fn, keep))
            return None
        # order the side stream after the work queued so far on the current stream: one raw
        # event record + wait (torch's wait_stream builds Stream / Event objects per call)
        if self._side_ev:
            ev = self._side_ev[self._side_i]
            self._side_i = (self._side_i + 1) % len(self._side_ev)
            ev.record()
            side.wait_event(ev)
        else:
            side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            r = fn()
        self._side_keep.extend(keep)
        return r

    def _side_layer(self, on):
        """start (on) / end a batch of side-stream handoffs: the layer's weight-gradient work is
        queued and issued at the end of its data-gradient chain behind ONE event wait, so the
        step stream records one event per layer instead of one per weight-gradient (the side
        stream then trails by at most one layer; its operands are never overwritten)"""
        if self.side is None:
            return
        if on:
            self._flush_side()
            self._side_defer = []
        else:
            self._flush_side()
            self._side_defer = None

    def _flush_side(self):
        q = self._side_defer
        if not q:
            return
        self._side_defer = None
        keep = [t for _, k in q for t in k]

        def run_all():
            for fn, _ in q:
                fn()
        self._on_side(run_all, *keep)
        self._side_defer = []

    def zero_grad_async(self):
        """arena.zero_grad() queued on the side stream (after the work queued so far on the
        current stream, e.g. the previous optimizer step): nothing in the forward reads
        gradients, and backward() joins the side stream before its first gradient write, so
        the 1.3 GB memset leaves the forward's serial chain"""
        if self.side is None:
            self.arena.zero_grad()
            return
        g = self.arena.grad
        arena = self.arena
        done = arena.grads_cleared      # the overlapped update zeroes what it reads
        arena.grads_cleared = False

        def clear():
            arena.wait_update()         # an overlapped optimizer update still reads the gradients
            if not done:
                g.zero_()
        self._on_side(clear, g)
        self.arena.attach_grads(zero=False)
        self.arena.ld_touched.clear()

    def join_side(self):
        """make the current stream wait for every weight gradient issued so far"""
        self._flush_side()
        self._side_defer = None
        if self.side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            if self._side_keep:
                # freed blocks return to the current stream's pool behind this wait
                self._side_keep.clear()

    def _wgrad(self, dy, x, dW, alpha=1.0):
        """dW (fp32) += alpha * dy^T x (side stream). When the output tile grid is at or below one
        block per CU the token dimension is split and the partial tiles go to a slab workspace
        (no atomics): measured in round 3 (M=6000) 4096x1024 100 -> 72 us with 2 splits."""
        M, N = dy.shape
        K = x.shape[1]
        splitk = wgrad_splitk(M, N, K)

        def run():
            ws = None
            if splitk > 1:
                ws = torch.empty(ops.slab_ws(1, splitk, N, K), device=dy.device, dtype=torch.float32)
            ops.gemm(dy, x, dW, M=N, N=K, K=M, a_kmajor=False, b_kmajor=False, lda=dy.stride(0), ldb=x.stride(0),
                     ldc=dW.stride(0), alpha=alpha, beta=1.0, splitk=splitk, ws=ws)
        self._on_side(run, dy, x)

    def _conv_wgrad(self, g, x, dy, dw):
        self._on_side(lambda: ops.conv_bwd_weight(g, x, dy, dw), x, dy)

    def _fused_db(self, name):
        """bias-gradient target handed to the data-grad that produces its operand (ops.linear_dgrad
        reduces it in the GEMM epilogue, or in a separate pass where that core does not apply)"""
        return self.g(name) if _DB_FUSE else None

    def _bias_grad(self, g, db, alpha=1.0, fused=False):
        """db += alpha * column sums of g (skipped when the producing data-grad already did it)"""
        if fused and _DB_FUSE:
            return
        ops.ew_bwd(g, db=db, alpha=alpha)

    def _bias_grad_side(self, g, db):
        """db += column sums of g on the weight-grad side stream (off the data-gradient chain; g is
        an operand the side stream's weight-grad reads anyway), finalised there at once"""
        if self.side is None or not _SIDE_BIAS:
            return self._bias_grad(g, db)
        self._on_side(lambda: ops.ew_bwd(g, db=db, inline=True), g)

    # ------------------------------------------------------------------------ batch prep
    def _stage(self, host_i32):
        """one H2D copy of a host int32 vector through a ring of pinned staging buffers:
        asynchronous (a pageable-memory copy makes the host wait for the stream to drain, which
        starves the GPU while the next step's launches are issued); a ring slot is reused only
        after the copy that last read it has executed."""
        n = host_i32.numel()
        ring = self._pinned
        i = self._pin_next = (self._pin_next + 1) % len(ring)
        buf, ev = ring[i]
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(n, 4096), dtype=torch.int32, pin_memory=True)
            ev = None
        if ev is not None:
            ev.synchronize()
        buf[:n].copy_(host_i32)
        dev = torch.empty(n, dtype=torch.int32, device=self.device)
        dev.copy_(buf[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        ring[i] = (buf, ev)
        return dev

    def prepare(self, videos, audios, video_lengths, labels=None):
        """index tensors of a batch (labels / lengths are host data in the collator layout; a
        device tensor is read back once). All of them reach the device in ONE asynchronous copy."""
        B, _, T = videos.shape[:3]
        if video_lengths.is_cuda and (labels is None or labels.is_cuda):
            return self._prepare_device(B, T, video_lengths, labels)
        lens = video_lengths.detach().cpu().to(torch.int64)
        b = {"B": B, "T": T, "lens_host": lens, "full": bool((lens == T).all())}
        parts = [lens.to(torch.int32)]
        if labels is not None:
            lab = labels.detach().cpu()
            ys = [r[r != -1] for r in lab]
            L1 = max(len(y) for y in ys) + 1
            ys_in = torch.full((B, L1), self.V - 1, dtype=torch.int32)
            ys_out = torch.full((B, L1), -1, dtype=torch.int32)
            Lmax = max(1, max(len(y) for y in ys))
            ctc_lab = torch.full((B, Lmax), -1, dtype=torch.int32)
            for i, y in enumerate(ys):
                ys_in[i, 1:len(y) + 1] = y
                ys_out[i, :len(y)] = y
                ys_out[i, len(y)] = self.V - 1
                ctc_lab[i, :len(y)] = y
            parts += [ys_in.flatten(), ys_out.flatten(), ctc_lab.flatten(),
                      torch.tensor([len(y) for y in ys], dtype=torch.int32)]
        dev = self._stage(torch.cat(parts))
        o = 0
        views = []
        for t in parts:
            views.append(dev[o:o + t.numel()])
            o += t.numel()
        b["lens"] = views[0]
        if labels is not None:
            b.update(L1=L1, ys_in=views[1], ys_out=views[2], ctc_lab=views[3].view(B, Lmax), ctc_len=views[4])
        return b

    def _prepare_device(self, B, T, video_lengths, labels):
        """prepare() for lengths / labels already on the device (HF Trainer moves the whole
        batch there): every index tensor is built by device ops, nothing is read back, so the
        host keeps issuing ahead of the GPU. Shapes come from the padded label width Lw
        (= the collator's max label count, avhubert_dataset.py:302-311): the decoder runs
        L1 = Lw + 1 positions. Columns past a row's labels are eos inputs with ignored (-1)
        targets behind a causal mask, so losses and gradients equal those of L1 = max len + 1."""
        dev = self.device
        b = {"B": B, "T": T, "lens_host": None, "full": False,
             "lens": video_lengths.detach().to(dev, torch.int32)}
        if labels is None:
            return b
        lab = labels.detach().to(dev)
        Lw = lab.shape[1]
        eos = self.V - 1
        valid = lab != -1
        ylen = valid.sum(1)
        # compaction of the non-(-1) labels of each row (the reference's ys = [y[y != ignore_id]])
        pos = torch.where(valid, torch.cumsum(valid, 1) - 1, torch.full_like(ylen[:, None], Lw))
        comp = torch.full((B, Lw + 1), -1, dtype=torch.int32, device=dev)
        comp.scatter_(1, pos, lab.to(torch.int32))
        comp = comp[:, :Lw].contiguous()
        ar = torch.arange(Lw + 1, device=dev)[None]
        ys_out = torch.full((B, Lw + 1), -1, dtype=torch.int32, device=dev)
        ys_out[:, :Lw] = comp
        ys_out = torch.where(ar == ylen[:, None], torch.full_like(ys_out, eos), ys_out)
        ys_in = torch.full((B, Lw + 1), eos, dtype=torch.int32, device=dev)
        ys_in[:, 1:] = torch.where(comp >= 0, comp, torch.full_like(comp, eos))
        ctc_lab = comp if Lw > 0 else torch.full((B, 1), -1, dtype=torch.int32, device=dev)
        b.update(L1=Lw + 1, ys_in=ys_in.reshape(-1), ys_out=ys_out.reshape(-1), ctc_lab=ctc_lab,
                 ctc_len=ylen.to(torch.int32))
        return b

    # ===================================================================== video frontend
    def _geom(self, nimg, hin, cin, cout, k, s):
        return ops.ConvGeom(nimg, hin, hin, cin, cout, k, k, (s, s), (k // 2, k // 2))

    def _count_bn(self, bn):
        """BatchNorm num_batches_tracked += 1: collected and applied by one multi-tensor add at the
        end of the ResNet forward (20 one-element kernel launches on the forward's chain before)"""
        if self._nbt is not None:
            self._nbt.append(bn.num_batches_tracked)
        else:
            bn.num_batches_tracked.add_(1)

    def _conv_bn(self, g, x, wname, bnprefix, train):
        """conv (implicit GEMM) + BN statistics (fused in the conv epilogue) + BN finalize."""
        h = self._e(g.out_pixels, g.cout)
        bn, gam, bet = self._bn(bnprefix)
        st = ops.BnState(g.cout, self.device)
        if train:
            part = self._e(g.cout, ops.conv_stat_tiles(g, ops.dtype_code(x)), 3, dtype=torch.float32)
            ops.conv_fwd(g, x, self.w(wname), h, part)
            ops.bn_finalize(st, gam, bet, bn.running_mean, bn.running_var, partials=part, training=True,
                            momentum=bn.momentum, eps=bn.eps)
            self._count_bn(bn)
        else:
            ops.conv_fwd(g, x, self.w(wname), h)
            ops.bn_finalize(st, gam, bet, bn.running_mean, bn.running_var, training=False, eps=bn.eps)
        return h, st

    def video_fwd(self, videos, train, save):
        B, _, T = videos.shape[:3]
        N = B * T
        R = "encoder.feature_extractor_video.resnet."
        ctx = {"N": N}
        gs = ops.ConvGeom(N, 88, 88, 8, 64, 7, 7, (2, 2), (3, 3))
        h0 = self._e(N * 44 * 44, 64)
        bn, gam, bet = self._bn(R + "frontend3D.1")
        st0 = ops.BnState(64, self.device)
        vid = videos.contiguous()
        # the direct kernel addresses the fp32 video with 32-bit buffer offsets (avsr_stem_conv_fwd
        # returns AVSR_E_SHAPE from 2^31 bytes, ~69 k frames): larger batches take the packed conv
        direct = (self.dtype == torch.bfloat16 and _STEM_DIRECT
                  and vid.numel() * vid.element_size() < ops.STEM_DIRECT_MAX_BYTES)
        # the packed 8-channel input: the general conv's operand, and the stem weight-grad's. With
        # the direct conv only the weight-grad (end of the backward) reads it: packed on the side
        # stream after the ResNet forward (beside the encoder's GEMMs rather than the HBM-heavy
        # stem conv), off the forward's serial chain (joined with the CTC branch at its end)
        xp = None
        side_pack = False
        if not direct:
            xp = self._e(N, 88, 88, 8)
            ops.stem_pack(vid, xp)
        elif save:
            xp = self._e(N, 88, 88, 8)
            side_pack = True
        if direct:      # bf16: the stem conv reads the video itself (stem.hip, K = 288 instead of 392)
            wk = self._e(64, ops.STEM_K)
            ops.stem_wpack2(self.arena.master(R + "frontend3D.0.weight"), wk)
            part = self._e(64, ops.stem_conv_tiles(B, T), 3, dtype=torch.float32) if train else None
            ops.stem_conv_fwd(vid, wk, h0, part)
        else:
            wp = self._e(64, 7, 7, 8)        # the packed weight (not an arena view)
            ops.stem_wpack(self.arena.master(R + "frontend3D.0.weight"), wp)
            part = self._e(64, ops.conv_stat_tiles(gs, ops.dtype_code(xp)), 3, dtype=torch.float32) if train else None
            ops.conv_fwd(gs, xp, wp, h0, part)
        if train:
            ops.bn_finalize(st0, gam, bet, bn.running_mean, bn.running_var, partials=part, training=True,
                            momentum=bn.momentum, eps=bn.eps)
            self._nbt = []
            self._count_bn(bn)
        else:
            ops.bn_finalize(st0, gam, bet, bn.running_mean, bn.running_var, training=False, eps=bn.eps)
        x = self._e(N * 22 * 22, 64)
        am = self._e(N * 22 * 22, 64, dtype=torch.uint8)
        hmax = self._e(N * 22 * 22, 64) if save else None
        ops.stem_pool_fwd(h0, N, 44, 44, st0, self.arena.master(R + "frontend3D.2.weight"), x, am, hmax=hmax)
        if save:
            ctx.update(xp=xp, gs=gs, h0=h0, st0=st0, am=am, hmax=hmax)
        blocks = []
        hw = 22
        for li, bi, cin, cout, s in self.RES_BLOCKS:
            p = f"{R}trunk.layer{li}.{bi}."
            g1 = self._geom(N, hw, cin, cout, 3, s)
            ho = g1.hout
            g2 = self._geom(N, ho, cout, cout, 3, 1)
            h1, st1 = self._conv_bn(g1, x, p + "conv1.weight", p + "bn1", train)
            a1 = self._e(N * ho * ho, cout)
            ops.bn_act_fwd(h1, st1, self.arena.master(p + "relu1.weight"), a1)
            h2, st2 = self._conv_bn(g2, a1, p + "conv2.weight", p + "bn2", train)
            out = self._e(N * ho * ho, cout)
            if cin != cout or s != 1:
                gd = ops.ConvGeom(N, hw, hw, cin, cout, 1, 1, (s, s), (0, 0))
                hd, std = self._conv_bn(gd, x, p + "downsample.0.weight", p + "downsample.1", train)
                ops.bn_act_fwd(h2, st2, self.arena.master(p + "relu2.weight"), out, res=hd, st2=std)
            else:
                gd, hd, std = None, None, None
                ops.bn_act_fwd(h2, st2, self.arena.master(p + "relu2.weight"), out, res=x)
            if save:
                blocks.append(dict(p=p, g1=g1, g2=g2, gd=gd, x=x, h1=h1, st1=st1, a1=a1, h2=h2, st2=st2, hd=hd,
                                   std=std, cin=cin, cout=cout, hw=hw))
            x = out
            hw = ho
        feat = self._e(N, 512)
        ops.avgpool_fwd(x, N, hw * hw, 512, feat)
        if side_pack:
            self._on_side(lambda: ops.stem_pack(vid, xp), vid, xp)
        if self._nbt:
            torch._foreach_add_(self._nbt, 1)
        self._nbt = None
        if save:
            ctx.update(blocks=blocks, hw_last=hw, feat=feat)
        return feat, ctx

    def video_bwd(self, ctx, dfeat):
        """ResNet backward. With bf16 compute the BatchNorm+PReLU backward reduction of each
        layer runs in the epilogue of the data-gradient that produces its output gradient
        (conv2 dgrad -> bn1; a block's last dgrad -> the previous block's bn2 or, for the first
        block, the stem on its pooled grid), so only the apply pass touches the tensors again."""
        N = ctx["N"]
        R = "encoder.feature_extractor_video.resnet."
        hw = ctx["hw_last"]
        fuse = self.dtype == torch.bfloat16 and _BN_FUSE
        blocks = ctx["blocks"]
        dout = self._e(N * hw * hw, 512)
        ops.avgpool_bwd(dfeat, N, hw * hw, 512, dout)
        red = None                 # (ws, tiles): dout already holds dz of the next bn2
        for j in range(len(blocks) - 1, -1, -1):
            blk = blocks[j]
            p, cout, cin = blk["p"], blk["cout"], blk["cin"]
            M2 = blk["h2"].shape[0]
            down = blk["gd"] is not None
            res, rst = (blk["hd"], blk["std"]) if down else (blk["x"], None)
            g2 = dict(dprelu=self.g(p + "relu2.weight"), dgamma=self.g(p + "bn2.weight"), dbeta=self.g(p + "bn2.bias"))
            if down:
                g2.update(dgamma2=self.g(p + "downsample.1.weight"), dbeta2=self.g(p + "downsample.1.bias"))
            # bn2 + prelu2 (+ downsample BN)
            if red is None:
                dz2, sums2 = ops.bn_act_bwd_reduce(dout, blk["h2"], blk["st2"], self.arena.master(p + "relu2.weight"),
                                                   res=res, st2=rst, **g2)
            else:
                dz2, sums2 = dout, ops.bn_bwd_finalize(red[0], red[1], cout, **g2)
            dh2 = self._e(M2, cout)
            dhd = self._e(M2, cout) if down else None
            ops.bn_bwd_apply(dz2, blk["h2"], blk["st2"], sums2, dh2, res=res, st2=rst, dh2=dhd)
            # conv2 (its data-grad carries bn1 + prelu1's reduction when fused)
            self._conv_wgrad(blk["g2"], blk["a1"], dh2, self.g(p + "conv2.weight"))
            da1 = self._e(M2, cout)
            g1 = dict(dprelu=self.g(p + "relu1.weight"), dgamma=self.g(p + "bn1.weight"), dbeta=self.g(p + "bn1.bias"))
            prelu1 = self.arena.master(p + "relu1.weight")
            if fuse:
                ws, tiles = ops.conv_bwd_data_bnr(blk["g2"], dh2, self.w(p + "conv2.weight"), da1, blk["h1"],
                                                  blk["st1"], prelu1)
                dz1, sums1 = da1, ops.bn_bwd_finalize(ws, tiles, cout, **g1)
            else:
                ops.conv_bwd_data(blk["g2"], dh2, self.w(p + "conv2.weight"), da1)
                dz1, sums1 = ops.bn_act_bwd_reduce(da1, blk["h1"], blk["st1"], prelu1, **g1)
            dh1 = self._e(M2, cout)
            ops.bn_bwd_apply(dz1, blk["h1"], blk["st1"], sums1, dh1)
            self._conv_wgrad(blk["g1"], blk["x"], dh1, self.g(p + "conv1.weight"))
            # block input gradient: conv1 (+ downsample) data-grads (+ dz2 through an identity
            # shortcut); the last one carries the reduction of the layer that produced the input
            if fuse:
                if j > 0:
                    pb = blocks[j - 1]
                    pdown = pb["gd"] is not None
                    tgt = dict(h=pb["h2"], st=pb["st2"], prelu=self.arena.master(pb["p"] + "relu2.weight"),
                               res=pb["hd"] if pdown else pb["x"], st2=pb["std"] if pdown else None)
                else:
                    tgt = dict(h=ctx["hmax"], st=ctx["st0"], prelu=self.arena.master(R + "frontend3D.2.weight"))
            red = None
            if not down:
                dx = dz2                     # identity shortcut: d(block input) starts as dz2
                if fuse:
                    red = ops.conv_bwd_data_bnr(blk["g1"], dh1, self.w(p + "conv1.weight"), dx, beta=1.0, **tgt)
                else:
                    ops.conv_bwd_data(blk["g1"], dh1, self.w(p + "conv1.weight"), dx, beta=1.0)
            else:
                dx = self._e(blk["x"].shape[0], cin)
                ops.conv_bwd_data(blk["g1"], dh1, self.w(p + "conv1.weight"), dx)
                self._conv_wgrad(blk["gd"], blk["x"], dhd, self.g(p + "downsample.0.weight"))
                if fuse:
                    red = ops.conv_bwd_data_bnr(blk["gd"], dhd, self.w(p + "downsample.0.weight"), dx, beta=1.0, **tgt)
                else:
                    ops.conv_bwd_data(blk["gd"], dhd, self.w(p + "downsample.0.weight"), dx, beta=1.0)
            dout = dx
        # stem: BN/PReLU reduction on the pooled grid, then the argmax-routed apply and the
        # weight-grad (pipelining the two over frame ranges on two streams measured no gain: both
        # slow down together, profiles/r04_stem_pipeline_ab.txt)
        dh0 = self._e(N * 44 * 44, 64)
        dzp, sums = ops.stem_pool_bwd_reduce(dout, ctx["hmax"], N, 44, 44, ctx["st0"],
                                             self.arena.master(R + "frontend3D.2.weight"),
                                             dprelu=self.g(R + "frontend3D.2.weight"),
                                             dgamma=self.g(R + "frontend3D.1.weight"),
                                             dbeta=self.g(R + "frontend3D.1.bias"), reduced=red)
        ops.stem_pool_bwd_apply(dzp, ctx["am"], ctx["h0"], N, 44, 44, ctx["st0"], sums, dh0)
        gp = self._z(64, 7, 7, 8, dtype=torch.float32)
        ops.conv_bwd_weight(ctx["gs"], ctx["xp"], dh0, gp)
        ops.stem_wgrad_unpack(gp, self.g(R + "frontend3D.0.weight"))

    # ============================================================================ encoder
    def _ln(self, x, name, eps, save=None):
        y, mean, rstd = ops.layernorm_fwd(x, self.arena.master(name + ".weight"), self.arena.master(name + ".bias"), eps)
        return y, mean, rstd

    def _ln_bwd(self, dy, x, name, mean, rstd, dres=None, dx=None, ew=None):
        """LayerNorm backward; ew = (g_out, drop_p, seed, db name): the dropout backward of the
        sublayer whose output was added to this LayerNorm's input, fused in (ew_bwd(dx, out=g_out,
        drop_p, seed, db)): dx is the residual gradient of that sublayer's output"""
        if ew is not None and _LN_EW_FUSE:
            g, p, seed, dbn = ew
            return ops.layernorm_bwd(dy, x, self.arena.master(name + ".weight"), mean, rstd, dx=dx, dres=dres,
                                     dgamma=self.g(name + ".weight"), dbeta=self.g(name + ".bias"), g=g, drop_p=p,
                                     seed=seed, db=self.g(dbn))
        out = ops.layernorm_bwd(dy, x, self.arena.master(name + ".weight"), mean, rstd, dx=dx, dres=dres,
                                dgamma=self.g(name + ".weight"), dbeta=self.g(name + ".bias"))
        if ew is not None:
            g, p, seed, dbn = ew
            ops.ew_bwd(out, out=g, drop_p=p, seed=seed, db=self.g(dbn))
        return out

    def encoder_fwd(self, audios, videos, bt, train, save, seeds, modality=None):
        """AVHubertModel.forward_gen(features_only=True) — returns (x (M, D), ctx)."""
        cfg = self.cfg
        B, T = bt["B"], bt["T"]
        M, D = B * T, self.D
        EN = "encoder."
        ctx = {"B": B, "T": T, "modality": modality}
        # LayerDrop: one torch.rand([]) (CPU generator) per layer on every call, train or eval, as
        # the reference draws them (avhubert.py:709-712; no other torch CPU draw happens between
        # the reference's frontends and its layer loop); training skips a layer whose draw is below
        # cfg.layerdrop (its context is None, the backward passes the gradient through)
        draws = [float(torch.rand([])) for _ in range(self.nl)]
        kept = [i for i in range(self.nl) if not (train and draws[i] < self.layerdrop)]
        # the self-attention dropout masks of every kept layer, on the side stream beside the
        # frontends (seeds: sd_in, sd_pc, then sd_att, sd_o, sd_a, sd_f per kept layer)
        p_att = cfg.attention_dropout if train else 0.0
        amask = self._attn_masks(B, T, p_att, {i: seeds.peek(3 + 4 * j) for j, i in enumerate(kept)})
        # audio / video frontends -> concat buffer [M][2D] (audio | video), or with
        # modality_fuse 'add' the sum [M][D] (avhubert.py:486-489: the video projection adds the
        # audio features as its residual)
        add = self.fuse_add
        fcat = self._e(M, D if add else 2 * D)
        fa = self._e(M, D) if add else fcat[:, :D]
        ain = self._e(M, cfg.audio_feat_dim)
        ops.audio_pack(audios.contiguous(), ain)
        if modality == "audio_off":
            fa.zero_()
        else:
            ops.linear_fwd(ain, self.w(EN + "feature_extractor_audio.proj.weight"),
                           self.arena.master(EN + "feature_extractor_audio.proj.bias"), out=fa)
        # video_off: the ResNet gradient is exactly zero (avhubert.py:480), so nothing of its
        # forward is kept for a backward (no packed stem input, no pooled-grid argmax values);
        # the forward itself still runs for the BatchNorm running statistics, as in the reference
        feat, vctx = self.video_fwd(videos, train, save and modality != "video_off")
        if modality == "video_off":
            if add:
                fcat.copy_(fa)
            else:
                fcat[:, D:].zero_()
        else:
            ops.linear_fwd(feat, self.w(EN + "feature_extractor_video.proj.weight"),
                           self.arena.master(EN + "feature_extractor_video.proj.bias"),
                           res=fa if add and modality != "audio_off" else None, out=fcat if add else fcat[:, D:])
        # an overlapped optimizer update of everything past the frontends (FusedAdamW(overlap=
        # True)) ran beside the frontends' forward: the first read of those parameters waits here
        self.arena.wait_update()
        ln0, m0, r0 = self._ln(fcat, EN + "layer_norm", 1e-5)
        sd_in = seeds.next()
        p_in = cfg.dropout_input if train else 0.0
        if add:        # embed dim = encoder dim: no post_extract_proj (avhubert.py:229-233)
            x = ops.dropout_fwd(ln0, self._e(M, D), p_in, sd_in) if p_in > 0 else ln0.clone()
        else:
            x = ops.linear_fwd(ln0, self.w(EN + "post_extract_proj.weight"),
                               self.arena.master(EN + "post_extract_proj.bias"), drop_p=p_in, seed=sd_in)
        if not bt["full"]:
            ops.mask_rows(x, B, T, bt["lens"])
        klen = None if bt["full"] else bt["lens"]
        # positional conv: y = x + gelu(conv(x) + b); x0 = dropout(y)
        pc = self.pc
        v = self.arena.master(pc + "parametrizations.weight.original1")     # [D][K][D/G]
        gpc = self.arena.master(pc + "parametrizations.weight.original0").reshape(-1)
        norm = self._e(self.PK, dtype=torch.float32)
        wpc = self._e(D, self.PK, D // self.G)
        ops.weightnorm_fwd(v, gpc, norm, wpc)
        geo = ops.ConvGeom(B, T, 1, D // self.G, D // self.G, self.PK, 1, (1, 1), (self.PK // 2, 0), groups=self.G,
                           hout=T, wout=1)
        pre = self._e(M, D)
        y = self._e(M, D)
        ops.conv_fwd(geo, x, wpc, y, bias=self.arena.master(pc + "bias"), act=GELU, preact=pre, res=x)
        sd_pc = seeds.next()
        p_h = cfg.hidden_dropout if train else 0.0
        if p_h > 0:
            ops.dropout_fwd(y, y, p_h, sd_pc)
        if save:
            ctx.update(ain=ain, fcat=fcat, ln0=ln0, m0=m0, r0=r0, sd_in=sd_in, p_in=p_in, x_pre=x, geo=geo, wpc=wpc,
                       norm=norm, pre=pre, sd_pc=sd_pc, p_h=p_h, vctx=vctx, feat=feat, klen=klen)
        x = y
        layers = []
        for i in range(self.nl):
            if i not in kept:
                if save:
                    layers.append(None)
                continue
            x, lc = self._enc_layer_fwd(i, x, B, T, klen, train, save, seeds, amask.get(i))
            if save:
                layers.append(lc)
        E = "encoder.encoder."
        out, mf, rf = self._ln(x, E + "layer_norm", 1e-5)
        if save:
            ctx.update(layers=layers, x_last=x, mf=mf, rf=rf)
        return out, ctx

    def _attn_masks(self, B, T, p_att, seeds_by_layer):
        """{layer: (seed, keep mask)} of the encoder self-attention dropout, generated on the side
        stream into a persistent per-layer buffer; the step stream waits for them before its first
        attention (ATTN_MASK, bf16 only)"""
        H = self.H
        if not (ATTN_MASK and p_att > 0 and self.dtype == torch.bfloat16 and seeds_by_layer
                and B * H * T * ((T + 1) // 2) <= 0xFFFFFFFF):
            return {}
        words = ops.attn_mask_words(B, H, T, T)
        if self._amask is None or self._amask.shape[1] != words:
            self._amask = None
            self._amask = torch.empty(self.nl, words, dtype=torch.int64, device=self.device)
        buf = self._amask

        def run():
            for i, sd in seeds_by_layer.items():
                ops.attn_dropmask(buf[i], B=B, H=H, Lq=T, Lk=T, drop_p=p_att, seed=sd)
        self._on_side(run)
        self._amask_wait = self.side is not None
        if self._amask_wait:
            self._amask_ev.record(self.side)
        return {i: (sd, buf[i]) for i, sd in seeds_by_layer.items()}

    def _enc_layer_fwd(self, i, x, B, T, klen, train, save, seeds, amask=None):
        cfg = self.cfg
        D, H = self.D, self.H
        M = B * T
        p = f"encoder.encoder.layers.{i}."
        a = p + "attention."
        ln1, m1, r1 = self._ln(x, p + "layer_norm", 1e-5)
        wqkv = self.arena.span([a + "q_proj.weight", a + "k_proj.weight", a + "v_proj.weight"])
        bqkv = self.arena.span([a + "q_proj.bias", a + "k_proj.bias", a + "v_proj.bias"], buf="master")
        qkv = ops.linear_fwd(ln1, wqkv, bqkv)
        o = self._e(M, D)
        lse = self._e(B, H, T, dtype=torch.float32)
        sd_att = seeds.next()
        p_att = cfg.attention_dropout if train else 0.0
        mask = None
        if amask is not None:
            assert amask[0] == sd_att, "attention mask seed out of step with the dropout sites"
            mask = amask[1]
            if self._amask_wait:            # the side stream's masks, once per forward
                torch.cuda.current_stream(self.device).wait_event(self._amask_ev)
                self._amask_wait = False
        ops.attn_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, lse, B=B, H=H, Lq=T, Lk=T, klen=klen,
                     scale=0.125, drop_p=p_att, seed=sd_att, mask=mask)
        sd_o = seeds.next()
        p_h = cfg.hidden_dropout if train else 0.0
        x1 = ops.linear_fwd(o, self.w(a + "out_proj.weight"), self.arena.master(a + "out_proj.bias"), res=x,
                            drop_p=p_h, seed=sd_o)
        ln2, m2, r2 = self._ln(x1, p + "final_layer_norm", 1e-5)
        ff = p + "feed_forward."
        h = self._e(M, self.F)
        sd_a = seeds.next()
        p_a = cfg.activation_dropout if train else 0.0
        act = ops.linear_fwd(ln2, self.w(ff + "intermediate_dense.weight"), self.arena.master(ff + "intermediate_dense.bias"),
                             act=GELU, preact=h, drop_p=p_a, seed=sd_a)
        sd_f = seeds.next()
        x2 = ops.linear_fwd(act, self.w(ff + "output_dense.weight"), self.arena.master(ff + "output_dense.bias"), res=x1,
                            drop_p=p_h, seed=sd_f)
        lc = None
        if save:
            lc = dict(i=i, x=x, ln1=ln1, m1=m1, r1=r1, qkv=qkv, o=o, lse=lse, sd_att=sd_att, p_att=p_att, mask=mask,
                      sd_o=sd_o, p_h=p_h,
                      x1=x1, ln2=ln2, m2=m2, r2=r2, h=h, act=act, sd_a=sd_a, p_a=p_a, sd_f=sd_f)
        return x2, lc

    def _ew_next(self, i, lc, M):
        """the FFN output dropout backward of layer i (x2 = x1 + drop(act W2^T + b2)), fused into
        the LayerNorm backward that produces dx2: (g2 buffer, p, seed, bias-gradient name)"""
        return (self._e(M, self.D), lc["p_h"], lc["sd_f"], f"encoder.encoder.layers.{i}.feed_forward.output_dense.bias")

    def _enc_layer_bwd(self, i, lc, dx2, B, T, klen, g2=None, lc_prev=None):
        """returns (d(layer input), g2 of layer i-1 or None); dx2 is consumed (may be reused).
        g2: this layer's FFN-output dropout backward of dx2, already computed by the LayerNorm
        backward that produced dx2 (else computed here); lc_prev: layer i-1's context, whose g2
        this layer's input LayerNorm backward computes."""
        D, H = self.D, self.H
        M = B * T
        p = f"encoder.encoder.layers.{i}."
        a = p + "attention."
        ff = p + "feed_forward."
        # x2 = x1 + drop(act W2^T + b2)
        if g2 is None:
            g2 = self._e(M, D)
            ops.ew_bwd(dx2, out=g2, drop_p=lc["p_h"], seed=lc["sd_f"], db=self.g(ff + "output_dense.bias"))
        # side-stream items of this layer, tagged as issued (reordered by SIDE_ORDER at the end)
        base = len(self._side_defer) if self._side_defer is not None else None
        tags = [] if base is not None else None

        def tag(t):
            if tags is not None and len(self._side_defer) == base + len(tags) + 1:
                tags.append(t)
        self._wgrad(g2, lc["act"], self.g(ff + "output_dense.weight"))
        tag("f2")
        dh = ops.linear_dgrad(g2, self.w(ff + "output_dense.weight"), gate=lc["h"], act=GELU, drop_p=lc["p_a"],
                              seed=lc["sd_a"], db=self._fused_db(ff + "intermediate_dense.bias"))
        self._bias_grad(dh, self.g(ff + "intermediate_dense.bias"), fused=True)
        self._wgrad(dh, lc["ln2"], self.g(ff + "intermediate_dense.weight"))
        tag("f1")
        dln2 = ops.linear_dgrad(dh, self.w(ff + "intermediate_dense.weight"))
        # x1 = x + drop(o Wo^T + bo): the out-proj dropout backward rides on this LN backward
        go = self._e(M, D)              # fresh: g2 may still be read by the side stream
        dx1 = self._ln_bwd(dln2, lc["x1"], p + "final_layer_norm", lc["m2"], lc["r2"], dres=dx2, dx=dx2,
                           ew=(go, lc["p_h"], lc["sd_o"], a + "out_proj.bias"))
        if not WGRAD_GROUP:
            self._wgrad(go, lc["o"], self.g(a + "out_proj.weight"))
            tag("o")
        do = ops.linear_dgrad(go, self.w(a + "out_proj.weight"))
        # attention
        qkv = lc["qkv"]
        dqkv = self._e(M, 3 * D)
        dq32 = self._dq32(M, D)
        delta = self._e(B, H, T, dtype=torch.float32)
        names_b = [a + "q_proj.bias", a + "k_proj.bias", a + "v_proj.bias"]
        names_w = [a + "q_proj.weight", a + "k_proj.weight", a + "v_proj.weight"]
        db_qkv = self.arena.span(names_b, buf="g")
        ops.attn_bwd(do, qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], lc["o"], lc["lse"], dq32, dqkv[:, D:2 * D],
                     dqkv[:, 2 * D:], delta, B=B, H=H, Lq=T, Lk=T, klen=klen, scale=0.125, drop_p=lc["p_att"],
                     seed=lc["sd_att"], dq=None if dq32 is not None else dqkv[:, :D], mask=lc["mask"])
        if dq32 is not None:
            ops.cast(dq32, dqkv[:, :D])
        # the q/k/v bias gradients (column sums of dqkv) on the side stream
        self._bias_grad_side(dqkv, db_qkv)
        tag("c")
        if WGRAD_GROUP:     # QKV (192 tiles) and out-proj (64 tiles) weight-gradients in one launch
            dwq, dwo = self.arena.span(names_w, buf="g"), self.g(a + "out_proj.weight")
            o = lc["o"]
            ln1 = lc["ln1"]
            self._on_side(lambda: ops.wgrad_group([(dqkv, ln1, dwq, 1.0), (go, o, dwo, 1.0)]), dqkv, ln1, go, o)
        else:
            self._wgrad(dqkv, lc["ln1"], self.arena.span(names_w, buf="g"))
        tag("q")
        if tags is not None and SIDE_ORDER:
            items = self._side_defer[base:]
            if len(tags) == len(items):
                by = dict(zip(tags, items))
                order = [t for t in SIDE_ORDER.replace(".", ",").split(",") if t in by]
                order += [t for t in tags if t not in order]
                self._side_defer[base:] = [by[t] for t in order]
        dln1 = ops.linear_dgrad(dqkv, self.arena.span(names_w))
        ew = self._ew_next(lc_prev["i"], lc_prev, M) if lc_prev is not None else None
        dx = self._ln_bwd(dln1, lc["x"], p + "layer_norm", lc["m1"], lc["r1"], dres=dx1, dx=dx1, ew=ew)
        return dx, (ew[0] if ew is not None else None)

    def encoder_bwd(self, ctx, dout):
        cfg = self.cfg
        B, T = ctx["B"], ctx["T"]
        M, D = B * T, self.D
        EN = "encoder."
        E = "encoder.encoder."
        layers = ctx["layers"]
        ex = [i for i in range(self.nl) if layers[i] is not None]       # layers LayerDrop kept
        self.arena.ld_touched.update(ex)
        ew = self._ew_next(ex[-1], layers[ex[-1]], M) if ex else None
        dx = self._ln_bwd(dout, ctx["x_last"], E + "layer_norm", ctx["mf"], ctx["rf"], ew=ew)
        g2 = ew[0] if ew is not None else None
        for i in reversed(range(self.nl)):
            if layers[i] is not None:
                j = ex.index(i)
                self._side_layer(True)
                dx, g2 = self._enc_layer_bwd(i, layers[i], dx, B, T, ctx["klen"], g2=g2,
                                             lc_prev=layers[ex[j - 1]] if j > 0 else None)
                self._side_layer(False)
                ops.colsum_flush()                  # this layer's bias / LayerNorm gradients
            if self.on_grad_ready is not None:      # layers >= i (and everything after them) final
                self.on_grad_ready(self._layer_decay_off[i])   # (the reducer also waits for the side stream)
        # pos-conv block: x0 = drop(x + gelu(conv(x) + b))
        pc = self.pc
        if ctx["p_h"] > 0:
            ops.ew_bwd(dx, out=dx, drop_p=ctx["p_h"], seed=ctx["sd_pc"])
        gp = self._e(M, D)
        ops.ew_bwd(dx, out=gp, gate=ctx["pre"], act=GELU, db=self.g(pc + "bias"))
        dwpc = self._z(D, self.PK, D // self.G, dtype=torch.float32)
        ops.conv_bwd_weight(ctx["geo"], ctx["x_pre"], gp, dwpc)
        ops.weightnorm_bwd(self.arena.master(pc + "parametrizations.weight.original1"),
                           self.arena.master(pc + "parametrizations.weight.original0").reshape(-1), ctx["norm"], dwpc,
                           self.g(pc + "parametrizations.weight.original1"),
                           self.g(pc + "parametrizations.weight.original0").reshape(-1),
                           self._e(self.PK, dtype=torch.float32))
        ops.conv_bwd_data(ctx["geo"], gp, ctx["wpc"], dx, beta=1.0)
        if ctx["klen"] is not None:
            ops.mask_rows(dx, B, T, ctx["klen"])
        # post_extract_proj (+ dropout_input)
        gi = gp
        if self.fuse_add:
            ops.ew_bwd(dx, out=gi, drop_p=ctx["p_in"], seed=ctx["sd_in"])
            dln0 = gi
        else:
            ops.ew_bwd(dx, out=gi, drop_p=ctx["p_in"], seed=ctx["sd_in"], db=self.g(EN + "post_extract_proj.bias"))
            self._wgrad(gi, ctx["ln0"], self.g(EN + "post_extract_proj.weight"))
            dln0 = ops.linear_dgrad(gi, self.w(EN + "post_extract_proj.weight"))
        dfcat = self._ln_bwd(dln0, ctx["fcat"], EN + "layer_norm", ctx["m0"], ctx["r0"])
        fgm = cfg.feature_grad_mult            # GradMultiply (avhubert.py:173-182) on both frontends
        # 'add': both streams receive the sum's gradient; 'concat': each its half
        da_all, dv_all = (dfcat, dfcat) if self.fuse_add else (dfcat[:, :D], dfcat[:, D:])
        if ctx["modality"] != "audio_off":
            da = da_all
            self._bias_grad(da, self.g(EN + "feature_extractor_audio.proj.bias"), alpha=fgm)
            self._wgrad(da, ctx["ain"], self.g(EN + "feature_extractor_audio.proj.weight"), alpha=fgm)
        if ctx["modality"] != "video_off":
            dv = dv_all
            self._bias_grad(dv, self.g(EN + "feature_extractor_video.proj.bias"), alpha=fgm)
            self._wgrad(dv, ctx["feat"], self.g(EN + "feature_extractor_video.proj.weight"), alpha=fgm)
            dfeat = self._e(M, 512)
            ops.gemm(dv, self.w(EN + "feature_extractor_video.proj.weight"), dfeat, M=M, N=512, K=D, a_kmajor=True,
                     b_kmajor=False, lda=dv.stride(0), ldb=512, ldc=512, alpha=fgm)
            self._grads_before_video()
            self.video_bwd(ctx["vctx"], dfeat)
        else:
            self._grads_before_video()
        self.join_side()

    def _grads_before_video(self):
        """every gradient but the ResNet frontend's is final here: pre_video_grads (e.g.
        FusedAdamW.early_sumsq, single process) runs on the side stream beside the ResNet backward
        instead of in the step's serial tail"""
        if self.pre_video_grads is not None:
            ops.colsum_flush()          # the deferred bias / LayerNorm finalise passes first
            self._on_side(self.pre_video_grads)

    # ============================================================================ decoder
    def decoder_fwd(self, enc, bt, train, save, seeds):
        cfg = self.cfg
        B, T, L1 = bt["B"], bt["T"], bt["L1"]
        R, D, H = B * L1, self.dD, self.dH
        klen = None if bt["full"] else bt["lens"]
        sd_e = seeds.next()
        p_d = cfg.dropout_rate if train else 0.0
        p_att = cfg.transformer_attn_dropout_rate if train else 0.0
        y = self._e(R, D)
        self.ensure_pe(L1)
        ops.embed_fwd(bt["ys_in"], self.w("decoder.embed.0.weight"), self._pe[:L1], math.sqrt(D), y, L1,
                      drop_p=p_d, seed=sd_e)
        ctx = {"sd_e": sd_e, "p_d": p_d, "p_att": p_att, "layers": [], "klen": klen, "L1": L1}
        for i in range(self.dl):
            p = f"decoder.decoders.{i}."
            sa, ca, ff = p + "self_attn.", p + "src_attn.", p + "feed_forward."
            n1, m1, r1 = ops.layernorm_fwd(y, self.arena.master(p + "norm1.weight"), self.arena.master(p + "norm1.bias"), 1e-12)
            qkv = ops.linear_fwd(n1, self.arena.span([sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight"]),
                                 self.arena.span([sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias"], buf="master"))
            o1 = self._e(R, D)
            lse1 = self._e(B, H, L1, dtype=torch.float32)
            s1 = seeds.next()
            ops.attn_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o1, lse1, B=B, H=H, Lq=L1, Lk=L1, causal=True,
                         scale=0.125, drop_p=p_att, seed=s1)
            s2 = seeds.next()
            y1 = ops.linear_fwd(o1, self.w(sa + "linear_out.weight"), self.arena.master(sa + "linear_out.bias"), res=y,
                                drop_p=p_d, seed=s2)
            n2, m2, r2 = ops.layernorm_fwd(y1, self.arena.master(p + "norm2.weight"), self.arena.master(p + "norm2.bias"), 1e-12)
            q2 = ops.linear_fwd(n2, self.w(ca + "linear_q.weight"), self.arena.master(ca + "linear_q.bias"))
            kv = ops.linear_fwd(enc, self.arena.span([ca + "linear_k.weight", ca + "linear_v.weight"]),
                                self.arena.span([ca + "linear_k.bias", ca + "linear_v.bias"], buf="master"))
            o2 = self._e(R, D)
            lse2 = self._e(B, H, L1, dtype=torch.float32)
            s3 = seeds.next()
            ops.attn_fwd(q2, kv[:, :D], kv[:, D:], o2, lse2, B=B, H=H, Lq=L1, Lk=T, klen=klen, scale=0.125,
                         drop_p=p_att, seed=s3)
            s4 = seeds.next()
            y2 = ops.linear_fwd(o2, self.w(ca + "linear_out.weight"), self.arena.master(ca + "linear_out.bias"), res=y1,
                                drop_p=p_d, seed=s4)
            n3, m3, r3 = ops.layernorm_fwd(y2, self.arena.master(p + "norm3.weight"), self.arena.master(p + "norm3.bias"), 1e-12)
            h = self._e(R, self.dF)
            s5 = seeds.next()
            a = ops.linear_fwd(n3, self.w(ff + "w_1.weight"), self.arena.master(ff + "w_1.bias"), act=RELU, preact=h,
                               drop_p=p_d, seed=s5)
            s6 = seeds.next()
            y3 = ops.linear_fwd(a, self.w(ff + "w_2.weight"), self.arena.master(ff + "w_2.bias"), res=y2, drop_p=p_d, seed=s6)
            if save:
                ctx["layers"].append(dict(y=y, n1=n1, m1=m1, r1=r1, qkv=qkv, o1=o1, lse1=lse1, s1=s1, s2=s2, y1=y1, n2=n2,
                                          m2=m2, r2=r2, q2=q2, kv=kv, o2=o2, lse2=lse2, s3=s3, s4=s4, y2=y2, n3=n3, m3=m3,
                                          r3=r3, h=h, a=a, s5=s5, s6=s6))
            y = y3
        yn, mf, rf = ops.layernorm_fwd(y, self.arena.master("decoder.after_norm.weight"),
                                       self.arena.master("decoder.after_norm.bias"), 1e-12)
        logits = self._e(R, self.Vp)
        ops.linear_fwd(yn, self.w("decoder.output_layer.weight"), self.arena.master("decoder.output_layer.bias"),
                       out=logits[:, :self.V])
        if save:
            ctx.update(y_last=y, yn=yn, mf=mf, rf=rf)
        return logits, ctx

    def decoder_bwd(self, ctx, dlogits, enc, denc, bt):
        B, T, L1 = bt["B"], bt["T"], ctx["L1"]
        R, D, H = B * L1, self.dD, self.dH
        klen = ctx["klen"]
        p_d, p_att = ctx["p_d"], ctx["p_att"]
        self._bias_grad(dlogits, self.arena.g_padded("decoder.output_layer.bias"))
        self._wgrad(dlogits, ctx["yn"], self.arena.g_padded("decoder.output_layer.weight"))   # padded vocab
        dyn = self._e(R, D)
        ops.gemm(dlogits, self.arena.w_padded("decoder.output_layer.weight"), dyn, M=R, N=D, K=self.Vp, a_kmajor=True,
                 b_kmajor=False, lda=dlogits.stride(0), ldb=D, ldc=D)
        def ln_bwd(dn, x, name, m, r, dres, ew):
            """LayerNorm backward (dx over the residual gradient dres, in place) with the dropout
            backward + bias gradient of the sublayer whose output fed it fused in (ew = (seed, bias
            name): g = ew_bwd(dx, drop_p, seed, db), as the encoder's _ln_bwd); returns (dx, g)"""
            g = None if ew is None else self._e(R, D)      # fresh: the previous g may still be read by the side stream
            if ew is not None and _LN_EW_FUSE:
                dx = ops.layernorm_bwd(dn, x, self.arena.master(name + ".weight"), m, r, dx=dres, dres=dres,
                                       dgamma=self.g(name + ".weight"), dbeta=self.g(name + ".bias"), g=g, drop_p=p_d,
                                       seed=ew[0], db=self.g(ew[1]))
                return dx, g
            dx = ops.layernorm_bwd(dn, x, self.arena.master(name + ".weight"), m, r, dx=dres, dres=dres,
                                   dgamma=self.g(name + ".weight"), dbeta=self.g(name + ".bias"))
            if ew is not None:
                ops.ew_bwd(dx, out=g, drop_p=p_d, seed=ew[0], db=self.g(ew[1]))
            return dx, g

        def ew_of(i, s, name):
            return (ctx["layers"][i][s], f"decoder.decoders.{i}." + name)

        top = self.dl - 1
        dy, g = ln_bwd(dyn, ctx["y_last"], "decoder.after_norm", ctx["mf"], ctx["rf"], None,
                       ew_of(top, "s6", "feed_forward.w_2.bias") if self.dl else None)
        for i in reversed(range(self.dl)):
            self._side_layer(True)              # flushes the previous layer's batch first
            lc = ctx["layers"][i]
            p = f"decoder.decoders.{i}."
            sa, ca, ff = p + "self_attn.", p + "src_attn.", p + "feed_forward."
            # FFN: g = the output dropout backward of dy (with w_2's bias gradient), fused into the
            # LayerNorm backward that produced dy
            self._wgrad(g, lc["a"], self.g(ff + "w_2.weight"))
            dh = ops.linear_dgrad(g, self.w(ff + "w_2.weight"), gate=lc["h"], act=RELU, drop_p=p_d, seed=lc["s5"],
                                  db=self._fused_db(ff + "w_1.bias"))
            self._bias_grad(dh, self.g(ff + "w_1.bias"), fused=True)
            self._wgrad(dh, lc["n3"], self.g(ff + "w_1.weight"))
            dn3 = ops.linear_dgrad(dh, self.w(ff + "w_1.weight"))
            dy, g = ln_bwd(dn3, lc["y2"], p + "norm3", lc["m3"], lc["r3"], dy, ew_of(i, "s4", "src_attn.linear_out.bias"))
            # source attention
            self._wgrad(g, lc["o2"], self.g(ca + "linear_out.weight"))
            do2 = ops.linear_dgrad(g, self.w(ca + "linear_out.weight"))
            dkv = self._e(B * T, 2 * D)
            dq32 = self._dq32(R, D)
            delta = self._e(B, H, L1, dtype=torch.float32)
            dq2 = self._e(R, D)
            ops.attn_bwd(do2, lc["q2"], lc["kv"][:, :D], lc["kv"][:, D:], lc["o2"], lc["lse2"], dq32, dkv[:, :D], dkv[:, D:],
                         delta, B=B, H=H, Lq=L1, Lk=T, klen=klen, scale=0.125, drop_p=p_att, seed=lc["s3"],
                         dq=None if dq32 is not None else dq2)
            if dq32 is not None:
                ops.cast(dq32, dq2)
            self._bias_grad(dq2, self.g(ca + "linear_q.bias"))
            self._wgrad(dq2, lc["n2"], self.g(ca + "linear_q.weight"))
            dn2 = ops.linear_dgrad(dq2, self.w(ca + "linear_q.weight"))
            kvw = [ca + "linear_k.weight", ca + "linear_v.weight"]
            self._bias_grad(dkv, self.arena.span([ca + "linear_k.bias", ca + "linear_v.bias"], buf="g"))
            self._wgrad(dkv, enc, self.arena.span(kvw, buf="g"))
            ops.linear_dgrad(dkv, self.arena.span(kvw), out=denc, beta=1.0)
            dy, g = ln_bwd(dn2, lc["y1"], p + "norm2", lc["m2"], lc["r2"], dy, ew_of(i, "s2", "self_attn.linear_out.bias"))
            # causal self attention
            self._wgrad(g, lc["o1"], self.g(sa + "linear_out.weight"))
            do1 = ops.linear_dgrad(g, self.w(sa + "linear_out.weight"))
            dqkv = self._e(R, 3 * D)
            dq32 = self._dq32(R, D)
            delta = self._e(B, H, L1, dtype=torch.float32)
            qkv = lc["qkv"]
            ops.attn_bwd(do1, qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], lc["o1"], lc["lse1"], dq32, dqkv[:, D:2 * D],
                         dqkv[:, 2 * D:], delta, B=B, H=H, Lq=L1, Lk=L1, causal=True, scale=0.125, drop_p=p_att, seed=lc["s1"],
                         dq=None if dq32 is not None else dqkv[:, :D])
            if dq32 is not None:
                ops.cast(dq32, dqkv[:, :D])
            nb = [sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias"]
            nw = [sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight"]
            self._bias_grad(dqkv, self.arena.span(nb, buf="g"))
            self._wgrad(dqkv, lc["n1"], self.arena.span(nw, buf="g"))
            dn1 = ops.linear_dgrad(dqkv, self.arena.span(nw))
            dy, g = ln_bwd(dn1, lc["y"], p + "norm1", lc["m1"], lc["r1"], dy,
                           ew_of(i - 1, "s6", "feed_forward.w_2.bias") if i > 0 else None)
        self._side_layer(False)
        ops.embed_bwd(bt["ys_in"], dy, math.sqrt(D), self.g("decoder.embed.0.weight"), L1, drop_p=p_d, seed=ctx["sd_e"])

    # ======================================================================== full model
    def forward(self, videos, audios, video_lengths, labels, train=True, need_grad=True, seed=None):
        """E2E.forward: returns (out4 = [loss, loss_ctc, loss_att, acc] on device, ctx)."""
        cfg = self.cfg
        if train and need_grad and self.before_forward is not None:
            self.before_forward()
        seeds = self.new_seeds(seed)
        bt = self.prepare(videos, audios, video_lengths, labels)
        B, T = bt["B"], bt["T"]
        M = B * T
        modality = self.draw_modality(train) if self.force_modality is None else self.force_modality[0]
        self.last_modality = modality
        enc, ectx = self.encoder_fwd(audios.to(self.device), videos.to(self.device), bt, train, need_grad, seeds, modality)
        # CTC branch: ctc_lo(dropout(enc)). It runs on the side stream (idle during the forward),
        # beside the decoder forward, whose small launches leave most CUs free; buffers are
        # allocated on the step stream, which waits for the branch before the loss combine
        sd_c = seeds.next()
        p_c = cfg.dropout_rate if train else 0.0
        xin = self._e(M, self.D) if p_c > 0 else enc
        clog = self._e(M, self.Vp)
        clse = self._e(M, dtype=torch.float32)
        Lmax = bt["ctc_lab"].shape[1]
        S = 2 * Lmax + 1
        alpha = self._e(B, T, S, dtype=torch.float32)
        gamma = self._e(B, T, S, dtype=torch.float32)
        nll = self._e(B, dtype=torch.float32)
        cp = ops.ctc_params(clog, B, T, self.V, bt["ctc_lab"], bt["ctc_len"], bt["lens"], clse, alpha, gamma, nll)

        def ctc_branch():
            if p_c > 0:
                ops.dropout_fwd(enc, xin, p_c, sd_c)
            ops.linear_fwd(xin, self.w("ctc.ctc_lo.weight"), self.arena.master("ctc.ctc_lo.bias"),
                           out=clog[:, :self.V])
            ops.row_lse(clog, self.V, clse)
            ops.ctc_fwd(cp)
        if _CTC_SIDE:
            self._on_side(ctc_branch, enc, xin, clog, clse, alpha, gamma, nll, bt["ctc_lab"], bt["ctc_len"], bt["lens"])
        else:
            ctc_branch()
        # attention branch
        dlog, dctx = self.decoder_fwd(enc, bt, train, need_grad, seeds)
        self.join_side()
        R = dlog.shape[0]
        dlse = self._e(R, dtype=torch.float32)
        rloss = self._e(R, dtype=torch.float32)
        rcorr = self._e(R, dtype=torch.int32)
        ops.lsm_fwd(dlog, self.V, bt["ys_out"], cfg.lsm_weight, dlse, rloss, rcorr)
        out4 = self._e(4, dtype=torch.float32)
        ops.loss_finalize(B, nll, rloss, rcorr, cfg.mtlalpha, out4, att_per_token=self.len_norm)
        if self.capture is not None:
            self.capture.update(enc=enc, clog=clog, dlog=dlog, bt=bt)
        ctx = None
        if need_grad:
            ctx = dict(bt=bt, enc=enc, ectx=ectx, xin=xin, p_c=p_c, sd_c=sd_c, clog=clog, cp=cp, dlog=dlog, dctx=dctx,
                       dlse=dlse)
        return out4, ctx

    def backward(self, ctx, d_ctc, d_att):
        """d_ctc / d_att: device fp32 scalars = d(total)/d(loss_ctc), d(total)/d(loss_att)
        (for total = loss: mtlalpha * dloss and (1 - mtlalpha) * dloss). Accumulates into
        arena.grad; nothing is synchronised with the host."""
        cfg = self.cfg
        bt = ctx["bt"]
        B, T = bt["B"], bt["T"]
        M = B * T
        d_ctc = d_ctc.reshape(1).to(torch.float32)
        d_att = d_att.reshape(1).to(torch.float32)
        self.join_side()            # a gradient clear queued on the side stream (zero_grad_async)
        if self.before_backward is not None:
            self.before_backward()
        # bias / LayerNorm parameter-gradient finalise passes are batched: one launch per
        # encoder layer (flushed before its on_grad_ready) and one for the rest at the end
        prev = ops.colsum_defer(_COLSUM_DEFER)
        try:
            self._backward(ctx, d_ctc, d_att)
            ops.colsum_flush()
        finally:
            ops.colsum_defer(prev)
        if self.after_backward is not None:
            self.after_backward()
        self.join_side()

    def encoder_backward(self, ectx, denc):
        """encoder-only backward (the reference call form model.encoder(...) trained alone,
        surface._EncoderStep) with backward()'s data-parallel hooks and finalise batching"""
        # as in backward(): the side stream's work from the forward (the bf16 stem's packed
        # input for its weight-grad, a zero_grad_async clear) must land before the first write
        self.join_side()
        if self.before_backward is not None:
            self.before_backward()
        prev = ops.colsum_defer(_COLSUM_DEFER)
        try:
            self.encoder_bwd(ectx, denc)
            ops.colsum_flush()
        finally:
            ops.colsum_defer(prev)
        if self.after_backward is not None:
            self.after_backward()
        self.join_side()

    def _backward(self, ctx, d_ctc, d_att):
        cfg = self.cfg
        bt = ctx["bt"]
        B, T = bt["B"], bt["T"]
        M = B * T
        # attention loss -> decoder
        dl = ctx["dlog"]
        ddl = self._e(dl.shape[0], self.Vp)
        if self.len_norm:      # / the number of target tokens (device count, no host sync)
            d_att = d_att / (bt["ys_out"] != -1).sum().clamp_min(1).to(torch.float32)
            ops.lsm_bwd(dl, self.V, bt["ys_out"], cfg.lsm_weight, ctx["dlse"], d_att, 1.0, ddl)
        else:
            ops.lsm_bwd(dl, self.V, bt["ys_out"], cfg.lsm_weight, ctx["dlse"], d_att, 1.0 / B, ddl)
        denc = self._e(M, self.D)
        # CTC -> denc (first write), then decoder adds
        dcl = self._e(M, self.Vp)
        ops.ctc_bwd(ctx["cp"], d_ctc, 1.0 / B, dcl)
        self._bias_grad(dcl, self.arena.g_padded("ctc.ctc_lo.bias"))
        # padded vocab (the backward writes zeros to columns V..Vp): Vp rows keep the weight-grad on
        # the LDS-DMA core (r-contiguous operands need a multiple of 8); the pad rows get exact zeros
        self._wgrad(dcl, ctx["xin"], self.arena.g_padded("ctc.ctc_lo.weight"))
        ops.gemm(dcl, self.arena.w_padded("ctc.ctc_lo.weight"), denc, M=M, N=self.D, K=self.Vp, a_kmajor=True,
                 b_kmajor=False, lda=dcl.stride(0), ldb=self.D, ldc=self.D, epi_bwd=True, drop_p=ctx["p_c"],
                 seed=ctx["sd_c"])
        self.decoder_bwd(ctx["dctx"], ddl, ctx["enc"], denc, bt)
        self.encoder_bwd(ctx["ectx"], denc)

    # ========================================================================= inference
    def encode(self, audios, videos, video_lengths=None, train=False):
        """encoder forward without graph (script/evaluation.py:96-101 call form: eval mode, no
        attention mask); train=True: dropouts / BatchNorm batch statistics, as the reference's
        encoder in train mode under no_grad."""
        B, _, T = videos.shape[:3]
        if video_lengths is None:
            video_lengths = torch.full((B,), T, dtype=torch.int64)
        bt = self.prepare(videos, audios, video_lengths)
        x, _ = self.encoder_fwd(audios.to(self.device), videos.to(self.device), bt, train, False,
                                self.new_seeds(None if train else 0), self.draw_modality(train))
        return x.view(B, T, self.D)
