"""Drop-in for src/avhubert_avsr/avhubert_avsr_model.py (AVHubertAVSR, AVHubertAVSROutput,
get_beam_search_decoder) and src/nets/backend/e2e_asr_avhubert.py (E2E).

Same class names, constructor, `forward` keyword names (the DataCollator keys, because HF
Trainer calls `model(**inputs)`), output dataclass and state-dict keys as the reference.
The computation runs in avsr_amd.engine.Engine (HIP kernels); there is no CPU / eager
fallback: using the model on a machine without the HIP library raises.
"""
import contextlib
from dataclasses import dataclass
from typing import Optional

import torch
from transformers.modeling_utils import PreTrainedModel
from transformers.utils import ModelOutput

from .configuration_avhubert_avsr import AVHubertAVSRConfig
from .decode import BatchBeamSearch, Hypothesis, get_beam_search_decoder  # noqa: F401  (reference surface)
from .nets.modules import E2EShell


@dataclass
class AVHubertAVSROutput(ModelOutput):
    loss: Optional[torch.FloatTensor] = None
    loss_ctc: Optional[torch.FloatTensor] = None
    loss_att: Optional[torch.FloatTensor] = None
    acc: Optional[torch.FloatTensor] = None


class _E2EStep(torch.autograd.Function):
    """Autograd boundary around the whole hot path: forward = Engine.forward, backward =
    Engine.backward (weight gradients land in the arena; no graph inside the model)."""

    @staticmethod
    def forward(fctx, anchor, engine, videos, audios, video_lengths, labels, train):
        out4, ectx = engine.forward(videos, audios, video_lengths, labels, train=train, need_grad=True)
        fctx.engine, fctx.ectx = engine, ectx
        fctx.mtl = engine.cfg.mtlalpha
        return out4[0].clone(), out4[1].clone(), out4[2].clone(), out4[3].clone()

    @staticmethod
    def backward(fctx, dloss, dctc, datt, dacc):
        z = torch.zeros((), device=dloss.device)
        dloss = z if dloss is None else dloss
        d_ctc = dloss * fctx.mtl + (z if dctc is None else dctc)
        d_att = dloss * (1.0 - fctx.mtl) + (z if datt is None else datt)
        # a per-parameter optimizer may have reset .grad to None since the last step
        fctx.engine.arena.attach_grads()
        fctx.engine.backward(fctx.ectx, d_ctc, d_att)
        fctx.ectx = None
        return (None,) * 7


class E2E(E2EShell):
    """src/nets/backend/e2e_asr_avhubert.py:24-159 (joint CTC / attention)."""

    def __init__(self, args, ignore_id=-1):
        super().__init__(args)
        self.cfg = args
        self.ignore_id = ignore_id
        self.mtlalpha = args.mtlalpha
        self.adim = args.adim
        self._engine = None
        self._anchor = torch.zeros(0, requires_grad=True)
        self.encoder._e2e = [self]        # list: not registered as a submodule
        self.decoder._e2e = [self]
        self.ctc._e2e = [self]

    def engine(self, device=None, dtype=None):
        """The HIP engine (built on first use: re-homes every parameter into the device arena;
        default compute dtype fp32 = the reference's evaluation precision). Every entry point
        fetches it here, which also refreshes the bf16 shadow after in-place parameter writes."""
        if self._engine is None:
            device = torch.device(device or "cuda")
            if device.type != "cuda":
                raise RuntimeError("the AVSR hot path runs on MI355X (HIP) only; no CPU fallback")
            from .engine import Engine
            self._engine = Engine(self, self.cfg, device, dtype or torch.float32)
        self._engine.arena.ensure_shadow()
        return self._engine

    def forward(self, video, audio, video_lengths, audio_lengths, label):
        eng = self.engine()
        if torch.is_grad_enabled():
            return _E2EStep.apply(self._anchor, eng, video, audio, video_lengths, label, self.training)
        out4, _ = eng.forward(video, audio, video_lengths, label, train=self.training, need_grad=False)
        return out4[0].clone(), out4[1].clone(), out4[2].clone(), out4[3].clone()


class AVHubertAVSR(PreTrainedModel):
    config_class = AVHubertAVSRConfig
    base_model_prefix = "avsr"

    def __init__(self, config: AVHubertAVSRConfig):
        super().__init__(config)
        self.avsr = E2E(config)
        self._ddp = None        # parallel.ArenaDDP once attached
        self.post_init()        # HF bookkeeping (tied-weight tables) that from_pretrained relies on

    def _init_weights(self, module):   # weights come from the module constructors / checkpoints
        pass

    def setup_engine(self, device="cuda", dtype=torch.bfloat16):
        """Move the model onto the HIP engine (flat fp32 arena + compute-dtype shadow).
        Calling it again with another compute dtype rebuilds the engine on the same weights."""
        e2e = self.avsr
        if e2e._engine is not None:
            eng = e2e._engine
            if torch.device(device).type != "cuda" or (torch.device(device).index not in (None, eng.device.index)):
                raise RuntimeError(f"the engine lives on {eng.device}; moving it is not supported")
            if dtype is None or dtype == eng.dtype:
                return self
            e2e._engine = None                  # re-home the arena views into a new arena
        e2e.engine(device, dtype)
        return self

    # ------------------------------------------------------------------ device / dtype moves
    # The reference's evaluation does `AVHubertAVSR.from_pretrained(...).eval().cuda()`
    # (script/evaluation.py:89-92) and HF Trainer does `model.to(args.device)`: on a GPU these
    # build the engine (fp32 parameters = fp32 compute, the reference's precision; bf16
    # parameters = bf16 compute with fp32 master weights).
    _DTYPES = (torch.float32, torch.bfloat16)

    def to(self, *args, **kwargs):
        device, dtype, _, _ = torch._C._nn._parse_to(*args, **kwargs)
        if dtype is not None and dtype not in self._DTYPES:
            raise NotImplementedError(f"compute dtype {dtype}: the HIP kernels run fp32 or bf16")
        eng = self.avsr._engine
        if device is not None and device.type == "cuda":
            return self.setup_engine(device, dtype or (eng.dtype if eng is not None else torch.float32))
        if eng is not None:
            if device is not None:
                raise RuntimeError("the model lives in the GPU parameter arena; there is no CPU path")
            return self.setup_engine(eng.device, dtype) if dtype is not None else self
        return super().to(*args, **kwargs)

    def cuda(self, device=None):
        if isinstance(device, int):
            device = torch.device("cuda", device)
        return self.to(device or "cuda")

    def float(self):
        return self.to(torch.float32)

    def bfloat16(self):
        return self.to(torch.bfloat16)

    def half(self):
        raise NotImplementedError("fp16 parameters: the HIP kernels run fp32 (parity) or bf16 (throughput)")

    def no_sync(self):
        """DistributedDataParallel.no_sync (accelerate calls it on non-final gradient-accumulation
        micro-steps): delegated to the attached parallel.ArenaDDP."""
        return self._ddp.no_sync() if self._ddp is not None else contextlib.nullcontext()

    def zero_grad(self, set_to_none: bool = True):
        """HF Trainer calls model.zero_grad() around every optimizer step: clear the gradient
        arena and keep the .grad views attached (set_to_none would detach them)."""
        if self.avsr._engine is not None:
            self.avsr._engine.arena.zero_grad()
        else:
            super().zero_grad(set_to_none=set_to_none)

    def forward(self, videos, audios, labels, video_lengths, audio_lengths, label_lengths):
        loss, loss_ctc, loss_att, acc = self.avsr(videos, audios, video_lengths, audio_lengths, labels)
        return AVHubertAVSROutput(loss=loss, loss_ctc=loss_ctc, loss_att=loss_att, acc=acc)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        if self.avsr._engine is not None:
            self.avsr._engine.arena.sync_shadow()
        return res

    def save_pretrained(self, save_directory, **kwargs):
        """HF save_pretrained with the reference's keys and shapes (config.json +
        model.safetensors). The arena's parameters are views of one buffer: hand HF a state
        dict of standalone contiguous host copies."""
        sd = kwargs.pop("state_dict", None)
        sd = self.state_dict() if sd is None else sd
        kwargs["state_dict"] = {k: v.detach().to("cpu", copy=True).contiguous() for k, v in sd.items()}
        return super().save_pretrained(save_directory, **kwargs)


