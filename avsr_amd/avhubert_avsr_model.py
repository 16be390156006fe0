"""Drop-in for src/avhubert_avsr/avhubert_avsr_model.py (AVHubertAVSR, AVHubertAVSROutput,
get_beam_search_decoder) and src/nets/backend/e2e_asr_avhubert.py (E2E).

Same class names, constructor, `forward` keyword names (the DataCollator keys, because HF
Trainer calls `model(**inputs)`), output dataclass and state-dict keys as the reference.
The computation runs in avsr_amd.engine.Engine (HIP kernels); there is no CPU / eager
fallback: using the model on a machine without the HIP library raises.
"""
from dataclasses import dataclass
from typing import Optional

import torch
from transformers.modeling_utils import PreTrainedModel
from transformers.modeling_outputs import BaseModelOutput
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
        """Build (once) the HIP engine: re-homes every parameter into the device arena."""
        if self._engine is None:
            device = torch.device(device or "cuda")
            if device.type != "cuda":
                raise RuntimeError("the AVSR hot path runs on MI355X (HIP) only; no CPU fallback")
            from .engine import Engine
            self._engine = Engine(self, self.cfg, device, dtype or torch.bfloat16)
        return self._engine

    def forward(self, video, audio, video_lengths, audio_lengths, label):
        eng = self.engine()
        loss, loss_ctc, loss_att, acc = _E2EStep.apply(self._anchor, eng, video, audio, video_lengths, label,
                                                       self.training)
        return loss, loss_ctc, loss_att, acc


class AVHubertAVSR(PreTrainedModel):
    config_class = AVHubertAVSRConfig
    base_model_prefix = "avsr"

    def __init__(self, config: AVHubertAVSRConfig):
        super().__init__(config)
        self.avsr = E2E(config)

    def _init_weights(self, module):   # weights come from the module constructors / checkpoints
        pass

    def setup_engine(self, device="cuda", dtype=torch.bfloat16):
        """Move the model onto the HIP engine (flat fp32 arena + compute-dtype shadow)."""
        self.avsr.engine(device, dtype)
        return self

    def forward(self, videos, audios, labels, video_lengths, audio_lengths, label_lengths):
        loss, loss_ctc, loss_att, acc = self.avsr(videos, audios, video_lengths, audio_lengths, labels)
        return AVHubertAVSROutput(loss=loss, loss_ctc=loss_ctc, loss_att=loss_att, acc=acc)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        if self.avsr._engine is not None:
            self.avsr._engine.arena.sync_shadow()
        return res


def encoder_forward(e2e, input_features, attention_mask=None, video=None):
    """AVHubertModel.forward (avhubert.py:546-561) on the engine: BaseModelOutput."""
    eng = e2e.engine()
    B, _, T = video.shape[:3]
    lengths = attention_mask.sum(-1) if attention_mask is not None else None
    x = eng.encode(input_features, video, lengths)
    return BaseModelOutput(last_hidden_state=x)
