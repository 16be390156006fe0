"""Parameter containers of the AVSR model, with the reference's exact module tree (and so its
exact state-dict keys, shapes and buffers — SURVEY.md §8(b) row b2).

These modules hold the parameters and buffers. The whole forward/backward runs in
avsr_amd.engine.Engine on HIP kernels over a flat parameter arena (avsr_amd.arena.Arena),
which re-homes every parameter defined here into one fp32 buffer. The sub-modules callers of
the reference use directly — `avsr.encoder(...)`, `avsr.decoder.batch_score(...)`,
`avsr.ctc.log_softmax(...)` — forward to the engine (avsr_amd.surface).

Reference module tree (file:line):
  E2E                        src/nets/backend/e2e_asr_avhubert.py:24-117
  AVHubertModel              src/nets/backend/backbones/avhubert.py:200-297
  SubModel                   avhubert.py:187-198
  ResEncoder/ResNet/BasicBlock src/nets/backend/backbones/resnet.py:30-164
  AVHubertEncoder(+Layer)    avhubert.py:668-768 on HF Wav2Vec2Encoder / EncoderLayer /
                             PositionalConvEmbedding / Attention / FeedForward
  Decoder / DecoderLayer     src/nets/backend/transformer/decoder.py:39-120, decoder_layer.py:15-56
  MultiHeadedAttention       src/nets/backend/transformer/attention.py:16-35
  CTC                        src/nets/backend/ctc.py:12-62
"""
import math

import torch
from torch import nn


class _Holder(nn.Module):
    def forward(self, *a, **k):  # pragma: no cover - never called
        raise RuntimeError("parameter container: the forward runs in avsr_amd.engine.Engine")


def _e2e(mod):
    """the E2E that owns this sub-module (set by avsr_amd.avhubert_avsr_model.E2E)"""
    owner = getattr(mod, "_e2e", None)
    if not owner:
        raise RuntimeError(f"{type(mod).__name__} is not attached to an E2E model")
    return owner[0]


def _conv3x3(i, o, stride=1):
    return nn.Conv2d(i, o, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(_Holder):
    """resnet.py:30-69 (relu_type='prelu')."""

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.PReLU(num_parameters=planes)
        self.relu2 = nn.PReLU(num_parameters=planes)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride


class ResNet(_Holder):
    """resnet.py:72-124 (ResNet-18 trunk, [2, 2, 2, 2])."""

    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.layer1 = self._make_layer(64, 2)
        self.layer2 = self._make_layer(128, 2, stride=2)
        self.layer3 = self._make_layer(256, 2, stride=2)
        self.layer4 = self._make_layer(512, 2, stride=2)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes, kernel_size=1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, down)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(BasicBlock(planes, planes))
        return nn.Sequential(*layers)


class ResEncoder(_Holder):
    """resnet.py:126-164: Conv3d stem + BN3d + PReLU + MaxPool3d, then ResNet-18."""

    def __init__(self):
        super().__init__()
        self.frontend_nout, self.backend_out = 64, 512
        self.frontend3D = nn.Sequential(
            nn.Conv3d(1, 64, kernel_size=(5, 7, 7), stride=(1, 2, 2), padding=(2, 3, 3), bias=False),
            nn.BatchNorm3d(64), nn.PReLU(num_parameters=64),
            nn.MaxPool3d(kernel_size=(1, 3, 3), stride=(1, 2, 2), padding=(0, 1, 1)))
        self.trunk = ResNet()


class SubModel(_Holder):
    """avhubert.py:187-198."""

    def __init__(self, resnet, input_dim, embed_dim):
        super().__init__()
        self.resnet = resnet
        self.proj = nn.Linear(input_dim, embed_dim)


class HFAttention(_Holder):
    """HF Wav2Vec2Attention projections (k, v, q, out — registration order as HF)."""

    def __init__(self, d):
        super().__init__()
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.q_proj = nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)


class HFFeedForward(_Holder):
    def __init__(self, d, f):
        super().__init__()
        self.intermediate_dense = nn.Linear(d, f)
        self.output_dense = nn.Linear(f, d)


class EncoderLayer(_Holder):
    """AVHubertEncoderLayer (avhubert.py:747-768) on HF Wav2Vec2EncoderLayer."""

    def __init__(self, d, f, eps):
        super().__init__()
        self.attention = HFAttention(d)
        self.layer_norm = nn.LayerNorm(d, eps=eps)
        self.feed_forward = HFFeedForward(d, f)
        self.final_layer_norm = nn.LayerNorm(d, eps=eps)


class PosConvEmbed(_Holder):
    """HF Wav2Vec2PositionalConvEmbedding: weight-normed grouped Conv1d (dim=2)."""

    def __init__(self, d, k, groups):
        super().__init__()
        conv = nn.Conv1d(d, d, kernel_size=k, padding=k // 2, groups=groups)
        self.conv = nn.utils.parametrizations.weight_norm(conv, name="weight", dim=2)


class AVHubertEncoder(_Holder):
    def __init__(self, cfg):
        super().__init__()
        d = cfg.hidden_size
        self.pos_conv_embed = PosConvEmbed(d, cfg.num_conv_pos_embeddings, cfg.num_conv_pos_embedding_groups)
        self.layer_norm = nn.LayerNorm(d, eps=cfg.layer_norm_eps)
        self.layers = nn.ModuleList(EncoderLayer(d, cfg.intermediate_size, cfg.layer_norm_eps)
                                    for _ in range(cfg.num_hidden_layers))


class AVHubertModel(_Holder):
    """avhubert.py:200-297 (fine-tune subset; mask_emb / label_embs_concat kept for keys)."""

    def __init__(self, cfg):
        super().__init__()
        e = cfg.encoder_embed_dim
        self.feature_extractor_audio = SubModel(None, cfg.audio_feat_dim, e)
        self.feature_extractor_video = SubModel(ResEncoder(), 512, e)
        self.embed = 2 * e if cfg.modality_fuse == "concat" else e
        self.post_extract_proj = nn.Linear(self.embed, e) if self.embed != e else None
        self.mask_emb = nn.Parameter(torch.FloatTensor(cfg.audio_feat_dim if cfg.masking_type == "input" else e).uniform_())
        self.encoder = AVHubertEncoder(cfg)
        self.layer_norm = nn.LayerNorm(self.embed)
        final_dim = cfg.final_dim if cfg.final_dim > 0 else e
        self.label_embs_concat = nn.Parameter(torch.FloatTensor(cfg.num_classes, final_dim).uniform_())

    def forward(self, input_features, attention_mask=None, video=None, **kwargs):
        """avhubert.py:546-561 on the engine -> BaseModelOutput(last_hidden_state (B, T, D))."""
        from ..surface import encoder_forward
        return encoder_forward(_e2e(self), input_features, attention_mask=attention_mask, video=video, **kwargs)


class MHA(_Holder):
    """MultiHeadedAttention (attention.py:16-35)."""

    def __init__(self, d):
        super().__init__()
        self.linear_q = nn.Linear(d, d)
        self.linear_k = nn.Linear(d, d)
        self.linear_v = nn.Linear(d, d)
        self.linear_out = nn.Linear(d, d)


class PositionwiseFeedForward(_Holder):
    def __init__(self, d, f):
        super().__init__()
        self.w_1 = nn.Linear(d, f)
        self.w_2 = nn.Linear(f, d)


class DecoderLayer(_Holder):
    def __init__(self, d, f):
        super().__init__()
        self.self_attn = MHA(d)
        self.src_attn = MHA(d)
        self.feed_forward = PositionwiseFeedForward(d, f)
        self.norm1 = nn.LayerNorm(d, eps=1e-12)
        self.norm2 = nn.LayerNorm(d, eps=1e-12)
        self.norm3 = nn.LayerNorm(d, eps=1e-12)


class _PE(_Holder):
    """PositionalEncoding has no parameters (embedding.py:33-87)."""


class Decoder(_Holder):
    def __init__(self, odim, d, f, nblocks):
        super().__init__()
        self.embed = nn.Sequential(nn.Embedding(odim, d), _PE())
        self.decoders = nn.ModuleList(DecoderLayer(d, f) for _ in range(nblocks))
        self.after_norm = nn.LayerNorm(d, eps=1e-12)
        self.output_layer = nn.Linear(d, odim)

    # decoder.py:122-227 on the engine (ESPnet BatchScorerInterface)
    def forward(self, tgt, tgt_mask, memory, memory_mask):
        from ..surface import decoder_forward
        return decoder_forward(_e2e(self), tgt, tgt_mask, memory, memory_mask)

    def forward_one_step(self, tgt, tgt_mask, memory, memory_mask=None, cache=None):
        from ..surface import decoder_forward_one_step
        return decoder_forward_one_step(_e2e(self), tgt, tgt_mask, memory, memory_mask=memory_mask, cache=cache)

    def score(self, ys, state, x):
        from ..surface import decoder_score
        return decoder_score(_e2e(self), ys, state, x)

    def batch_score(self, ys, states, xs):
        from ..surface import decoder_batch_score
        return decoder_batch_score(_e2e(self), ys, states, xs)

    def init_state(self, x):              # scorer_interface.py (decoder state = None)
        return None

    def select_state(self, state, i, new_id=None):
        return None if state is None else state[i]

    def batch_init_state(self, x):
        return None


class CTCHead(_Holder):
    """CTC (ctc.py:12-180): ctc_lo + the loss / log-softmax / argmax entry points on the engine."""

    def __init__(self, odim, d):
        super().__init__()
        self.ctc_lo = nn.Linear(d, odim)

    def forward(self, hs_pad, hlens, ys_pad):
        from ..surface import ctc_forward
        return ctc_forward(_e2e(self), hs_pad, hlens, ys_pad)

    def log_softmax(self, hs_pad):
        from ..surface import ctc_log_softmax
        return ctc_log_softmax(_e2e(self), hs_pad)

    def softmax(self, hs_pad):
        return self.log_softmax(hs_pad).exp_()

    def argmax(self, hs_pad):
        from ..surface import ctc_argmax
        return ctc_argmax(_e2e(self), hs_pad)


CTC = CTCHead


class E2EShell(_Holder):
    """Parameter tree of E2E (e2e_asr_avhubert.py:24-117)."""

    def __init__(self, cfg):
        super().__init__()
        self.encoder = AVHubertModel(cfg)
        self.decoder = Decoder(cfg.odim, cfg.ddim, cfg.dunits, cfg.dlayers)
        self.ctc = CTCHead(cfg.odim, cfg.adim)
        self.blank = 0
        self.sos = self.eos = cfg.odim - 1
        self.odim = cfg.odim
        self.ignore_id = -1
