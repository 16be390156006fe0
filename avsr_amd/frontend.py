"""Input front end on the GPU: the collator's per-clip audio / video transforms
as HIP kernels (avsr_fbank_stack, avsr_video_normalize in libavsr_hip.so), producing the
`audios` (B, 104, T) and `videos` (B, 1, T, 88, 88) tensors `AVHubertAVSR.forward` takes.

Mirrors src/dataset/avhubert_dataset.py: `cut_or_pad` (:22-33), `FBanksAndStack` (:86-116),
`VideoTransform` (:225-246, eval branch; train RandomCrop = explicit crop offsets), and the
`DataCollator` audio/video part (:335-351). Waveforms and frames are device tensors; there is no
CPU path (the library raises AvsrLibError when it is missing).
"""
import ctypes
import math

import torch

from . import _lib as L

SAMPLE_RATE, FRAME_LEN, FRAME_STEP, NFFT, NFILT, STACK = 16000, 400, 160, 512, 26, 4
RATE_RATIO = 640


def _filter_bins():
    """get_filterbanks' edges (python_speech_features 0.6): floor(513 * mel2hz(mel points) / sr)."""
    hz2mel = lambda hz: 2595 * math.log10(1 + hz / 700.0)          # noqa: E731
    lo, hi = hz2mel(0), hz2mel(SAMPLE_RATE / 2)
    pts = [lo + (hi - lo) * i / (NFILT + 1) for i in range(NFILT + 2)]
    return [int(math.floor((NFFT + 1) * (700 * (10 ** (m / 2595.0) - 1)) / SAMPLE_RATE)) for m in pts]


_BINS = _filter_bins()


def num_rows(n_samples):
    """stacked rows of a clip with n samples (frames = 1 + ceil((n - 400) / 160), 4 per row)."""
    nf = 1 if n_samples <= FRAME_LEN else 1 + -(-(n_samples - FRAME_LEN) // FRAME_STEP)
    return -(-nf // STACK)


def cut_or_pad(wav, size):
    """avhubert_dataset.py:22-33 along dim 0 (zero padding / truncation)."""
    if wav.shape[0] < size:
        return torch.nn.functional.pad(wav, (0, 0) * (wav.dim() - 1) + (0, size - wav.shape[0]))
    return wav[:size]


def audio_features(wav, n_samples, T=None, out=None):
    """wav (B, S) float32 on the GPU, n_samples (B,) int64 (samples used per clip) ->
    (B, 104, T) float32: logfbank -> stack 4 -> per-row LayerNorm, zero rows beyond a clip."""
    assert wav.is_cuda and wav.dtype == torch.float32 and wav.dim() == 2 and wav.stride(1) == 1
    B = wav.shape[0]
    ns = n_samples.to(device=wav.device, dtype=torch.int64).contiguous()
    if T is None:
        T = max(num_rows(int(n)) for n in n_samples.tolist()) if B else 0
    if out is None:
        out = torch.empty(B, STACK * NFILT, T, device=wav.device, dtype=torch.float32)
    p = L.FbankParams()
    p.B, p.T, p.wav, p.ldw, p.n_samples = B, T, wav.data_ptr(), wav.stride(0), ns.data_ptr()
    for i, b in enumerate(_BINS):
        p.bins[i] = b
    p.preemph, p.ln_eps, p.out = 0.97, 1e-5, out.data_ptr()
    L.check(L.load().avsr_fbank_stack(ctypes.byref(p), L.stream_ptr()), "avsr_fbank_stack")
    return out


class FBanksAndStack(torch.nn.Module):
    """avhubert_dataset.py:86-116 on one clip: x (S, 1) or (S,) float32 GPU -> (rows, 104)."""

    def __init__(self, stack_order=4):
        super().__init__()
        if stack_order != STACK:
            raise ValueError("the device kernel stacks 4 frames (the reference's only setting)")
        self.stack_order = stack_order

    def forward(self, x):
        w = x.reshape(1, -1).contiguous()
        n = torch.tensor([w.shape[1]], dtype=torch.int64)
        return audio_features(w, n)[0].t().contiguous()


def video_transform(frames, crop=88, offsets=None, mean=0.421, std=0.165, out=None):
    """frames (B, T, H, W) uint8 GPU -> (B, 1, T, crop, crop) float32 = Normalize(CenterCrop(x/255))
    (VideoTransform 'test'); `offsets=(oy, ox)` gives the train branch's RandomCrop position."""
    assert frames.is_cuda and frames.dtype == torch.uint8 and frames.dim() == 4 and frames.is_contiguous()
    B, T, H, W = frames.shape
    oy, ox = offsets if offsets is not None else (int(round((H - crop) / 2.0)), int(round((W - crop) / 2.0)))
    if out is None:
        out = torch.empty(B, 1, T, crop, crop, device=frames.device, dtype=torch.float32)
    p = L.VideoNormParams()
    p.B, p.T, p.H, p.W, p.crop, p.oy, p.ox = B, T, H, W, crop, oy, ox
    p.frames, p.mean, p.std, p.out = frames.data_ptr(), mean, std, out.data_ptr()
    L.check(L.load().avsr_video_normalize(ctypes.byref(p), L.stream_ptr()), "avsr_video_normalize")
    return out


def collate(wavs, frames):
    """DataCollator audio/video part (avhubert_dataset.py:335-351) for clips already on the GPU:
    wavs: list of 1-D float32 waveforms, frames: list of (T_i, H, W) uint8 -> dict with `videos`
    (B, 1, Tmax, 88, 88), `audios` (B, 104, Tmax), `video_lengths`, `audio_lengths`."""
    lens = [f.shape[0] for f in frames]
    tmax = max(lens)
    dev = frames[0].device
    wav = torch.zeros(len(wavs), RATE_RATIO * tmax, device=dev, dtype=torch.float32)
    for b, (w, t) in enumerate(zip(wavs, lens)):
        wav[b, :RATE_RATIO * t] = cut_or_pad(w.reshape(-1), RATE_RATIO * t)
    ns = torch.tensor([RATE_RATIO * t for t in lens], dtype=torch.int64)
    fr = torch.zeros(len(frames), tmax, *frames[0].shape[1:], device=dev, dtype=torch.uint8)
    for b, f in enumerate(frames):
        fr[b, :f.shape[0]] = f
    videos = video_transform(fr)
    for b, t in enumerate(lens):          # collate_pad fills padded frames with 0.0 after the transform
        videos[b, :, t:] = 0
    audios = audio_features(wav, ns, T=tmax)
    lengths = torch.tensor(lens, dtype=torch.int64)
    return {"videos": videos, "audios": audios, "video_lengths": lengths, "audio_lengths": lengths.clone()}
