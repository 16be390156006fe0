"""Input front end on the GPU: the collator's per-clip audio / video transforms
as HIP kernels (avsr_fbank_stack, avsr_video_normalize in libavsr_hip.so), producing the
`audios` (B, 104, T) and `videos` (B, 1, T, 88, 88) tensors `AVHubertAVSR.forward` takes, and
the train-time augmentations (AdaptiveTimeMask, AddNoise, AddMultiSpk, RGB -> gray: avsr_time_mask,
avsr_add_noise, avsr_rgb_to_gray). Media decoding (torchcodec) stays outside: these take decoded
device tensors.

Mirrors src/dataset/avhubert_dataset.py: `cut_or_pad` (:22-33), `FBanksAndStack` (:86-116),
`VideoTransform` (:225-246, eval branch; train RandomCrop = explicit crop offsets), and the
`DataCollator` audio/video part (:335-351). Waveforms and frames are device tensors; there is no
CPU path (the library raises AvsrLibError when it is missing).
"""
import ctypes
import math
import random

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


# ---------------------------------------------------------------------------------------
# train-time augmentation (src/dataset/avhubert_dataset.py:131-222)
# ---------------------------------------------------------------------------------------

def time_mask(x, spans):
    """Zero time steps [start, end) of each clip in place: x (B, L, ...) contiguous device tensor
    of any dtype, spans = one list of (start, end) pairs per clip (host ints; ends past L clip)."""
    assert x.is_cuda and x.is_contiguous() and x.dim() >= 2
    B, Lx = x.shape[0], x.shape[1]
    ns = max((len(s) for s in spans), default=0)
    if ns == 0 or B == 0:
        return x
    tab = torch.zeros(B, ns, 2, dtype=torch.int32)
    for b, sp in enumerate(spans):
        for i, (a, e) in enumerate(sp):
            tab[b, i, 0], tab[b, i, 1] = int(a), int(e)
    tab = tab.to(x.device)
    row = x[0, 0].numel() * x.element_size()
    p = L.fill(L.TimeMaskParams, B=B, L=Lx, nspan=ns, row_bytes=row, clip_stride_bytes=x.stride(0) * x.element_size(),
               x=x, spans=tab)
    L.check(L.load().avsr_time_mask(ctypes.byref(p), L.stream_ptr()), "avsr_time_mask")
    return x


def adaptive_time_mask_spans(length, window, stride):
    """AdaptiveTimeMask.forward's draws (avhubert_dataset.py:140-150), same RNG calls in the same
    order (torch.randint for the pairs, Python's random.randrange for the starts): the spans
    [t_start, t_start + t_end) it zeroes."""
    n_mask = int((length + stride - 0.1) // stride)
    ts = torch.randint(0, window, size=(n_mask, 2))
    spans = []
    for t, t_end in ts.tolist():
        if length - t <= 0:
            continue
        t_start = random.randrange(0, length - t)
        if t_start == t_start + t:
            continue
        spans.append((t_start, t_start + t_end))
    return spans


class AdaptiveTimeMask(torch.nn.Module):
    """avhubert_dataset.py:131-151 on a device tensor x (T, ...): returns a masked copy."""

    def __init__(self, window, stride):
        super().__init__()
        self.window, self.stride = window, stride

    def forward(self, x):
        out = x.clone().contiguous()
        spans = adaptive_time_mask_spans(out.size(0), self.window, self.stride)
        time_mask(out.unsqueeze(0), [spans])
        return out


def add_noise(waveform, noise, snr, lengths=None, out=None):
    """torchaudio.functional.add_noise as the reference calls it (avhubert_dataset.py:178, 214,
    220): waveform, noise (B, L) or (L,) float32 device tensors, snr (B,) or scalar dB:
    y = x + 10^((snr0 - snr) / 20) * noise, snr0 = 10 log10(|x|^2 / |n|^2) over each clip (its first
    lengths[b] samples when given)."""
    one = waveform.dim() == 1
    x = waveform.reshape(1, -1) if one else waveform
    n = noise.reshape(1, -1) if one else noise
    assert x.is_cuda and x.dtype == n.dtype == torch.float32 and x.shape == n.shape
    assert x.stride(1) == 1 and n.stride(1) == 1
    B, Lx = x.shape
    snr_t = torch.as_tensor(snr, dtype=torch.float32).reshape(-1).expand(B).contiguous().to(x.device)
    y = torch.empty_like(x) if out is None else out.reshape(B, Lx)
    ws = torch.empty(2 * 64 * B, dtype=torch.float64, device=x.device)
    lens = None if lengths is None else torch.as_tensor(lengths, dtype=torch.int32).to(x.device)
    p = L.fill(L.AddNoiseParams, B=B, L=Lx, x=x, ldx=x.stride(0), noise=n, ldn=n.stride(0), lengths=lens,
               snr_db=snr_t, y=y, ldy=y.stride(0), ws=ws)
    L.check(L.load().avsr_add_noise(ctypes.byref(p), L.stream_ptr()), "avsr_add_noise")
    return y.reshape(-1) if one else y


class AddNoise(torch.nn.Module):
    """avhubert_dataset.py:154-179: `noise` is the decoded noise waveform on the device ((1, N) or
    (N,), 16 kHz; the reference loads it from `noise_filename` with torchaudio)."""

    def __init__(self, noise=None, snr_target=None):
        super().__init__()
        self.snr_levels = [snr_target] if snr_target else [-5, 0, 5, 10, 15, 20, 999999]
        self.noise = None if noise is None else noise.reshape(1, -1)

    def forward(self, speech):
        # speech: T x 1 -> T x 1
        if self.noise is None:
            return speech
        s = speech.t()
        start_idx = random.randint(0, self.noise.shape[1] - s.shape[1])
        seg = self.noise[:, start_idx:start_idx + s.shape[1]].contiguous()
        snr = random.choice(self.snr_levels)
        return add_noise(s.contiguous(), seg, snr).t()


class AddMultiSpk(torch.nn.Module):
    """avhubert_dataset.py:181-222: mixes 0-2 interfering speakers. `load_audio(entry)` returns
    an entry's decoded waveform (T, 1) on the device (the reference decodes `entry['video']`)."""

    def __init__(self, speech_dataset=None, snr_target=None, interferer_spk=None, load_audio=None):
        super().__init__()
        self.snr_levels = [snr_target] if snr_target else [-5, 0, 5, 10, 15, 20]
        self.interferer_spk = [interferer_spk] if interferer_spk else [0, 0, 1, 2]
        self.speech_dataset = speech_dataset
        self.load_audio = load_audio

    def forward(self, speech):
        if self.speech_dataset is None:
            return speech
        speech_length = speech.size(0) / 16000
        if speech_length < 2:
            return speech
        num_interferer = random.choice(self.interferer_spk)
        interferer_signal = None
        for _ in range(num_interferer):
            interferer = self.load_audio(random.choice(self.speech_dataset))
            interferer_length = interferer.size(0) / 16000
            if 2 <= interferer_length <= 10:
                interferer = cut_or_pad(interferer, len(speech))
                if interferer_signal is None:
                    interferer_signal = interferer
                else:
                    snr_level = random.choice([-5, 0, 5, 10, 15])
                    interferer_signal = add_noise(interferer_signal.t().contiguous(), interferer.t().contiguous(),
                                                  snr_level).t()
        if interferer_signal is None:
            return speech
        snr_level = random.choice(self.snr_levels)
        return add_noise(speech.t().contiguous(), interferer_signal.t().contiguous(), snr_level).t()


def rgb_to_gray(frames):
    """uint8 (..., 3) RGB device frames -> uint8 (...) = cv2.cvtColor(f, cv2.COLOR_RGB2GRAY)
    (load_video, avhubert_dataset.py:45), fixed point (R*4899 + G*9617 + B*1868 + 8192) >> 14."""
    assert frames.is_cuda and frames.dtype == torch.uint8 and frames.shape[-1] == 3 and frames.is_contiguous()
    out = torch.empty(frames.shape[:-1], dtype=torch.uint8, device=frames.device)
    L.check(L.load().avsr_rgb_to_gray(ctypes.c_void_p(frames.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                      out.numel(), L.stream_ptr()), "avsr_rgb_to_gray")
    return out


def random_crop_offsets(h, w, th=88, tw=88):
    """torchvision RandomCrop.get_params draws (avhubert_dataset.py:230): top, left."""
    if h == th and w == tw:
        return 0, 0
    i = torch.randint(0, h - th + 1, size=(1,)).item()
    j = torch.randint(0, w - tw + 1, size=(1,)).item()
    return i, j


class TrainCollator:
    """DataCollator (avhubert_dataset.py:313-353) with the train transforms (VideoTransform /
    AudioTransform 'train', :225-275) on decoded device clips: per clip, in the reference's
    order, RandomCrop(88) + AdaptiveTimeMask(10, 25) on the frames, then cut_or_pad to 640 T
    samples, AdaptiveTimeMask(6400, 16000), AddMultiSpk, AddNoise and FBanksAndStack on the
    audio; collate_pad's zero padding. `noise` / `speech_dataset` + `load_audio` as for AddNoise /
    AddMultiSpk (None: those steps pass the clip through, as in the reference)."""

    def __init__(self, noise=None, speech_dataset=None, load_audio=None, text_transform=None):
        self.vmask = AdaptiveTimeMask(10, 25)
        self.amask = AdaptiveTimeMask(6400, 16000)
        self.multispk = AddMultiSpk(speech_dataset=speech_dataset, load_audio=load_audio)
        self.noise = AddNoise(noise)
        self.text_transform = text_transform

    def __call__(self, wavs, frames, labels=None):
        """wavs: list of (S_i,) or (S_i, 1) float32 device waveforms; frames: list of (T_i, H, W)
        uint8 device frames (gray); labels: optional list of strings (needs text_transform) or
        token lists."""
        dev = frames[0].device
        lens = [f.shape[0] for f in frames]
        tmax = max(lens)
        B = len(frames)
        videos = torch.zeros(B, 1, tmax, 88, 88, device=dev, dtype=torch.float32)
        wav = torch.zeros(B, RATE_RATIO * tmax, device=dev, dtype=torch.float32)
        for b in range(B):
            f = frames[b]
            oy, ox = random_crop_offsets(f.shape[1], f.shape[2])
            spans = adaptive_time_mask_spans(f.shape[0], 10, 25)
            fr = f.contiguous().clone()
            time_mask(fr.unsqueeze(0), [spans])          # zero frames == zero after /255 and crop
            video_transform(fr.unsqueeze(0), offsets=(oy, ox), out=videos[b:b + 1, :, :lens[b]])
            a = cut_or_pad(wavs[b].reshape(-1, 1), RATE_RATIO * lens[b])
            a = self.amask(a)
            a = self.multispk(a)
            a = self.noise(a)
            wav[b, :RATE_RATIO * lens[b]] = a.reshape(-1)
        ns = torch.tensor([RATE_RATIO * t for t in lens], dtype=torch.int64)
        audios = audio_features(wav, ns, T=tmax)
        lengths = torch.tensor(lens, dtype=torch.int64)
        out = {"videos": videos, "audios": audios, "video_lengths": lengths, "audio_lengths": lengths.clone()}
        if labels is not None:
            toks = [self.text_transform.tokenize(l) if isinstance(l, str) else torch.as_tensor(l) for l in labels]
            Lm = max(len(t) for t in toks)
            lab = torch.full((B, Lm), -1, dtype=torch.int64)
            for b, t in enumerate(toks):
                lab[b, :len(t)] = torch.as_tensor(t, dtype=torch.int64)
            out["labels"] = lab
            out["label_lengths"] = torch.tensor([len(t) for t in toks], dtype=torch.int64)
        return out
