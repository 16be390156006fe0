"""CPU restatement of the AVSR input front end -- TEST INFRASTRUCTURE
ONLY: imported by tests/ as the checker of the HIP front-end kernels, never by the product path.

Audio: `FBanksAndStack.forward` (reference src/dataset/avhubert_dataset.py:86-116) =
python_speech_features 0.6 `logfbank(x, samplerate=16000)` (called at :111) -> `stacker` (:91-106,
zero rows appended to a multiple of 4, then 4 consecutive frames concatenated) -> per-frame
LayerNorm over the 104 features (no affine, eps 1e-5, :114-115). `cut_or_pad` (:22-33) fits the
waveform to 640 samples per video frame (:335); `collate_pad` (:280-311) pads rows with 0.0.

python_speech_features is a third-party dependency (requirements pin: python_speech_features
0.6) absent from this image and from /root/reference; its published algorithm is restated here:
  logfbank = log(fbank(...)[0]);  fbank: preemphasis(0.97) -> framesig(winlen 0.025 s = 400
  samples, winstep 0.01 s = 160, rectangular window, zero-padded to cover the signal:
  numframes = 1 if len <= 400 else 1 + ceil((len - 400) / 160)) -> powspec = |rfft(frame, 512)|^2
  / 512 -> dot with 26 triangular mel filters (get_filterbanks: mel = 2595 log10(1 + hz/700),
  26 + 2 points linear in mel over [0, 8000] Hz, bin = floor((nfft + 1) * hz / samplerate)) ->
  zeros replaced by float eps.
PARITY UNPINNED: the reference holds no fixture for this path and the library cannot be run
here; the restatement is checked by known-answer properties in tests/test_frontend_oracle.py.

Video (eval): `VideoTransform('test')` (:225-246): x / 255 -> CenterCrop(88) -> Normalize(0.421,
0.165); the collator permutes (B, T, 1, H, W) -> (B, 1, T, H, W) (:350).
"""
import math

import numpy as np

SAMPLE_RATE = 16000
FRAME_LEN = 400
FRAME_STEP = 160
NFFT = 512
NFILT = 26
STACK = 4
PREEMPH = 0.97
LN_EPS = 1e-5
RATE_RATIO = 640          # audio samples per video frame (avhubert_dataset.py:318)


def hz2mel(hz):
    return 2595 * np.log10(1 + hz / 700.0)


def mel2hz(mel):
    return 700 * (10 ** (mel / 2595.0) - 1)


def filterbank_bins(nfilt=NFILT, nfft=NFFT, samplerate=SAMPLE_RATE, lowfreq=0, highfreq=None):
    """get_filterbanks' bin edges: floor((nfft + 1) * mel2hz(linspace(lowmel, highmel, nfilt + 2)) / sr)."""
    highfreq = highfreq or samplerate / 2
    melpoints = np.linspace(hz2mel(lowfreq), hz2mel(highfreq), nfilt + 2)
    return np.floor((nfft + 1) * mel2hz(melpoints) / samplerate)


def get_filterbanks(nfilt=NFILT, nfft=NFFT, samplerate=SAMPLE_RATE):
    b = filterbank_bins(nfilt, nfft, samplerate)
    fb = np.zeros([nfilt, nfft // 2 + 1])
    for j in range(nfilt):
        for i in range(int(b[j]), int(b[j + 1])):
            fb[j, i] = (i - b[j]) / (b[j + 1] - b[j])
        for i in range(int(b[j + 1]), int(b[j + 2])):
            fb[j, i] = (b[j + 2] - i) / (b[j + 2] - b[j + 1])
    return fb


def num_frames(n):
    return 1 if n <= FRAME_LEN else 1 + int(math.ceil((1.0 * n - FRAME_LEN) / FRAME_STEP))


def logfbank(sig):
    """python_speech_features 0.6 logfbank(sig, samplerate=16000) with its defaults."""
    sig = np.asarray(sig)
    emph = np.append(sig[0], sig[1:] - PREEMPH * sig[:-1])
    nf = num_frames(len(emph))
    padlen = (nf - 1) * FRAME_STEP + FRAME_LEN
    pad = np.concatenate((emph, np.zeros((padlen - len(emph),), dtype=emph.dtype)))
    idx = np.arange(FRAME_LEN)[None, :] + FRAME_STEP * np.arange(nf)[:, None]
    frames = pad[idx] * np.ones((FRAME_LEN,))
    pspec = 1.0 / NFFT * np.square(np.absolute(np.fft.rfft(frames, NFFT)))
    feat = np.dot(pspec, get_filterbanks().T)
    feat = np.where(feat == 0, np.finfo(float).eps, feat)
    return np.log(feat)


def stacker(feats, stack_order=STACK):
    """avhubert_dataset.py:91-106."""
    feat_dim = feats.shape[1]
    if len(feats) % stack_order != 0:
        res = np.zeros([stack_order - len(feats) % stack_order, feat_dim]).astype(feats.dtype)
        feats = np.concatenate([feats, res], axis=0)
    return feats.reshape((-1, stack_order, feat_dim)).reshape(-1, stack_order * feat_dim)


def fbanks_and_stack(wav):
    """FBanksAndStack.forward (avhubert_dataset.py:108-116): [samples] -> [rows][104] float32."""
    f = stacker(logfbank(wav).astype(np.float32))
    mu = f.mean(1, keepdims=True, dtype=np.float64)
    var = ((f - mu) ** 2).mean(1, keepdims=True)
    return ((f - mu) / np.sqrt(var + LN_EPS)).astype(np.float32)


def cut_or_pad(wav, size):
    """avhubert_dataset.py:22-33 on a 1-D waveform."""
    wav = np.asarray(wav)
    if len(wav) < size:
        return np.concatenate([wav, np.zeros(size - len(wav), dtype=wav.dtype)])
    return wav[:size]


def collate_audio(wavs, video_frames):
    """per clip: cut_or_pad to 640 * T, FBanksAndStack; then collate_pad (0.0) and permute to the
    model's (B, 104, Tmax) layout (avhubert_dataset.py:335-351)."""
    feats = [fbanks_and_stack(cut_or_pad(w, RATE_RATIO * t)) for w, t in zip(wavs, video_frames)]
    tmax = max(len(f) for f in feats)
    out = np.zeros((len(feats), STACK * NFILT, tmax), dtype=np.float32)
    for b, f in enumerate(feats):
        out[b, :, :len(f)] = f.T
    return out


def video_eval_transform(frames_u8, crop=88, mean=0.421, std=0.165):
    """(B, T, H, W) uint8 -> (B, 1, T, crop, crop) float32: /255, CenterCrop, Normalize."""
    B, T, H, W = frames_u8.shape
    oy, ox = int(round((H - crop) / 2.0)), int(round((W - crop) / 2.0))
    x = frames_u8[:, :, oy:oy + crop, ox:ox + crop].astype(np.float32) / np.float32(255.0)
    return ((x - np.float32(mean)) / np.float32(std))[:, None]
