"""Front-end HIP kernels (log-fbank + stack + LN, lip-frame crop/normalise) vs the CPU oracle."""
import numpy as np
import pytest
import torch

from avsr_amd import frontend as F
from oracle import frontend_oracle as O

pytestmark = pytest.mark.gpu

# fp32 DFT / log / LN on the device vs float64 numpy: features are O(1) after the LayerNorm
TOL_AUDIO = 2e-3


def test_fbank_stack_ragged(dev):
    rng = np.random.default_rng(11)
    ts = [25, 17, 1, 9]
    wavs = [(0.3 * rng.standard_normal(640 * t + 123)).astype(np.float32) for t in ts]
    ref = O.collate_audio(wavs, ts)
    S = 640 * max(ts)
    w = torch.zeros(len(ts), S)
    for b, (x, t) in enumerate(zip(wavs, ts)):
        w[b, :640 * t] = torch.from_numpy(O.cut_or_pad(x, 640 * t))
    got = F.audio_features(w.to(dev), torch.tensor([640 * t for t in ts]), T=max(ts))
    assert got.shape == ref.shape
    err = (got.cpu() - torch.from_numpy(ref)).abs().max().item()
    assert err < TOL_AUDIO, err


@pytest.mark.parametrize("n", [1, 250, 400, 401, 561, 16000])
def test_fbank_short_and_odd_lengths(dev, n):
    x = (0.5 * np.random.default_rng(n).standard_normal(n)).astype(np.float32)
    ref = O.fbanks_and_stack(x)
    got = F.FBanksAndStack()(torch.from_numpy(x).to(dev)[:, None]).cpu().numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < TOL_AUDIO


def test_fbank_full_clip_c2(dev):
    """C2 clip length (15 s at 25 fps = 240000 samples -> 375 rows); two clips."""
    rng = np.random.default_rng(5)
    wavs = [(0.1 * rng.standard_normal(240000)).astype(np.float32) for _ in range(2)]
    ref = O.collate_audio(wavs, [375, 375])
    w = torch.from_numpy(np.stack(wavs)).to(dev)
    got = F.audio_features(w, torch.tensor([240000, 240000]))
    assert got.shape == (2, 104, 375)
    assert (got.cpu() - torch.from_numpy(ref)).abs().max().item() < TOL_AUDIO


@pytest.mark.parametrize("offsets", [None, (0, 8), (5, 3)])
def test_video_normalize(dev, offsets):
    fr = np.random.default_rng(2).integers(0, 256, size=(2, 7, 96, 96), dtype=np.uint8)
    got = F.video_transform(torch.from_numpy(fr).to(dev), offsets=offsets).cpu().numpy()
    oy, ox = offsets or (4, 4)
    ref = ((fr[:, :, oy:oy + 88, ox:ox + 88].astype(np.float64) / 255.0 - 0.421) / 0.165)[:, None]
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-5


def test_collate_matches_reference_collator(dev):
    rng = np.random.default_rng(8)
    ts = [12, 5]
    wavs = [(0.2 * rng.standard_normal(640 * t - 37)).astype(np.float32) for t in ts]
    frames = [rng.integers(0, 256, size=(t, 96, 96), dtype=np.uint8) for t in ts]
    out = F.collate([torch.from_numpy(w).to(dev) for w in wavs], [torch.from_numpy(f).to(dev) for f in frames])
    assert (out["audios"].cpu() - torch.from_numpy(O.collate_audio(wavs, ts))).abs().max().item() < TOL_AUDIO
    v = out["videos"].cpu().numpy()
    assert v.shape == (2, 1, 12, 88, 88)
    np.testing.assert_allclose(v[1, :, :5], O.video_eval_transform(frames[1][None])[0], atol=1e-5)
    assert (v[1, :, 5:] == 0).all()
    assert out["video_lengths"].tolist() == ts
