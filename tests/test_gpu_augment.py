"""f3 augmentation kernels (avsr_time_mask, avsr_add_noise, avsr_rgb_to_gray) against the CPU
restatement (oracle/augment_oracle.py) and the reference's module behaviour."""
import random

import numpy as np
import pytest
import torch

from avsr_amd import frontend as F
from oracle import augment_oracle as A

pytestmark = pytest.mark.gpu


def test_time_mask_frames_and_audio(dev):
    g = torch.Generator().manual_seed(1)
    frames = torch.randint(0, 256, (3, 375, 96, 96), generator=g, dtype=torch.uint8)
    spans = [[(0, 5), (100, 111), (370, 400)], [], [(-3, 2), (50, 50), (200, 230)]]
    got = F.time_mask(frames.clone().to(dev), spans).cpu().numpy()
    ref = frames.numpy().copy()
    for b, sp in enumerate(spans):
        for a, e in sp:
            ref[b, max(a, 0):max(e, 0)] = 0
    assert np.array_equal(got, ref)
    wav = torch.randn(2, 48000, generator=g)
    sp2 = [[(10, 6410), (47000, 48000)], [(1, 2)]]
    got = F.time_mask(wav.clone().to(dev).unsqueeze(-1), sp2).squeeze(-1).cpu().numpy()
    ref = wav.numpy().copy()
    for b, sp in enumerate(sp2):
        for a, e in sp:
            ref[b, a:e] = 0
    assert np.array_equal(got, ref)


def test_adaptive_time_mask_module(dev):
    x = torch.randn(375, 88, 88)
    for seed in range(3):
        torch.manual_seed(seed); random.seed(seed + 10)
        got = F.AdaptiveTimeMask(10, 25)(x.to(dev)).cpu().numpy()
        torch.manual_seed(seed); random.seed(seed + 10)
        ref = A.adaptive_time_mask(x.numpy(), 10, 25)
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("lengths", [None, [48000, 30000, 17]])
def test_add_noise(dev, lengths):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, 48000, generator=g)
    n = 0.5 * torch.randn(3, 48000, generator=g)
    snr = torch.tensor([-5.0, 10.0, 999999.0])
    got = F.add_noise(x.to(dev), n.to(dev), snr, lengths=lengths).cpu().numpy()
    ref = A.add_noise(x.numpy(), n.numpy(), snr.numpy(), lengths=lengths)
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-6
    # 1-D call form (AddNoise: one clip)
    got1 = F.add_noise(x[0].to(dev), n[0].to(dev), 5.0).cpu().numpy()
    ref1 = A.add_noise(x[0:1].numpy(), n[0:1].numpy(), np.array([5.0]))[0]
    assert np.abs(got1 - ref1).max() / np.abs(ref1).max() < 1e-6


def test_add_noise_and_multispk_modules(dev):
    g = torch.Generator().manual_seed(3)
    speech = torch.randn(48000, 1, generator=g)
    noise = torch.randn(1, 160000, generator=g)
    random.seed(7)
    got = F.AddNoise(noise.to(dev))(speech.to(dev)).cpu().numpy()
    random.seed(7)
    start = random.randint(0, noise.shape[1] - speech.shape[0])
    snr = random.choice([-5, 0, 5, 10, 15, 20, 999999])
    ref = A.add_noise(speech.t().numpy(), noise[:, start:start + speech.shape[0]].numpy(), np.array([snr])).T
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-6
    # interferers: same draws as the reference module, loader returns device waveforms
    pool = [torch.randn(int(16000 * s), 1, generator=g) for s in (3.0, 5.5, 12.0)]
    mod = F.AddMultiSpk(speech_dataset=list(range(3)), load_audio=lambda i: pool[i].to(dev))
    for seed in range(6):
        random.seed(seed)
        out = mod(speech.to(dev)).cpu().numpy()
        random.seed(seed)
        k = random.choice([0, 0, 1, 2])
        sig = None
        for _ in range(k):
            itf = pool[random.choice(list(range(3)))]
            if 2 <= itf.shape[0] / 16000 <= 10:
                itf = F.cut_or_pad(itf, len(speech)).numpy()
                if sig is None:
                    sig = itf
                else:
                    s2 = random.choice([-5, 0, 5, 10, 15])
                    sig = A.add_noise(sig.T, itf.T, np.array([s2])).T
        if sig is None:
            ref = speech.numpy()
        else:
            s1 = random.choice([-5, 0, 5, 10, 15, 20])
            ref = A.add_noise(speech.t().numpy(), sig.T, np.array([s1])).T
        assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-5, seed


def test_rgb_to_gray(dev):
    g = torch.Generator().manual_seed(4)
    rgb = torch.randint(0, 256, (5, 96, 96, 3), generator=g, dtype=torch.uint8)
    got = F.rgb_to_gray(rgb.to(dev)).cpu().numpy()
    assert np.array_equal(got, A.rgb_to_gray(rgb.numpy()))
