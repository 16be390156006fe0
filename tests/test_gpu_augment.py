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


def _oracle_multispk(speech, pool):
    """AddMultiSpk.forward's draws (avhubert_dataset.py:196-222) on numpy (S, 1) clips."""
    if speech.shape[0] / 16000 < 2:
        return speech
    sig = None
    for _ in range(random.choice([0, 0, 1, 2])):
        itf = pool[random.choice(list(range(len(pool))))]
        if 2 <= itf.shape[0] / 16000 <= 10:
            itf = F.cut_or_pad(torch.from_numpy(itf), len(speech)).numpy()
            if sig is None:
                sig = itf
            else:
                sig = A.add_noise(sig.T, itf.T, np.array([random.choice([-5, 0, 5, 10, 15])])).T
    if sig is None:
        return speech
    return A.add_noise(speech.T, sig.T, np.array([random.choice([-5, 0, 5, 10, 15, 20])])).T


def test_train_collator(dev):
    """DataCollator with the 'train' transforms (avhubert_dataset.py:225-275, 313-353): the device
    collator against the same pipeline on numpy, with the RNG draws replayed in the same order."""
    from oracle import frontend_oracle as O
    g = torch.Generator().manual_seed(5)
    ts = [75, 60]
    frames = [torch.randint(0, 256, (t, 96, 96), generator=g, dtype=torch.uint8) for t in ts]
    wavs = [0.2 * torch.randn(640 * t - 50, generator=g) for t in ts]
    noise = 0.3 * torch.randn(1, 200000, generator=g)
    pool = [0.2 * torch.randn(int(16000 * s), 1, generator=g) for s in (2.5, 4.0, 11.0)]
    col = F.TrainCollator(noise=noise.to(dev), speech_dataset=list(range(3)), load_audio=lambda i: pool[i].to(dev))
    for seed in range(3):
        torch.manual_seed(seed); random.seed(100 + seed)
        out = col([w.to(dev) for w in wavs], [f.to(dev) for f in frames], labels=[[3, 9, 4], [7]])
        torch.manual_seed(seed); random.seed(100 + seed)
        vids, auds = [], []
        for f, w, t in zip(frames, wavs, ts):
            oy = torch.randint(0, 96 - 88 + 1, size=(1,)).item()
            ox = torch.randint(0, 96 - 88 + 1, size=(1,)).item()
            x = f.numpy()[:, oy:oy + 88, ox:ox + 88].astype(np.float32) / np.float32(255.0)
            x = A.adaptive_time_mask(x, 10, 25)
            vids.append((x - np.float32(0.421)) / np.float32(0.165))
            a = O.cut_or_pad(w.numpy(), 640 * t)[:, None]
            a = A.adaptive_time_mask(a, 6400, 16000)
            a = _oracle_multispk(a, [p.numpy() for p in pool])
            start = random.randint(0, noise.shape[1] - a.shape[0])
            snr = random.choice([-5, 0, 5, 10, 15, 20, 999999])
            a = A.add_noise(a.T, noise[:, start:start + a.shape[0]].numpy(), np.array([snr])).T
            auds.append(a[:, 0].astype(np.float32))
        v = out["videos"].cpu().numpy()
        assert v.shape == (2, 1, 75, 88, 88)
        for b, t in enumerate(ts):
            assert np.abs(v[b, 0, :t] - vids[b]).max() < 1e-5, seed
            assert (v[b, 0, t:] == 0).all()
        ref = O.collate_audio(auds, ts)
        assert (out["audios"].cpu() - torch.from_numpy(ref)).abs().max().item() < 2e-3, seed
        assert out["labels"].tolist() == [[3, 9, 4], [7, -1, -1]]
        assert out["video_lengths"].tolist() == ts and out["label_lengths"].tolist() == [3, 1]
