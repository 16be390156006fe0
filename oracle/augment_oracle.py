"""CPU restatement of the train-time augmentations (TEST INFRASTRUCTURE ONLY: imported by tests/,
never by the product path) — SURVEY.md §8 f3.

  * AdaptiveTimeMask (src/dataset/avhubert_dataset.py:131-151): the reference loop itself on a
    numpy copy, with its RNG calls (torch.randint, random.randrange) in the same order;
  * torchaudio.functional.add_noise (torchaudio 2.x, called at avhubert_dataset.py:178, 214, 220;
    torchaudio is not importable here): energy = ||x||^2 over the last dim (masked to `lengths`),
    snr0 = 10 (log10 E_x - log10 E_n), y = x + 10^((snr0 - snr) / 20) * n;
  * cv2.cvtColor(..., COLOR_RGB2GRAY) on uint8 (load_video :45; cv2 absent here): OpenCV's fixed
    point with yuv_shift 14, Y = (4899 R + 9617 G + 1868 B + 2^13) >> 14.
Parity: unpinned by reference fixtures (torchaudio / cv2 / torchcodec are not installed and the
reference holds no vectors for these transforms); the tests use known answers instead (pure-colour
gray levels 76 / 150 / 29, the SNR the mix achieves, the masking loop itself).
"""
import random

import numpy as np
import torch


def adaptive_time_mask(x, window, stride):
    """avhubert_dataset.py:137-151 verbatim in behaviour, on a numpy array (T, ...)."""
    cloned = np.array(x, copy=True)
    length = cloned.shape[0]
    n_mask = int((length + stride - 0.1) // stride)
    ts = torch.randint(0, window, size=(n_mask, 2))
    for t, t_end in ts.tolist():
        if length - t <= 0:
            continue
        t_start = random.randrange(0, length - t)
        if t_start == t_start + t:
            continue
        t_end += t_start
        cloned[t_start:t_end] = 0
    return cloned


def add_noise(x, n, snr, lengths=None):
    """torchaudio.functional.add_noise over the last dim, energies in float64."""
    x = np.asarray(x, dtype=np.float64)
    n = np.asarray(n, dtype=np.float64)
    L = x.shape[-1]
    if lengths is not None:
        mask = np.arange(L)[None, :] < np.asarray(lengths)[:, None]
    else:
        mask = np.ones(x.shape, dtype=bool)
    es = np.sum(np.where(mask, x * x, 0.0), axis=-1)
    en = np.sum(np.where(mask, n * n, 0.0), axis=-1)
    with np.errstate(divide="ignore"):
        snr0 = 10.0 * (np.log10(es) - np.log10(en))
    scale = 10.0 ** ((snr0 - np.asarray(snr, dtype=np.float64)) / 20.0)
    return np.where(mask, x + scale[..., None] * n, x)


def rgb_to_gray(rgb):
    """uint8 (..., 3) -> uint8 (...), OpenCV RGB2GRAY fixed point."""
    r = rgb[..., 0].astype(np.uint32)
    g = rgb[..., 1].astype(np.uint32)
    b = rgb[..., 2].astype(np.uint32)
    return ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)
