"""f3 augmentation: oracle known answers and the host-side span draws (CPU only)."""
import random

import numpy as np
import torch

from avsr_amd.frontend import adaptive_time_mask_spans
from oracle import augment_oracle as A


def test_rgb_to_gray_known_levels():
    px = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [128, 128, 128]], np.uint8)
    # OpenCV's documented RGB2GRAY results for pure red / green / blue, white, black, mid grey
    assert A.rgb_to_gray(px).tolist() == [76, 150, 29, 255, 0, 128]


def test_add_noise_reaches_target_snr():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((3, 16000))
    n = 0.3 * rng.standard_normal((3, 16000))
    snr = np.array([-5.0, 0.0, 20.0])
    y = A.add_noise(x, n, snr)
    got = 10 * np.log10((x ** 2).sum(-1) / ((y - x) ** 2).sum(-1))
    np.testing.assert_allclose(got, snr, atol=1e-9)
    # lengths: samples past a clip's length are untouched and do not enter the energies
    y2 = A.add_noise(x, n, snr, lengths=[8000, 16000, 100])
    assert np.array_equal(y2[0, 8000:], x[0, 8000:]) and np.array_equal(y2[2, 100:], x[2, 100:])
    got2 = 10 * np.log10((x[0, :8000] ** 2).sum() / ((y2[0, :8000] - x[0, :8000]) ** 2).sum())
    assert abs(got2 - snr[0]) < 1e-9


def test_time_mask_spans_match_reference_loop():
    for length, window, stride in ((375, 10, 25), (240000, 6400, 16000), (7, 10, 25)):
        torch.manual_seed(3); random.seed(4)
        spans = adaptive_time_mask_spans(length, window, stride)
        torch.manual_seed(3); random.seed(4)
        ref = A.adaptive_time_mask(np.ones(length, np.float32), window, stride)
        got = np.ones(length, np.float32)
        for a, e in spans:
            got[a:e] = 0
        assert np.array_equal(got, ref)
