"""CPU checks of the front-end oracle (oracle/frontend_oracle.py) -- parity unpinned: the reference
holds no fixture for logfbank and python_speech_features is absent, so the restatement is held to
known answers of its published algorithm -- and of the host-side logic of avsr_amd.frontend."""
import numpy as np
import pytest

from oracle import frontend_oracle as O

# get_filterbanks(26, 512, 16000) edges as published by python_speech_features 0.6 users
BINS_26_512_16K = [0, 2, 4, 7, 10, 13, 16, 20, 24, 29, 34, 40, 46, 53, 60, 68, 77, 87, 97, 109, 122, 136, 152,
                   169, 188, 209, 231, 256]


def test_filterbank_edges_and_shape():
    assert O.filterbank_bins().astype(int).tolist() == BINS_26_512_16K
    fb = O.get_filterbanks()
    assert fb.shape == (26, 257)
    for j in range(26):                       # triangle peaks at 1 on its centre bin
        assert fb[j, BINS_26_512_16K[j + 1]] == pytest.approx(1.0)
        assert fb[j].max() <= 1.0 and fb[j].min() >= 0.0


@pytest.mark.parametrize("n,frames", [(1, 1), (400, 1), (401, 2), (560, 2), (561, 3), (240000, 1499), (16000, 99)])
def test_num_frames(n, frames):
    assert O.num_frames(n) == frames


def test_clip_rows_match_video_frames():
    for t in (1, 2, 25, 375):
        f = O.fbanks_and_stack(np.random.default_rng(t).standard_normal(640 * t).astype(np.float32))
        assert f.shape == (t, 104) and f.dtype == np.float32
        np.testing.assert_allclose(f.mean(1), 0, atol=1e-5)
        np.testing.assert_allclose(f.var(1), 1, atol=1e-3)


def test_silence_is_log_eps():
    feat = O.logfbank(np.zeros(1000, dtype=np.float32))
    np.testing.assert_allclose(feat, np.log(np.finfo(float).eps))


def test_tone_lands_in_its_filter():
    j = 12                                    # filter 12 peaks at bin 46 -> 46 * 16000 / 512 Hz
    hz = BINS_26_512_16K[j + 1] * 16000 / 512
    sig = np.sin(2 * np.pi * hz * np.arange(4000) / 16000).astype(np.float32)
    feat = O.logfbank(sig)
    assert (feat[2:-2].argmax(1) == j).all()


def test_stacker_pads_zero_rows_after_log():
    f = np.arange(5 * 26, dtype=np.float32).reshape(5, 26)
    s = O.stacker(f)
    assert s.shape == (2, 104)
    np.testing.assert_array_equal(s[1, 26:], 0)
    np.testing.assert_array_equal(s[0], f[:4].reshape(-1))


def test_collate_pads_and_cuts():
    rng = np.random.default_rng(3)
    wavs = [rng.standard_normal(640 * 10 + 77).astype(np.float32), rng.standard_normal(640 * 4 - 5).astype(np.float32)]
    out = O.collate_audio(wavs, [10, 4])
    assert out.shape == (2, 104, 10)
    np.testing.assert_array_equal(out[1, :, 4:], 0)
    np.testing.assert_allclose(out[0].T, O.fbanks_and_stack(wavs[0][:6400]))


def test_video_center_crop():
    fr = np.arange(2 * 3 * 96 * 96, dtype=np.int64).reshape(2, 3, 96, 96).astype(np.uint8)
    v = O.video_eval_transform(fr)
    assert v.shape == (2, 1, 3, 88, 88)
    np.testing.assert_allclose(v[1, 0, 2, 0, 0], (fr[1, 2, 4, 4] / 255.0 - 0.421) / 0.165, rtol=1e-6)


def test_host_mirror_bins_and_rows():
    from avsr_amd import frontend as F
    assert F._BINS == BINS_26_512_16K
    for n in (1, 399, 400, 401, 560, 561, 16000, 240000):
        assert F.num_rows(n) == -(-O.num_frames(n) // 4)
