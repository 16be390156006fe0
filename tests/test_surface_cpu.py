"""Host-side checks of the drop-in surface (no GPU): checkpoint round trip with the
reference's keys, the modality-dropout draw rule, mask handling, refused dtypes."""
import types

import numpy as np
import pytest
import torch

from avsr_amd.avhubert_avsr_model import AVHubertAVSR
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from avsr_amd.engine import Engine
from avsr_amd.surface import lengths_from_mask
from oracle.weights import NO_DROPOUT, TINY_CONFIG
from tests.oracle_util import golden_state, load_golden, load_golden_full


def test_save_from_pretrained_round_trip(tmp_path):
    """HF save_pretrained / from_pretrained(local_dir) (script/evaluation.py:89-91,
    script/train.py:221-237): config.json model_type + model.safetensors with the reference's
    keys and shapes; the loaded model is bit-identical and in eval mode."""
    g = load_golden()
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
    m.save_pretrained(tmp_path)
    import json
    cfg = json.load(open(tmp_path / "config.json"))
    assert cfg["model_type"] == "avhubert_avsr" and cfg["hidden_size"] == TINY_CONFIG["hidden_size"]
    from safetensors.numpy import load_file
    st = load_file(str(tmp_path / "model.safetensors"))
    want = {str(k): tuple(int(x) for x in s.split(",") if x) for k, s in zip(g["param_keys"], g["param_shapes"])}
    assert {k: tuple(v.shape) for k, v in st.items()} == want
    m2 = AVHubertAVSR.from_pretrained(str(tmp_path))
    assert not m2.training
    sd1, sd2 = m.state_dict(), m2.state_dict()
    assert all(torch.equal(sd1[k], sd2[k]) for k in sd1)


def test_full_size_keys_match_reference():
    g = load_golden_full()
    m = AVHubertAVSR(AVHubertAVSRConfig(odim=5049))
    got = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    want = {str(k): tuple(int(x) for x in s.split(",") if x) for k, s in zip(g["param_keys"], g["param_shapes"])}
    assert got == want


@pytest.mark.parametrize("p_mod,p_audio", [(0.5, 0.5), (0.3, 0.7), (0.0, 0.5), (1.0, 0.0)])
def test_modality_dropout_draws_match_reference_rule(p_mod, p_audio):
    """avhubert.py:476-482: two np.random.random() draws per training forward,
    unconditionally; drop a modality if the first < modality_dropout, audio if the second <
    audio_dropout. Same global RNG and order => same decisions as the reference."""
    cfg = AVHubertAVSRConfig(**TINY_CONFIG, modality_dropout=p_mod, audio_dropout=p_audio)
    fake = types.SimpleNamespace(cfg=cfg)
    np.random.seed(123)
    got = [Engine.draw_modality(fake, True) for _ in range(200)]
    np.random.seed(123)
    want = []
    for _ in range(200):
        a, b = np.random.random(), np.random.random()
        want.append(("audio_off" if b < p_audio else "video_off") if a < p_mod else None)
    assert got == want
    np.random.seed(5)
    assert Engine.draw_modality(fake, False) is None
    assert np.random.random() == np.random.RandomState(5).random_sample()   # eval draws nothing


def test_modality_config_fixed_streams():
    for mod, want in (("audio", "video_off"), ("video", "audio_off")):
        fake = types.SimpleNamespace(cfg=AVHubertAVSRConfig(**TINY_CONFIG, modality=mod))
        assert Engine.draw_modality(fake, True) == want
        assert Engine.draw_modality(fake, False) == want


def test_lengths_from_mask():
    m = torch.tensor([[1, 1, 1, 0], [1, 1, 1, 1]], dtype=torch.bool)
    assert lengths_from_mask(m, 2, 4).tolist() == [3, 4]
    assert lengths_from_mask(m.unsqueeze(1), 2, 4).tolist() == [3, 4]
    assert lengths_from_mask(None, 2, 4).tolist() == [4, 4]
    with pytest.raises(NotImplementedError):
        lengths_from_mask(torch.tensor([[1, 0, 1, 0]], dtype=torch.bool), 1, 4)


def test_refused_dtypes_and_cpu_path():
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT))
    with pytest.raises(NotImplementedError):
        m.half()
    with pytest.raises(NotImplementedError):
        m.to(torch.float16)
    assert m.to("cpu") is m          # no engine yet: a plain module move
    with pytest.raises(RuntimeError):
        m.avsr.engine("cpu")
