"""TEST INFRASTRUCTURE — deterministic per-tensor weight recipe.

Used only by tests/, tests/golden/make_golden.py, bench.py's cpu_baseline leg and
__graft_entry__.smoke(). Weights are never committed: both the golden-vector generator
(which loads them into the reference model) and the parity tests (which load them into
the oracle and into the HIP model) regenerate them from (key, shape, seed).

Recipe per state-dict key (numpy Generator(PCG64(seed ^ crc32(key)))), N = standard normal:
  running_var U(0.5, 1.5) · running_mean 0.1·N · num_batches_tracked 0
  PReLU weight 0.25 + 0.05·N · other 1-D weight (BN / LN / weight-norm g) 1 + 0.1·N
  bias 0.02·N · everything else (linear / conv / embedding / weight-norm v) 0.02·N
"""
import zlib

import numpy as np


def _is_prelu(key):
    # resnet.py:44-48 (BasicBlock relu1/relu2 = PReLU), :129-131 (frontend3D.2 = PReLU)
    return ".relu" in key or key.endswith("frontend3D.2.weight")


def gen_tensor(key, shape, seed=0, dtype=np.float32):
    rng = np.random.Generator(np.random.PCG64((seed ^ zlib.crc32(key.encode())) & 0xFFFFFFFF))
    shape = tuple(int(s) for s in shape)
    if key.endswith("num_batches_tracked"):
        return np.zeros(shape, dtype=np.int64)
    if key.endswith("running_var"):
        return rng.uniform(0.5, 1.5, size=shape).astype(dtype)
    if key.endswith("running_mean"):
        return (0.1 * rng.standard_normal(shape)).astype(dtype)
    n = rng.standard_normal(shape)
    if key.endswith("bias"):
        return (0.02 * n).astype(dtype)
    if key.endswith("weight") and len(shape) == 1:
        if _is_prelu(key):
            return (0.25 + 0.05 * n).astype(dtype)
        return (1.0 + 0.1 * n).astype(dtype)
    if key.endswith("original0"):  # weight-norm magnitude g (1, 1, k)
        return (1.0 + 0.1 * n).astype(dtype)
    return (0.02 * n).astype(dtype)


def make_state_dict(shapes, seed=0):
    """shapes: {key: shape} -> {key: np.ndarray}"""
    return {k: gen_tensor(k, s, seed) for k, s in shapes.items()}


# Tiny configuration used by the golden vectors (19 M params)
TINY_CONFIG = dict(
    odim=5049, adim=256, ddim=256, dheads=4, dunits=1024, dlayers=1,
    hidden_size=256, encoder_embed_dim=256, num_attention_heads=4,
    intermediate_size=1024, num_hidden_layers=2,
)

# all dropouts off for parity (SURVEY.md §7 "Random training features can't be bit-matched")
NO_DROPOUT = dict(
    dropout_rate=0.0, transformer_attn_dropout_rate=0.0, dropout_input=0.0, dropout_features=0.0,
    hidden_dropout=0.0, attention_dropout=0.0, activation_dropout=0.0, modality_dropout=0.0,
    dropout=0.0, feat_proj_dropout=0.0, final_dropout=0.0, layerdrop=0.0,
)


def make_inputs(B=2, T=25, lengths=(25, 19), labels=((5, 17, 301, 42, 4000, 9), (77, 5047, 1, 2)), seed=1234):
    """Seeded synthetic batch in the DataCollator layout (src/dataset/avhubert_dataset.py:313-353).

    videos: uint8 lip frames (B, T, 96, 96) center-cropped to 88 (offset 4), /255,
    (x - 0.421) / 0.165 -> float32 (B, 1, T, 88, 88); padded frames are zero
    (collate_pad pads with 0 after normalisation).
    audios: standard normal (B, T, 104) -> per-frame LayerNorm (no affine) -> (B, 104, T).
    labels: int64 (B, Lmax) padded with -1.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    frames = rng.integers(0, 256, size=(B, T, 96, 96), dtype=np.uint8)
    feats = rng.standard_normal((B, T, 104)).astype(np.float32)
    return frames, feats, np.array(lengths, dtype=np.int64), labels


def collate(frames, feats, lengths, labels):
    """numpy -> the collator's float32/int64 arrays (video normalisation as VideoTransform
    'val': avhubert_dataset.py:225-246; audio per-frame LN as FBanksAndStack :110-116)."""
    B, T = frames.shape[:2]
    v = frames[:, :, 4:92, 4:92].astype(np.float32) / 255.0
    v = (v - 0.421) / 0.165
    a = feats.astype(np.float64)
    a = (a - a.mean(-1, keepdims=True)) / np.sqrt(a.var(-1, keepdims=True) + 1e-5)
    a = a.astype(np.float32)
    for b in range(B):
        v[b, lengths[b]:] = 0.0
        a[b, lengths[b]:] = 0.0
    Lmax = max(len(l) for l in labels)
    lab = np.full((B, Lmax), -1, dtype=np.int64)
    for b, l in enumerate(labels):
        lab[b, :len(l)] = l
    return {
        "videos": v[:, None],                       # (B, 1, T, 88, 88)
        "audios": np.ascontiguousarray(a.transpose(0, 2, 1)),  # (B, 104, T)
        "labels": lab,
        "video_lengths": lengths.copy(),
        "audio_lengths": lengths.copy(),
        "label_lengths": np.array([len(l) for l in labels], dtype=np.int64),
    }
