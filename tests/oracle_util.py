"""Helpers shared by the parity tests: golden fixture loading and oracle state building."""
import os

import numpy as np
import torch

from oracle import avsr_oracle as O
from oracle.weights import TINY_CONFIG, collate, gen_tensor

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "avsr_tiny.npz")


def load_golden():
    return dict(np.load(GOLDEN, allow_pickle=False))


def golden_state(g, seed=0):
    shapes = {k: tuple(int(x) for x in s.split(",") if x) for k, s in zip(g["param_keys"], g["param_shapes"])}
    return {k: gen_tensor(k, s, seed) for k, s in shapes.items()}


def golden_batch(g):
    labels = [row[row != -1].tolist() for row in g["labels"]]
    return collate(g["frames"], g["feats"], g["lengths"], labels)


def tiny_cfg():
    return O.OracleConfig.from_dict(TINY_CONFIG)


# ---------------------------------------------------------------------------- full size
GOLDEN_FULL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "avsr_full.npz")
TOKENS = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]


def load_golden_full():
    return dict(np.load(GOLDEN_FULL, allow_pickle=False))


def full_state(g, seed=0):
    return golden_state(g, seed)


def _digest(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def full_c1_batch(g):
    """C1 inputs of tests/golden/make_golden_full.py, regenerated from their seed and
    checked against the digest the generator stored."""
    from tests.golden.full_inputs import C1
    from oracle.weights import make_inputs
    frames, feats, lengths, _ = make_inputs(B=C1["B"], T=C1["T"], lengths=C1["lengths"], seed=C1["seed"])
    b = collate(frames, feats, lengths, [(1,)] * C1["B"])
    assert _digest(b["videos"], b["audios"]) == str(g["c1_digest"]), "C1 input regeneration drifted"
    return b


def full_train_batch(g):
    """the T=375 train-step batch of make_golden_full.py (B=2, second row padded to 300)."""
    from tests.golden.full_inputs import TR, TR_LABELS
    from oracle.weights import make_inputs
    frames, feats, lengths, _ = make_inputs(B=TR["B"], T=TR["T"], lengths=TR["lengths"], seed=TR["seed"])
    b = collate(frames, feats, lengths, TR_LABELS)
    assert _digest(b["videos"], b["audios"], b["labels"]) == str(g["tr_digest"]), "train input regeneration drifted"
    return b


def rel(a, b):
    a = torch.as_tensor(np.asarray(a), dtype=torch.float64)
    b = torch.as_tensor(np.asarray(b), dtype=torch.float64)
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def zero_grad_by_symmetry(key):
    """key-projection biases get a mathematically zero gradient (softmax over keys is invariant
    to adding q.b to every score): reference and engine both return round-off there, so their
    norms are compared against an absolute floor instead of relatively."""
    return key.endswith("k_proj.bias") or key.endswith("linear_k.bias")


GOLDEN_ENDBEAM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "avsr_endbeam.npz")


def load_golden_endbeam():
    return dict(np.load(GOLDEN_ENDBEAM, allow_pickle=False))


def endbeam_case(ge, off, beam, clip):
    """the reference's ended hypotheses (best first) of one early-ending search
    (tests/golden/make_golden_endbeam.py): list of (yseq, score, decoder score, ctc score)"""
    key = f"eb_{off:g}_b{beam}_{clip}"
    lens, flat = ge[key + "_len"], ge[key + "_yseq"]
    out, o = [], 0
    for i, n in enumerate(lens):
        out.append((flat[o:o + n].tolist(), float(ge[key + "_score"][i]), float(ge[key + "_dec"][i]),
                    float(ge[key + "_ctc"][i])))
        o += n
    return out


def endbeam_state(g, off):
    """recipe weights with the <eos> logit bias raised by `off` (make_golden_endbeam.py)"""
    st = full_state(g)
    st["avsr.decoder.output_layer.bias"] = st["avsr.decoder.output_layer.bias"].copy()
    st["avsr.decoder.output_layer.bias"][5048] += np.float32(off)
    return st


# ------------------------------------------------------------------ config-option variants
GOLDEN_CFGVAR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "avsr_cfgvar.npz")
# the reference config options of tests/golden/make_golden_cfgvar.py (tiny config, dropouts 0)
CFGVAR = {"add": dict(modality_fuse="add"), "lnorm": dict(transformer_length_normalized_loss=True),
          "ldrop": dict(layerdrop=0.5)}
LDROP_SEED = 1


def load_cfgvar():
    return dict(np.load(GOLDEN_CFGVAR, allow_pickle=False))


def cfgvar_state(gv, name, seed=0):
    shapes = {k: tuple(int(x) for x in s.split(",") if x)
              for k, s in zip(gv[f"{name}_param_keys"], gv[f"{name}_param_shapes"])}
    return {k: gen_tensor(k, s, seed) for k, s in shapes.items()}


def cfgvar_oracle_cfg(name):
    return O.OracleConfig.from_dict({**TINY_CONFIG, **CFGVAR[name]})
