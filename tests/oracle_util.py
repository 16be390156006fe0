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


def rel(a, b):
    a = torch.as_tensor(np.asarray(a), dtype=torch.float64)
    b = torch.as_tensor(np.asarray(b), dtype=torch.float64)
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
