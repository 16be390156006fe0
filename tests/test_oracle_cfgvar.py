"""Pin the CPU oracle's restatement of three reference config options — modality_fuse='add',
transformer_length_normalized_loss=True, layerdrop > 0 — to the reference's own outputs
(tests/golden/make_golden_cfgvar.py -> avsr_cfgvar.npz). CPU only."""
import pytest
import torch

from oracle import avsr_oracle as O
from tests.oracle_util import (LDROP_SEED, cfgvar_oracle_cfg, cfgvar_state, golden_batch, load_cfgvar, load_golden,
                               rel)


@pytest.fixture(scope="module")
def gv():
    return load_cfgvar()


@pytest.fixture(scope="module")
def batch():
    return {k: torch.from_numpy(v) for k, v in golden_batch(load_golden()).items()}


def test_modality_fuse_add_eval(gv, batch):
    sd = O.to_torch_state(cfgvar_state(gv, "add"))
    assert not any("post_extract_proj" in k for k in sd)
    with torch.no_grad():
        x = O.encoder_forward(sd, cfgvar_oracle_cfg("add"), batch["audios"], batch["videos"], None, False)
    assert rel(x, gv["add_enc_eval"]) < 1e-4


@pytest.mark.parametrize("name", ["add", "lnorm", "ldrop"])
def test_train_step(gv, batch, name):
    torch.set_num_threads(8)
    sd = O.to_torch_state(cfgvar_state(gv, name), requires_grad=True)
    if name == "ldrop":
        torch.manual_seed(LDROP_SEED)
    loss, lc, la, acc, ex = O.e2e_forward(sd, cfgvar_oracle_cfg(name), batch["videos"], batch["audios"],
                                          batch["video_lengths"], batch["labels"], True)
    loss.backward()
    ref = gv[f"{name}_loss"]
    for got, want in zip((loss.item(), lc.item(), la.item()), ref[:3]):
        assert abs(got - want) <= 1e-5 * abs(want), (name, got, want)
    assert rel(ex["enc"].detach(), gv[f"{name}_enc_train"]) < 1e-4
    keys = [k for k, t in sd.items() if t.grad is not None]
    assert sorted(keys) == sorted(gv[f"{name}_grad_keys"].tolist())        # skipped layer: no gradient
    for k, n in zip(gv[f"{name}_grad_keys"], gv[f"{name}_grad_norm"]):
        assert abs(sd[k].grad.double().norm().item() - n) <= 1e-4 * abs(n) + 1e-9, (name, k)
    if name == "ldrop":
        assert not any(".layers.1." in k for k in keys) and any(".layers.0." in k for k in keys)
