"""avsr_amd.trainer.AVSRTrainer (drop-in for src/custom_trainer.py as script/train.py drives it)
on the tiny model, fp32 parity mode, one GPU:

  * gradient accumulation 2 (the reference's default, script/train.py:177): the gradients the
    optimizer sees equal the mean of the two micro-batches' gradients computed directly on the
    engine (HF divides each micro-step loss by 2);
  * the optimizer step equals torch.optim.AdamW (weight decay on all but biases / LayerNorm,
    clip_grad_norm_(1.0)) applied to the same gradients;
  * checkpoint + resume (script/train.py:280-287,310-314): training 2 steps straight equals
    training 1 step, saving, and resuming from the checkpoint for the second (model weights,
    AdamW moments, LR schedule and RNG state restored)."""
import numpy as np
import pytest
import torch
from torch.utils.data import SequentialSampler
from transformers import TrainerCallback, TrainingArguments

from avsr_amd.avhubert_avsr_model import AVHubertAVSR
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from avsr_amd.trainer import AVSRTrainer
from oracle.weights import NO_DROPOUT, TINY_CONFIG
from tests.oracle_util import golden_batch, golden_state, load_golden

pytestmark = pytest.mark.gpu

LABELS2 = [[12, 5, 9, 40], [77, 301, 17]]


def _samples(g):
    """4 samples (2 micro-batches of 2): the golden batch, then the same clips with other labels"""
    b = golden_batch(g)
    out = []
    for labels in (None, LABELS2):
        for i in range(2):
            lab = b["labels"][i][b["labels"][i] != -1] if labels is None else np.array(labels[i])
            out.append({"videos": b["videos"][i], "audios": b["audios"][i], "labels": lab,
                        "video_lengths": b["video_lengths"][i], "audio_lengths": b["audio_lengths"][i]})
    return out


def collate(samples):
    L = max(len(s["labels"]) for s in samples)
    lab = torch.full((len(samples), L), -1, dtype=torch.int64)
    for i, s in enumerate(samples):
        lab[i, :len(s["labels"])] = torch.as_tensor(s["labels"])
    return {"videos": torch.from_numpy(np.stack([s["videos"] for s in samples])),
            "audios": torch.from_numpy(np.stack([s["audios"] for s in samples])),
            "labels": lab,
            "video_lengths": torch.tensor([int(s["video_lengths"]) for s in samples]),
            "audio_lengths": torch.tensor([int(s["audio_lengths"]) for s in samples]),
            "label_lengths": torch.tensor([len(s["labels"]) for s in samples])}


class SeqTrainer(AVSRTrainer):
    def _get_train_sampler(self, *a, **k):
        return SequentialSampler(self.train_dataset)


class StopAfter(TrainerCallback):
    def __init__(self, n):
        self.n = n

    def on_step_end(self, args, state, control, **kw):
        if state.global_step >= self.n:
            control.should_save = True
            control.should_training_stop = True
        return control


class Capture(TrainerCallback):
    def __init__(self, model):
        self.model, self.grads, self.before, self.after, self.lrs = model, [], [], [], []

    def on_pre_optimizer_step(self, args, state, control, **kw):
        a = self.model.avsr.engine().arena
        self.grads.append(a.grad.clone())
        self.before.append(a.data.clone())
        opt = kw.get("optimizer")
        if opt is not None:
            inner = getattr(opt, "optimizer", opt)
            self.lrs.append((float(inner.param_groups[0]["lr"]), int(inner.fused.step_count)))

    def on_optimizer_step(self, args, state, control, **kw):
        self.after.append(self.model.avsr.engine().arena.data.clone())


def _model(g):
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
    return m


def _args(out, steps, **kw):
    a = dict(output_dir=str(out), per_device_train_batch_size=2, gradient_accumulation_steps=2, max_steps=steps,
             learning_rate=1e-3, weight_decay=0.005, warmup_steps=0, max_grad_norm=1.0, report_to="none",
             remove_unused_columns=False, dataloader_num_workers=0, logging_steps=1, seed=0, save_strategy="no",
             dataloader_drop_last=True)
    a.update(kw)
    return TrainingArguments(**a)


@pytest.fixture(scope="module")
def g():
    return load_golden()


def test_trainer_ga_and_adamw_step(g, tmp_path):
    m = _model(g)
    ds = _samples(g)
    cap = Capture(m)
    tr = SeqTrainer(model=m, args=_args(tmp_path, 1), data_collator=collate, valid_data_collator=collate,
                    train_dataset=ds, callbacks=[cap])
    tr.train()
    assert len(cap.grads) == 1
    # the micro-batches' gradients computed directly on a second engine
    ref = _model(g)
    ref.setup_engine("cuda", torch.float32)
    ref.train()
    ref.zero_grad()
    for mb in (collate(ds[0:2]), collate(ds[2:4])):
        (ref(**{k: v.cuda() for k, v in mb.items()}).loss / 2).backward()
    want = ref.avsr.engine().arena.grad
    err = (cap.grads[0] - want).abs().max().item() / want.abs().max().item()
    assert err < 1e-5, err
    # the step == torch.optim.AdamW on the same gradients (clip by the global norm first)
    arena = m.avsr.engine().arena
    d0, d1 = arena.segments["decay"]
    n0, n1 = arena.segments["no_decay"]
    p = cap.before[0].clone()
    gr = cap.grads[0].clone()
    norm = gr[d0:n1].double().norm().item()
    gr *= min(1.0, 1.0 / (norm + 1e-6))
    pd = torch.nn.Parameter(p[d0:d1].clone())
    pn = torch.nn.Parameter(p[n0:n1].clone())
    pd.grad, pn.grad = gr[d0:d1].clone(), gr[n0:n1].clone()
    opt = torch.optim.AdamW([{"params": [pd], "weight_decay": 0.005}, {"params": [pn], "weight_decay": 0.0}],
                            lr=1e-3, betas=(0.9, 0.999), eps=1e-8, foreach=False)
    opt.step()
    got = cap.after[0]
    assert (got[d0:d1] - pd.detach()).abs().max().item() < 2e-6
    assert (got[n0:n1] - pn.detach()).abs().max().item() < 2e-6
    assert torch.equal(got[n1:], p[n1:])            # frozen segment untouched
    assert tr.state.log_history and "grad_norm" in tr.state.log_history[0]
    assert abs(float(tr.state.log_history[0]["grad_norm"]) - norm) <= 1e-4 * norm


def test_trainer_checkpoint_resume(g, tmp_path):
    ds = _samples(g) * 2                  # 2 optimizer steps of GA 2 x batch 2
    m1 = _model(g)
    cap1 = Capture(m1)
    SeqTrainer(model=m1, args=_args(tmp_path / "a", 2), data_collator=collate, train_dataset=ds,
               callbacks=[cap1]).train()
    m2 = _model(g)
    # the same 2-step schedule, stopped after step 1 with its checkpoint saved (a max_steps=1 run
    # would checkpoint the LR of a 1-step schedule, 0, and the resumed step would use it)
    SeqTrainer(model=m2, args=_args(tmp_path / "b", 2, save_strategy="steps", save_steps=1), data_collator=collate,
               train_dataset=ds, callbacks=[StopAfter(1)]).train()
    m3 = _model(g)
    cap3 = Capture(m3)
    tr3 = SeqTrainer(model=m3, args=_args(tmp_path / "b", 2, save_strategy="no"), data_collator=collate,
                     train_dataset=ds, callbacks=[cap3])
    tr3.train(resume_from_checkpoint=str(tmp_path / "b" / "checkpoint-1"))
    assert len(cap3.grads) == 1                     # only the second step ran after resuming
    # every reduction of the training step has a fixed order (split-K slabs reduced in split
    # order, deterministic embedding backward and gradient norm; no fp32 atomics), so the
    # resumed run reproduces the straight run bit for bit
    e_w = (cap3.before[0] - cap1.before[1]).abs().max().item()
    assert e_w == 0.0, e_w                          # weights restored exactly
    e_g = (cap3.grads[0] - cap1.grads[1]).abs().max().item() / cap1.grads[1].abs().max().item()
    assert e_g == 0.0, (e_g, e_w)
    a1, a3 = m1.avsr.engine().arena, m3.avsr.engine().arena
    assert torch.equal(a1.exp_avg, a3.exp_avg) and torch.equal(a1.exp_avg_sq, a3.exp_avg_sq)   # AdamW moments
    assert cap3.lrs[-1] == cap1.lrs[-1], (cap1.lrs, cap3.lrs)    # same LR and AdamW step count
    assert torch.equal(a1.data, a3.data)                            # so the same update, bit for bit
    assert tr3.state.global_step == 2
