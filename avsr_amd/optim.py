"""Fused clip-grad-norm + AdamW over the flat arena, with the HF Trainer schedule used by
the reference (script/train.py:259-299: AdamW lr 1e-4, betas (0.9, 0.999), eps 1e-8,
weight_decay 0.005 on all but biases / LayerNorm weights, max_grad_norm 1.0, linear
warm-up then linear decay). One sumsq launch + one AdamW launch per segment, no host sync:
the clip coefficient is computed on the device from the gradient norm."""
import torch

from . import ops


class LinearWarmupDecay:
    def __init__(self, lr, warmup_steps, total_steps):
        self.lr, self.warm, self.total = lr, warmup_steps, total_steps

    def __call__(self, step):       # step counts from 1 (HF get_linear_schedule_with_warmup)
        s = step - 1
        if s < self.warm:
            return self.lr * s / max(1, self.warm)
        return self.lr * max(0.0, (self.total - s) / max(1, self.total - self.warm))


class FusedAdamW:
    def __init__(self, arena, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.005, max_grad_norm=1.0,
                 schedule=None):
        self.arena = arena
        arena.init_optimizer()
        self.lr, self.betas, self.eps, self.wd, self.max_norm = lr, betas, eps, weight_decay, max_grad_norm
        self.schedule = schedule
        self.step_count = 0
        self._sumsq = torch.zeros(1, device=arena.device)

    def step(self, grad_scale=1.0):
        a = self.arena
        self.step_count += 1
        lr = self.schedule(self.step_count) if self.schedule else self.lr
        d0, d1 = a.segments["decay"]
        n0, n1 = a.segments["no_decay"]
        self._sumsq.zero_()
        if self.max_norm and self.max_norm > 0:
            ops.sumsq(a.grad[d0:n1], self._sumsq)
        for (s, e), wd in (((d0, d1), self.wd), ((n0, n1), 0.0)):
            if e <= s:
                continue
            ops.adamw(a.data[s:e], a.grad[s:e], a.exp_avg[s:e], a.exp_avg_sq[s:e], lr=lr, beta1=self.betas[0],
                      beta2=self.betas[1], eps=self.eps, weight_decay=wd, step=self.step_count,
                      shadow=None if a.shadow is None else a.shadow[s:e],
                      sumsq_buf=self._sumsq if self.max_norm else None, max_norm=self.max_norm or 1.0,
                      grad_scale=grad_scale)
        return lr
