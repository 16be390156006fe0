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


class ParamGate:
    """Readiness events of an overlapped optimizer step. The update runs on its own stream in
    chunks that follow the arena's (module = forward) order; `marks` holds (end offset, event)
    per chunk, `zeroed` the event after the gradient arena was cleared behind the update.
    A reader of parameters [.., end) waits for the first chunk reaching `end` (wait), the
    backward for the cleared gradients (wait_grads); events are recorded on one stream, so
    waiting on one implies every earlier chunk."""

    def __init__(self, device):
        self.stream = torch.cuda.Stream(device=device)     # default priority: below the step stream
        self.marks = []
        self.zeroed = None
        self.final = None

    def wait(self, end):
        """current stream waits until every parameter below arena offset `end` is updated"""
        if not self.marks:
            return
        cur = torch.cuda.current_stream(self.stream.device)
        for i, (off, ev) in enumerate(self.marks):
            if off >= end:
                cur.wait_event(ev)
                del self.marks[:i + 1]
                return
        self.wait_params()

    def wait_params(self):
        if self.marks:
            torch.cuda.current_stream(self.stream.device).wait_event(self.marks[-1][1])
            self.marks = []

    def wait_grads(self):
        if self.zeroed is not None:
            torch.cuda.current_stream(self.stream.device).wait_event(self.zeroed)
            self.zeroed = None

    def wait_all(self):
        """everything the overlapped step wrote (parameters, moments, cleared gradients)"""
        if self.final is not None:
            torch.cuda.current_stream(self.stream.device).wait_event(self.final)
        self.marks, self.zeroed, self.final = [], None, None


class FusedAdamW:
    """overlap=True (with stage_bounds = sorted arena offsets inside the weight-decay segment,
    Engine.param_stage_bounds()): step() computes the gradient norm on the current stream, then
    runs the update on a side stream — no-decay segment first, then the decay segment chunk by
    chunk in forward order — and clears the gradients there (step(zero_grad=True)); the next
    forward waits per stage only for the chunk it reads (Engine.encoder_fwd), so the update of
    the later layers runs beside the frontends' forward. Results are bit-identical to the
    serial step (the update is elementwise). Readers outside Engine.forward call sync()."""

    def __init__(self, arena, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.005, max_grad_norm=1.0,
                 schedule=None, overlap=False, stage_bounds=()):
        self.arena = arena
        arena.init_optimizer()
        self.lr, self.betas, self.eps, self.wd, self.max_norm = lr, betas, eps, weight_decay, max_grad_norm
        self.schedule = schedule
        self.step_count = 0
        self._sumsq = torch.zeros(1, device=arena.device)
        self._sumsq_ws = torch.empty(ops.SUMSQ_WS, device=arena.device)
        self.gate = None
        if overlap:
            d0, d1 = arena.segments["decay"]
            self._bounds = sorted({b for b in stage_bounds if d0 < b < d1} | {d1})
            self.gate = ParamGate(arena.device)
            self._events = [torch.cuda.Event() for _ in range(len(self._bounds) + 2)]

    def sync(self):
        """make the current stream wait for an overlapped step's writes"""
        if self.gate is not None:
            self.gate.wait_all()

    def grad_sumsq(self):
        """sum of squared gradients over the trainable segments (device scalar, no sync)"""
        a = self.arena
        d0, _ = a.segments["decay"]
        _, n1 = a.segments["no_decay"]
        self._sumsq.zero_()
        ops.sumsq(a.grad[d0:n1], self._sumsq, self._sumsq_ws)
        return self._sumsq

    def step(self, grad_scale=1.0, sumsq_ready=False, zero_grad=False):
        """one AdamW step; with max_grad_norm > 0 the gradients are clipped by the global norm
        inside the kernel (coef = min(1, max_norm / (norm + 1e-6)), torch.nn.utils.
        clip_grad_norm_); sumsq_ready: grad_sumsq() was already computed for this step;
        zero_grad: clear the gradient arena after the update (on the update's stream when
        overlapped: no separate zero_grad() before the next backward)."""
        a = self.arena
        self.step_count += 1
        lr = self.schedule(self.step_count) if self.schedule else self.lr
        d0, d1 = a.segments["decay"]
        n0, n1 = a.segments["no_decay"]
        if self.gate is not None:
            self.gate.wait_all()                  # a previous overlapped step (no forward between)
        if self.max_norm and self.max_norm > 0 and not sumsq_ready:
            self.grad_sumsq()

        def launch(s, e, wd):
            ops.adamw(a.data[s:e], a.grad[s:e], a.exp_avg[s:e], a.exp_avg_sq[s:e], lr=lr, beta1=self.betas[0],
                      beta2=self.betas[1], eps=self.eps, weight_decay=wd, step=self.step_count,
                      shadow=None if a.shadow is None else a.shadow[s:e],
                      sumsq_buf=self._sumsq if self.max_norm else None, max_norm=self.max_norm or 1.0,
                      grad_scale=grad_scale)

        if self.gate is None:
            for (s, e), wd in (((d0, d1), self.wd), ((n0, n1), 0.0)):
                if e > s:
                    launch(s, e, wd)
            if zero_grad:
                a.zero_grad()
            return lr
        g, ev = self.gate, self._events
        g.stream.wait_stream(torch.cuda.current_stream(a.device))
        marks = []
        with torch.cuda.stream(g.stream):
            if n1 > n0:
                launch(n0, n1, 0.0)               # biases / LayerNorm weights: every stage reads some
            s = d0
            for i, e in enumerate(self._bounds):
                if e > s:
                    launch(s, e, self.wd)
                ev[i].record(g.stream)
                marks.append((e, ev[i]))
                s = e
            if zero_grad:
                a.grad.zero_()
            ev[-1].record(g.stream)
        g.marks = marks
        g.zeroed = ev[-1] if zero_grad else None
        g.final = ev[-1]
        a.gate = g
        if zero_grad:
            a.attach_grads(zero=False)
        return lr

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self):
        """optimizer state for resume (script/train.py:280-287,310-314): step count and the
        arena-layout moments (tensors only: loadable with torch.load(weights_only=True))."""
        a = self.arena
        return {"step": self.step_count, "exp_avg": a.exp_avg.detach().clone(),
                "exp_avg_sq": a.exp_avg_sq.detach().clone(),
                "hyper": {"lr": self.lr, "betas": list(self.betas), "eps": self.eps, "weight_decay": self.wd,
                          "max_grad_norm": self.max_norm}}

    def load_state_dict(self, sd):
        a = self.arena
        if sd["exp_avg"].numel() != a.exp_avg.numel():
            raise ValueError("optimizer state was saved for a different parameter arena")
        a.exp_avg.copy_(sd["exp_avg"])
        a.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])


class ArenaAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics over the parameter arena, for per-parameter training loops
    (HF Trainer, avsr_amd.trainer.AVSRTrainer): one fused launch per weight-decay segment.
    param_groups[0] carries lr / betas / eps / weight_decay (HF's LR scheduler writes lr);
    the state dict has torch's layout (state[0] = step, exp_avg, exp_avg_sq), so Trainer
    checkpoints save and resume it unchanged. `clip_grad_norm_` computes the global norm and
    folds the clip coefficient into the next step (no extra pass over the gradients)."""

    def __init__(self, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
        super().__init__([arena.data], dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.arena = arena
        self.fused = FusedAdamW(arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, max_grad_norm=0.0)
        self._clip = 0.0
        self.state[arena.data] = {"step": torch.zeros((), dtype=torch.float32),
                                  "exp_avg": arena.exp_avg, "exp_avg_sq": arena.exp_avg_sq}

    def grad_norm(self):
        return self.fused.grad_sumsq().sqrt()

    def clip_grad_norm_(self, max_norm):
        """returns the pre-clip global gradient norm; the next step() applies the clip"""
        norm = self.fused.grad_sumsq().sqrt()
        self._clip = float(max_norm)
        return norm

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        f = self.fused
        f.lr, f.betas, f.eps, f.wd = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
        f.max_norm = self._clip
        f.step(sumsq_ready=self._clip > 0)
        self._clip = 0.0
        st = self.state[self.arena.data]
        st["step"] = torch.tensor(float(f.step_count))
        return loss

    def zero_grad(self, set_to_none=True):
        self.arena.zero_grad()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        a = self.arena
        st = self.state[a.data]
        a.exp_avg.copy_(st["exp_avg"])
        a.exp_avg_sq.copy_(st["exp_avg_sq"])
        self.fused.step_count = int(float(st["step"]))
        self.state[a.data] = {"step": st["step"], "exp_avg": a.exp_avg, "exp_avg_sq": a.exp_avg_sq}
