"""Fused clip-grad-norm + AdamW over the flat arena, with the HF Trainer schedule used by
the reference (script/train.py:259-299: AdamW lr 1e-4, betas (0.9, 0.999), eps 1e-8,
weight_decay 0.005 on all but biases / LayerNorm weights, max_grad_norm 1.0, linear
warm-up then linear decay). One sumsq launch + one AdamW launch per segment, no host sync:
the clip coefficient is computed on the device from the gradient norm."""
import torch
import torch.distributed as dist

from . import ops


def union_touched(touched, n, device=None):
    """LayerDrop under data parallelism: the encoder layers some rank's backward touched. The
    all-reduce hands every rank the average gradient, so a layer kept on any rank has a gradient
    everywhere and every rank must update it (a per-rank skip would let the replicas drift). One
    MAX all-reduce of an n-flag vector and a host read (one sync per step, LayerDrop + DDP only);
    single process: the local set."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return set(touched)
    dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    m = torch.zeros(n, dtype=torch.int32, device=dev)
    if touched:
        m[list(touched)] = 1
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return set(torch.nonzero(m).flatten().tolist())


class LinearWarmupDecay:
    def __init__(self, lr, warmup_steps, total_steps):
        self.lr, self.warm, self.total = lr, warmup_steps, total_steps

    def __call__(self, step):       # step counts from 1 (HF get_linear_schedule_with_warmup)
        s = step - 1
        if s < self.warm:
            return self.lr * s / max(1, self.warm)
        return self.lr * max(0.0, (self.total - s) / max(1, self.total - self.warm))


class FusedAdamW:
    """step(): gradient norm, then one fused clip + AdamW launch per weight-decay segment, all
    on the current stream.

    overlap=True: the update of the parameters the next training forward reads first (the audio
    and video frontends: FRONT) runs on the current stream, the rest (encoder, decoder, CTC:
    ~97 % of the arena) on an update stream that waits for the current one, on a capped grid
    (overlap_blocks); each launch also zeroes the gradients it has read (the next step's
    gradient clear, arena.grads_cleared). The engine's next
    training forward runs the frontends (the ResNet forward, several ms of single-stream work)
    beside it and waits for the update (arena.update_event) before the first encoder parameter
    is read; the gradient clear waits for it too. The update is elementwise, so results equal the
    serial step bit for bit. Other readers of parameters, moments or gradients call sync() (or
    arena.wait_update()) first. (Round 3 measured no gain from a similar overlap while the host
    issued each step only just ahead of the GPU, profiles/r03_opt_overlap_ab.txt; the host now
    runs 80-110 ms ahead, profiles/r06_host_lead.txt.)"""

    FRONT = ("encoder.feature_extractor_audio.", "encoder.feature_extractor_video.")

    def __init__(self, arena, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.005, max_grad_norm=1.0,
                 schedule=None, overlap=False):
        self.arena = arena
        self.overlap = bool(overlap) and arena.device.type == "cuda"
        self._ustream = torch.cuda.Stream(device=arena.device) if self.overlap else None
        self._uevent = torch.cuda.Event() if self.overlap else None
        # grid cap of the overlapped launches: the update's grid-stride blocks live for the whole
        # launch, and at the default 4096 blocks (8 resident per CU) they hold every wave slot, so
        # the next forward's kernels (even its 5-us batch copy) wait for the update to finish
        self.overlap_blocks = 128
        self.clear_in_update = True      # overlapped launches zero the gradients they read
        arena.init_optimizer()
        self.lr, self.betas, self.eps, self.wd, self.max_norm = lr, betas, eps, weight_decay, max_grad_norm
        self.schedule = schedule
        self.step_count = 0
        self.layer_steps = None      # LayerDrop: per encoder layer, the steps that updated it
        self._sumsq = torch.zeros(1, device=arena.device)
        self._sumsq_ws = torch.empty(ops.SUMSQ_WS, device=arena.device)
        self._early = False
        # gradients the backward finalises last (the ResNet frontend, resnet.py): early_sumsq()
        # sums the others beforehand, grad_sumsq() then adds these
        d0, _ = arena.segments["decay"]
        _, n1 = arena.segments["no_decay"]
        late = [(max(s, d0), min(e, n1)) for s, e in arena.ranges_of("encoder.feature_extractor_video.resnet.")]
        self._late = [(s, e) for s, e in late if s < e]
        self._early_ranges, pos = [], d0
        for s, e in self._late:
            if pos < s:
                self._early_ranges.append((pos, s))
            pos = max(pos, e)
        if pos < n1:
            self._early_ranges.append((pos, n1))

    def early_sumsq(self):
        """sum of squares of every trainable gradient outside the ResNet frontend (current stream;
        the engine calls it on its side stream once those gradients are final — single process
        only: under DDP the norm must follow the all-reduce)"""
        a = self.arena
        self._sumsq.zero_()
        for s, e in self._early_ranges:
            ops.sumsq(a.grad[s:e], self._sumsq, self._sumsq_ws)
        self._early = True

    def grad_sumsq(self):
        """sum of squared gradients over the trainable segments (device scalar, no sync); after
        early_sumsq() only the ResNet frontend's ranges are left to add"""
        a = self.arena
        if self._early:
            self._early = False
            for s, e in self._late:
                ops.sumsq(a.grad[s:e], self._sumsq, self._sumsq_ws)
            return self._sumsq
        d0, _ = a.segments["decay"]
        _, n1 = a.segments["no_decay"]
        self._sumsq.zero_()
        ops.sumsq(a.grad[d0:n1], self._sumsq, self._sumsq_ws)
        return self._sumsq

    def step(self, grad_scale=1.0, sumsq_ready=False, zero_grad=False):
        """one AdamW step; with max_grad_norm > 0 the gradients are clipped by the global norm
        inside the kernel (coef = min(1, max_norm / (norm + 1e-6)), torch.nn.utils.
        clip_grad_norm_); sumsq_ready: grad_sumsq() was already computed for this step;
        zero_grad: clear the gradient arena after the update."""
        a = self.arena
        self.step_count += 1
        lr = self.schedule(self.step_count) if self.schedule else self.lr
        d0, d1 = a.segments["decay"]
        n0, n1 = a.segments["no_decay"]
        if self.max_norm and self.max_norm > 0 and not sumsq_ready:
            self.grad_sumsq()

        def launch(s, e, wd, step, max_blocks=0):
            ops.adamw(a.data[s:e], a.grad[s:e], a.exp_avg[s:e], a.exp_avg_sq[s:e], lr=lr, beta1=self.betas[0],
                      beta2=self.betas[1], eps=self.eps, weight_decay=wd, step=step,
                      shadow=None if a.shadow is None else a.shadow[s:e],
                      sumsq_buf=self._sumsq if self.max_norm else None, max_norm=self.max_norm or 1.0,
                      grad_scale=grad_scale, max_blocks=max_blocks, clear_grad=self.overlap and self.clear_in_update)

        if a.ld_ranges is not None:
            if self.layer_steps is None:
                self.layer_steps = [self.step_count - 1] * len(a.ld_ranges)
            self._touched = union_touched(a.ld_touched, len(a.ld_ranges), a.device)
            for i in self._touched:
                self.layer_steps[i] += 1
        if not self.overlap:
            for (s, e), wd in (((d0, d1), self.wd), ((n0, n1), 0.0)):
                for ps, pe, step in self._pieces(s, e):
                    if step is not None:
                        launch(ps, pe, wd, step)
        else:
            a.wait_update()          # a previous overlapped update with no forward in between
            front, rest = self._split()
            for s, e, wd in front:
                for ps, pe, step in self._pieces(s, e):
                    if step is not None:
                        launch(ps, pe, wd, step)
            us = self._ustream
            us.wait_stream(torch.cuda.current_stream(a.device))
            with torch.cuda.stream(us):
                for s, e, wd in rest:
                    for ps, pe, step in self._pieces(s, e):
                        if step is not None:
                            launch(ps, pe, wd, step, self.overlap_blocks)
                self._uevent.record(us)
            a.update_event = self._uevent
            # every gradient the update read is zero again (the ranges it skips — LayerDrop layers no
            # backward touched — were never written): the next gradient clear has nothing to do
            a.grads_cleared = self.clear_in_update
        self._early = False          # the early partial belongs to this step's gradients only
        if zero_grad:
            a.zero_grad()
        return lr

    def sync(self):
        """current stream waits for an overlapped update (parameters, moments, gradients read)"""
        self.arena.wait_update()

    def _split(self):
        """(front, rest): [start, end, weight decay] ranges of both segments, front = the FRONT
        modules' parameters (the next forward reads them before any other), rest = the others"""
        a = self.arena
        fr = sorted(r for p in self.FRONT for r in a.ranges_of(p))
        front, rest = [], []
        for (s, e), wd in ((a.segments["decay"], self.wd), (a.segments["no_decay"], 0.0)):
            pos = s
            for r0, r1 in fr:
                lo, hi = max(r0, s), min(r1, e)
                if lo >= hi:
                    continue
                if pos < lo:
                    rest.append((pos, lo, wd))
                front.append((lo, hi, wd))
                pos = hi
            if pos < e:
                rest.append((pos, e, wd))
        return front, rest

    def _pieces(self, s, e):
        """[s, e) as (start, end, step) launches: without LayerDrop one piece at the global step;
        with it, each encoder layer's ranges at that layer's own step count, or step None (no
        launch) for a layer no backward touched since the last gradient clear — torch.optim.AdamW
        skips a parameter whose grad is None (no decay, no moment update, its own step count)"""
        a = self.arena
        if a.ld_ranges is None or e <= s:
            return [(s, e, self.step_count)] if e > s else []
        cuts = []
        for i, rs in enumerate(a.ld_ranges):
            st = self.layer_steps[i] if i in self._touched else None
            for r0, r1 in rs:
                lo, hi = max(r0, s), min(r1, e)
                if lo < hi:
                    cuts.append((lo, hi, st))
        out, pos = [], s
        for lo, hi, st in sorted(cuts):
            if pos < lo:
                out.append((pos, lo, self.step_count))
            out.append((lo, hi, st))
            pos = hi
        if pos < e:
            out.append((pos, e, self.step_count))
        merged = []
        for p in out:
            if merged and merged[-1][2] == p[2] and merged[-1][1] == p[0]:
                merged[-1] = (merged[-1][0], p[1], p[2])
            else:
                merged.append(p)
        return merged

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self):
        """optimizer state for resume (script/train.py:280-287,310-314): step count and the
        arena-layout moments (tensors only: loadable with torch.load(weights_only=True))."""
        a = self.arena
        extra = {} if self.layer_steps is None else {"layer_steps": torch.tensor(self.layer_steps)}
        return {"step": self.step_count, **extra, "exp_avg": a.exp_avg.detach().clone(),
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
        if "layer_steps" in sd:
            self.layer_steps = [int(v) for v in sd["layer_steps"]]


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
        if f.layer_steps is not None:        # LayerDrop: each encoder layer's own AdamW step count
            st["layer_steps"] = torch.tensor(f.layer_steps, dtype=torch.float32)
        return loss

    def zero_grad(self, set_to_none=True):
        self.fused._early = False
        self.arena.zero_grad()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        a = self.arena
        st = self.state[a.data]
        a.exp_avg.copy_(st["exp_avg"])
        a.exp_avg_sq.copy_(st["exp_avg_sq"])
        self.fused.step_count = int(float(st["step"]))
        self.state[a.data] = {"step": st["step"], "exp_avg": a.exp_avg, "exp_avg_sq": a.exp_avg_sq}
        if "layer_steps" in st:             # torch casts saved state tensors to the parameter dtype
            ls = st["layer_steps"]
            self.fused.layer_steps = [int(round(float(v))) for v in ls.flatten().tolist()]
            self.state[a.data]["layer_steps"] = ls.detach().cpu().float()
        else:
            self.fused.layer_steps = None
