"""Flat parameter arena: every parameter of the model lives in ONE fp32 device buffer, its
gradient in a second, the AdamW moments in two more, and (bf16 mode) a bf16 shadow copy
that the GEMM / conv kernels read. This is the MI355X-native replacement for per-tensor
parameters + DDP buckets: one cast/AdamW/clip launch per step and contiguous gradient
slices for the RCCL bucketed all-reduce (avsr_amd/parallel.py).

Layout rules (chosen for the kernels, invisible to state_dict users):
  * conv weights are stored channels-last ([cout][kh][kw][cin]); the nn.Parameter is a
    permuted view, so `state_dict()` / `load_state_dict()` keep the reference shapes.
  * the pos-conv weight-norm direction v (D, D/G, K) is stored [D][K][D/G] (the conv
    kernel's weight layout), again exposed as a permuted view.
  * q/k/v projections of each attention block are adjacent (one fused QKV GEMM), the
    decoder source-attention k/v likewise (one fused KV GEMM over the encoder memory).
  * the two 5049-row output projections are padded to 5056 zero rows (K-aligned GEMMs).
  * segments: [weight-decayed | not decayed (biases, LayerNorm weights) | frozen (unused:
    mask_emb, label_embs_concat — they get no gradient in the reference)].
"""
import torch
from torch import nn

from . import ops

ALIGN = 64


def _round(n, a=ALIGN):
    return (n + a - 1) // a * a


class Arena:
    def __init__(self, root: nn.Module, device, compute_dtype=torch.bfloat16, fuse_groups=(), pad_rows=None,
                 perms=None, frozen=(), no_decay=None):
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        pad_rows = pad_rows or {}
        perms = perms or {}
        named = list(root.named_parameters())
        owners = {}
        for mname, mod in root.named_modules():
            for pname, p in mod._parameters.items():
                if p is not None:
                    owners[(mname + "." if mname else "") + pname] = (mod, pname)
        names = [n for n, _ in named]
        params = dict(named)
        if no_decay is None:
            ln_names = set()
            for mname, mod in root.named_modules():
                if isinstance(mod, nn.LayerNorm):
                    ln_names.add(mname + ".weight")
            no_decay = lambda n: n.endswith("bias") or n in ln_names  # noqa: E731
        frozen = set(frozen)
        group_of = {}
        for gi, grp in enumerate(fuse_groups):
            for n in grp:
                group_of[n] = gi
        # order: segment, then fused groups kept adjacent in their given order
        segs = {0: [], 1: [], 2: []}
        placed = set()
        for n in names:
            if n in placed:
                continue
            members = list(fuse_groups[group_of[n]]) if n in group_of else [n]
            seg = 2 if n in frozen else (1 if no_decay(n) else 0)
            for m in members:
                segs[seg].append(m)
                placed.add(m)
        self.order = segs[0] + segs[1] + segs[2]
        # offsets
        self.meta = {}
        off = 0
        seg_bounds = []
        for s in (0, 1, 2):
            start = off
            for n in segs[s]:
                p = params[n]
                shape = tuple(p.shape)
                perm = perms.get(n)
                phys = tuple(shape[i] for i in perm) if perm else shape
                rows = pad_rows.get(n, phys[0] if phys else 1)
                phys_alloc = (rows,) + phys[1:] if phys else ()
                numel = 1
                for d in phys_alloc:
                    numel *= d
                if n in group_of and numel % ALIGN:
                    raise ValueError(f"fused member {n} size {numel} not a multiple of {ALIGN}")
                off = off if (n in group_of and self._prev_in_group(n, fuse_groups, group_of)) else _round(off)
                self.meta[n] = dict(off=off, shape=shape, phys=phys, phys_alloc=phys_alloc, perm=perm, numel=numel)
                off += numel
            off = _round(off)
            seg_bounds.append((start, off))
        self.total = off
        self.segments = {"decay": seg_bounds[0], "no_decay": seg_bounds[1], "frozen": seg_bounds[2]}
        dev = self.device
        self.data = torch.zeros(self.total, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(self.total, device=dev, dtype=torch.float32)
        self.exp_avg = None
        self.exp_avg_sq = None
        self.shadow = torch.zeros(self.total, device=dev, dtype=compute_dtype) if compute_dtype != torch.float32 else None
        # re-home parameters; .grad of each trainable parameter is a view of the gradient arena
        # (the frozen ones — mask_emb, label_embs_concat — get no gradient, as in the reference)
        self.params = {}
        self._frozen = frozen
        for n in self.order:
            m = self.meta[n]
            old = params[n]
            view = self._logical(self.data, m)
            view.copy_(old.detach().to(dev))
            newp = nn.Parameter(view, requires_grad=old.requires_grad)
            mod, attr = owners[n]
            mod._parameters[attr] = newp
            self.params[n] = newp
        self.grad_views = {n: self._logical(self.grad, self.meta[n]) for n in self.order if n not in frozen}
        # LayerDrop (engine): per encoder layer its arena ranges, and the layers a backward has
        # touched since the last gradient clear (the others have no gradient: the optimizer skips
        # them as torch.optim.AdamW skips parameters whose grad is None)
        self.ld_ranges = None
        self.ld_touched = set()
        self.update_event = None     # an overlapped optimizer update in flight (wait_update)
        self.grads_cleared = False   # that update also zeroed the gradients (Engine.zero_grad_async)
        self.attach_grads(zero=False)
        self.sync_shadow()

    @staticmethod
    def _prev_in_group(n, groups, group_of):
        g = groups[group_of[n]]
        return g.index(n) > 0

    def _phys(self, buf, m):
        v = buf[m["off"]:m["off"] + m["numel"]].view(m["phys_alloc"]) if m["phys_alloc"] else buf[m["off"]:m["off"] + 1].view(())
        if m["phys_alloc"] and m["phys_alloc"][0] != m["phys"][0]:
            v = v[:m["phys"][0]]
        return v

    def _logical(self, buf, m):
        v = self._phys(buf, m)
        if m["perm"]:
            inv = [0] * len(m["perm"])
            for i, p in enumerate(m["perm"]):
                inv[p] = i
            v = v.permute(*inv)
        return v

    # ------------------------------------------------------------------ accessors
    def _cbuf(self):
        return self.shadow if self.shadow is not None else self.data

    def _view(self, kind, buf, name, make):
        """per-(buffer, parameter) view cache: the arena buffers are allocated once, so a view
        stays valid; building it anew on every launch costs the step a few ms of host time"""
        key = (kind, id(buf), name)
        v = self._vc.get(key) if hasattr(self, "_vc") else None
        if v is None:
            if not hasattr(self, "_vc"):
                self._vc = {}
            v = self._vc[key] = make()
        return v

    def w(self, name):
        """compute-dtype weight in PHYSICAL layout (e.g. conv: [cout][kh][kw][cin])."""
        buf = self._cbuf()
        return self._view("w", buf, name, lambda: self._phys(buf, self.meta[name]))

    def w_padded(self, name):
        m = self.meta[name]
        return self._cbuf()[m["off"]:m["off"] + m["numel"]].view(m["phys_alloc"])

    def master(self, name):
        return self._view("m", self.data, name, lambda: self._phys(self.data, self.meta[name]))

    def g(self, name):
        """fp32 gradient accumulator in PHYSICAL layout."""
        return self._view("g", self.grad, name, lambda: self._phys(self.grad, self.meta[name]))

    def g_padded(self, name):
        m = self.meta[name]
        return self.grad[m["off"]:m["off"] + m["numel"]].view(m["phys_alloc"])

    def span(self, names, buf="w"):
        """view over adjacent (fused) parameters: 1-D for vectors, [sum rows][cols] for matrices."""
        ms = [self.meta[n] for n in names]
        for a, b in zip(ms, ms[1:]):
            assert b["off"] == a["off"] + a["numel"], f"{names} not adjacent"
        base = {"w": self._cbuf(), "g": self.grad, "master": self.data}[buf]
        total = sum(m["numel"] for m in ms)
        flat = base[ms[0]["off"]:ms[0]["off"] + total]
        if len(ms[0]["phys_alloc"]) <= 1:
            return flat
        return flat.view(-1, ms[0]["numel"] // ms[0]["phys_alloc"][0])

    # ------------------------------------------------------------------ maintenance
    def sync_shadow(self):
        """refresh the compute-dtype shadow from the fp32 master (after loading weights or an
        update by a per-parameter optimizer). One flat vectorised cast launch."""
        if self.shadow is not None:
            if self.device.type == "cpu":          # layout tests only (no kernels run on CPU)
                self.shadow.copy_(self.data)
            else:
                ops.cast_flat(self.data, self.shadow)
        self._synced_version = self.data._version

    def ensure_shadow(self):
        """in-place writes through the parameter views (torch.optim steps, load_state_dict,
        param.data.copy_) bump the arena's version counter: refresh the shadow if any happened
        since the last sync. The fused optimizer writes master + shadow in one kernel."""
        if self.data._version != self._synced_version:
            self.sync_shadow()

    def attach_grads(self, zero=True):
        """(re)attach the gradient-arena views as .grad. A per-parameter optimizer's
        zero_grad(set_to_none=True) (HF Trainer, torch.optim) sets .grad to None: those
        parameters' gradients restart from zero, so their arena slices are cleared first (one
        memset when every parameter was reset)."""
        missing = [n for n, v in self.grad_views.items() if self.params[n].grad is not v]
        if not missing:
            return
        if zero:
            if len(missing) == len(self.grad_views):
                self.grad.zero_()
            else:
                for n in missing:
                    if self.params[n].grad is None:
                        self.grad_views[n].zero_()
        for n in missing:
            self.params[n].grad = self.grad_views[n]

    def wait_update(self, stream=None):
        """make `stream` (default: the current stream) wait for an overlapped optimizer update
        still running on its own stream (FusedAdamW(overlap=True)); no-op otherwise. The event
        stays set: every reader of parameters, moments or gradients may wait on it."""
        ev = self.update_event
        if ev is not None:
            (stream or torch.cuda.current_stream(self.device)).wait_event(ev)

    def zero_grad(self):
        self.wait_update()
        self.grad.zero_()
        self.attach_grads(zero=False)
        self.ld_touched.clear()

    def ranges_of(self, prefix):
        """merged [start, end) arena ranges of the parameters whose names start with prefix"""
        out = []
        for s, e in sorted((m["off"], m["off"] + m["numel"]) for n, m in self.meta.items() if n.startswith(prefix)):
            if out and s <= out[-1][1]:
                out[-1] = (out[-1][0], max(out[-1][1], e))
            else:
                out.append((s, e))
        return out

    def init_optimizer(self):
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(self.data)
            self.exp_avg_sq = torch.zeros_like(self.data)
