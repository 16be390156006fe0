"""Utterance-level data parallelism: one process per GPU, RCCL over xGMI.

Replaces the DDP reducer that HF Trainer / accelerate wrap around the reference
(script/train.py:259-308, src/custom_trainer.py:4-41): gradients live in ONE flat fp32 arena
buffer, so the all-reduce is a handful of large contiguous buckets (no per-parameter copy
into bucket storage) issued on a dedicated communication stream. Gradients are averaged
(sum / world), like DDP.

`ArenaDDP` reproduces the DistributedDataParallel semantics the reference trains under
(HF Trainer -> accelerate -> DDP, broadcast_buffers=True):
  * at construction: parameters and buffers broadcast from rank 0;
  * before a training forward: the BatchNorm running statistics are broadcast from rank 0
    (one collective over the engine's flat statistics buffer) when the previous forward was a
    synchronising one — DDP's require_forward_param_sync rule;
  * backward: buckets all-reduced as soon as their layers' gradients are final, overlapped
    with the rest of the backward on a communication stream; under `no_sync()` (non-final
    gradient-accumulation micro-steps) nothing is exchanged and gradients accumulate locally.
"""
import contextlib
import os

import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20   # 64 MiB buckets: ~7 links x ~153 GB/s per GPU want big messages
COMPRESS_MODES = (None, "bf16")


def _cast(src, dst):
    """flat dtype cast for the compressed exchange: the library's HIP kernel for device
    tensors; CPU tensors exist only in the gloo-on-CPU tests of this module's logic"""
    if src.is_cuda:
        from . import ops
        ops.cast_flat(src, dst)
    else:
        dst.copy_(src)


def init_from_env(backend=None):
    """torchrun / torch.distributed.run environment -> (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            # RCCL's internal streams at high priority: the step runs on a high-priority stream
            # (engine.prioritize_step_stream) and the gradient exchange must not queue behind it
            os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


class GradReducer:
    """Bucketed all-reduce (sum) of the flat fp32 gradient arena on a dedicated stream,
    overlapped with the backward pass.

    Buckets tile the weight-decay segment from its END backwards (64 MiB each), then the
    small no-decay / frozen tail. The engine reports readiness with `ready(offset)`: the
    decay segment is final from `offset` on (encoder layer i done => layers >= i, decoder
    and CTC head final). Every newly complete bucket is all-reduced right away on the comm
    stream, which first waits on an event of the compute stream; `finish()` reduces the
    rest and makes the compute stream wait for the comm stream. `allreduce()` = begin +
    finish (no overlap).

    compress="bf16" (off by default: fp32 keeps gradient parity with the reference's DDP)
    halves the bytes on xGMI: a bucket is cast to bf16 on the comm stream, summed in bf16 by
    RCCL and cast back into the fp32 arena (torch DDP's bf16_compress_hook, minus its
    pre-division: the 1/world factor stays in the optimizer or finish(average=True))."""

    def __init__(self, flat_grad, bucket_bytes=BUCKET_BYTES, group=None, use_stream=True, segment=None,
                 compress=None):
        if compress not in COMPRESS_MODES:
            raise ValueError(f"compress={compress!r}: one of {COMPRESS_MODES}")
        self.flat = flat_grad
        self.compress = compress
        self.cbuf = None
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        n = flat_grad.numel()
        step = max(1, bucket_bytes // flat_grad.element_size())
        d0, d1 = segment if segment is not None else (0, n)
        self.seg = (d0, d1)
        self.buckets = []                       # decay segment, last bucket first
        e = d1
        while e > d0:
            s = max(d0, e - step)
            self.buckets.append((s, e))
            e = s
        self.tail = [(a, min(n, a + step)) for a in range(d1, n, step)]
        if d0 > 0:
            self.tail = [(a, min(d0, a + step)) for a in range(0, d0, step)] + self.tail
        # high priority like the step stream (engine.prioritize_step_stream): bucket all-reduces
        # start as soon as their gradients are ready instead of waiting behind the backward
        self.stream = (torch.cuda.Stream(device=flat_grad.device, priority=-1)
                       if (use_stream and flat_grad.is_cuda) else None)
        self._next = 0
        self._works = []
        self.enabled = True          # False inside ArenaDDP.no_sync(): gradients accumulate locally
        self.extra_streams = []      # other streams that produce gradients (the engine's side stream)
        # optional timing (bench.py): per reduced step, HIP events (comm start, comm end) on
        # the comm stream and (backward end, join) on the compute stream — join - backward
        # end is the all-reduce time the step could not hide
        self.timing = None           # list to enable
        self._t0 = None

    def _reduce(self, a, b):
        buf = self.flat
        if self.compress == "bf16":
            if self.cbuf is None:
                self.cbuf = torch.empty(self.flat.numel(), dtype=torch.bfloat16, device=self.flat.device)
            _cast(self.flat[a:b], self.cbuf[a:b])
            buf = self.cbuf
        w = dist.all_reduce(buf[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=self.stream is not None)
        if w is not None:
            self._works.append((w, a, b))
        elif buf is not self.flat:
            _cast(self.cbuf[a:b], self.flat[a:b])

    def _launch(self, ranges):
        if not ranges:
            return
        if self.stream is None:
            for a, b in ranges:
                self._reduce(a, b)
            return
        cur = torch.cuda.current_stream(self.flat.device)
        self.stream.wait_stream(cur)             # gradients of these ranges are complete
        for s in self.extra_streams:             # ... including those computed on side streams
            self.stream.wait_stream(s)
        with torch.cuda.stream(self.stream):
            if self.timing is not None and self._t0 is None:
                self._t0 = torch.cuda.Event(enable_timing=True)
                self._t0.record()
            for a, b in ranges:
                self._reduce(a, b)

    def begin(self):
        self._next = 0
        self._works = []
        self._t0 = None

    def ready(self, offset):
        """the decay segment is final from `offset` on: reduce every bucket inside it"""
        if self.world == 1 or not self.enabled:
            return
        todo = []
        while self._next < len(self.buckets) and self.buckets[self._next][0] >= offset:
            todo.append(self.buckets[self._next])
            self._next += 1
        self._launch(todo)

    def finish(self, average=False):
        if self.world == 1 or not self.enabled:
            return
        self._launch(self.buckets[self._next:] + self.tail)
        self._next = len(self.buckets)
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                for w, a, b in self._works:
                    w.wait()
                    if self.compress == "bf16":
                        _cast(self.cbuf[a:b], self.flat[a:b])
                if average:
                    self.flat.mul_(1.0 / self.world)
                if self.timing is not None:
                    t1 = torch.cuda.Event(enable_timing=True)
                    t1.record()
            cur = torch.cuda.current_stream(self.flat.device)
            if self.timing is not None:
                j0, j1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for s in self.extra_streams:      # the backward ends when its side streams do
                    cur.wait_stream(s)
                j0.record(cur)
            cur.wait_stream(self.stream)
            if self.timing is not None:
                j1.record(cur)
                self.timing.append((self._t0, t1, j0, j1))
        elif average:
            self.flat.mul_(1.0 / self.world)
        self._works = []

    def allreduce(self, average=True):
        """sum over ranks; average=False leaves the 1/world scale to the optimizer
        (FusedAdamW.step(grad_scale=1/world)) and saves a pass over the buffer."""
        self.begin()
        self.finish(average=average)


def broadcast_state(flat_params, buffers, src=0, group=None):
    """Make every rank start from rank 0's parameters and buffers (DDP construction)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.broadcast(flat_params, src=src, group=group)
    for b in buffers:
        dist.broadcast(b, src=src, group=group)


class ArenaDDP:
    """DistributedDataParallel semantics for an AVHubertAVSR on the HIP engine (see module
    docstring). Attach once per process after the engine exists:

        ddp = ArenaDDP(model)                   # broadcasts rank 0's state
        with ddp.no_sync():                     # GA micro-steps 1..n-1
            model(**mb).loss.backward()
        model(**mb_last).loss.backward()        # all-reduce overlapped with this backward

    average=True divides the summed gradients by the world size (DDP); average=False leaves
    the 1/world factor to FusedAdamW.step(grad_scale=1/world) and saves one pass."""

    def __init__(self, model, bucket_bytes=BUCKET_BYTES, broadcast_buffers=True, average=True, use_stream=True,
                 group=None, compress=None):
        eng = model.avsr.engine()
        self.model, self.eng, self.group = model, eng, group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        arena = eng.arena
        int_buffers = [b for b in model.buffers() if not b.is_floating_point()]
        broadcast_state(arena.data, [eng.bn_flat] + int_buffers, group=group)
        arena.sync_shadow()
        self.reducer = GradReducer(arena.grad, bucket_bytes=bucket_bytes, group=group, use_stream=use_stream,
                                   segment=arena.segments["decay"], compress=compress)
        if getattr(eng, "side", None) is not None:
            self.reducer.extra_streams.append(eng.side)
        self.average = average
        self.broadcast_buffers = broadcast_buffers
        self.require_backward_grad_sync = True
        self.require_forward_param_sync = True
        self.buffer_broadcasts = 0
        eng.before_forward = self._pre_forward
        eng.before_backward = self._pre_backward
        eng.on_grad_ready = self.reducer.ready
        eng.after_backward = self._post_backward
        model._ddp = self

    def _pre_forward(self):
        if self.world > 1 and self.broadcast_buffers and self.require_forward_param_sync:
            dist.broadcast(self.eng.bn_flat, src=0, group=self.group)
            self.buffer_broadcasts += 1
        # DDP _post_forward: the next forward syncs buffers iff this one synchronises grads
        self.require_forward_param_sync = self.require_backward_grad_sync

    def _pre_backward(self):
        self.reducer.enabled = self.require_backward_grad_sync
        self.reducer.begin()

    def _post_backward(self):
        self.reducer.finish(average=self.average)

    @contextlib.contextmanager
    def no_sync(self):
        """DDP.no_sync: backward passes inside accumulate gradients without communication"""
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    def detach(self):
        e = self.eng
        e.before_forward = e.before_backward = e.on_grad_ready = e.after_backward = None
        self.model._ddp = None
