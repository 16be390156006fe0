"""Utterance-level data parallelism: one process per GPU, RCCL over xGMI.

Replaces the DDP reducer that HF Trainer / accelerate wrap around the reference
(script/train.py:259-308, src/custom_trainer.py:4-41): gradients live in ONE flat fp32 arena
buffer, so the all-reduce is a handful of large contiguous buckets (no per-parameter copy
into bucket storage) issued on a dedicated communication stream. Gradients are averaged
(sum / world), like DDP. Parameters and BN buffers are broadcast from rank 0 at start; BN
running statistics follow DDP's broadcast_buffers=True semantics (rank 0's buffers win).
"""
import os

import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20   # 64 MiB buckets: ~7 links x ~153 GB/s per GPU want big messages


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
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


class GradReducer:
    """Bucketed averaging all-reduce of a flat fp32 gradient buffer."""

    def __init__(self, flat_grad, bucket_bytes=BUCKET_BYTES, group=None, use_stream=True):
        self.flat = flat_grad
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        n = flat_grad.numel()
        step = max(1, bucket_bytes // flat_grad.element_size())
        self.buckets = [(s, min(n, s + step)) for s in range(0, n, step)]
        self.stream = torch.cuda.Stream(device=flat_grad.device) if (use_stream and flat_grad.is_cuda) else None

    def allreduce(self, average=True):
        """sum over ranks; average=False leaves the 1/world scale to the optimizer
        (FusedAdamW.step(grad_scale=1/world)) and saves a pass over the buffer."""
        if self.world == 1:
            return
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.flat.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                works = [dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                         for a, b in self.buckets]
                for w in works:
                    w.wait()
                if average:
                    self.flat.mul_(1.0 / self.world)
            cur.wait_stream(self.stream)
        else:
            for a, b in self.buckets:
                dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, group=self.group)
            if average:
                self.flat.mul_(1.0 / self.world)


def broadcast_state(flat_params, buffers, src=0, group=None):
    """Make every rank start from rank 0's parameters and buffers (DDP construction)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.broadcast(flat_params, src=src, group=group)
    for b in buffers:
        dist.broadcast(b, src=src, group=group)
