"""ArenaDDP (avsr_amd/parallel.py) on CPU, gloo, world_size 2: the DistributedDataParallel
semantics the reference trains under — rank-0 broadcast at construction, gradient
averaging with readiness-watermark buckets, no_sync() accumulation over gradient-accumulation
micro-steps, and the per-forward BatchNorm statistics broadcast that follows DDP's
require_forward_param_sync rule (a forward after a no_sync backward does not broadcast).
The engine is replaced by a stub that calls ArenaDDP's hooks in the engine's order."""
import os
import socket
import types

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from avsr_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _StubArena:
    def __init__(self, n, rank):
        self.data = torch.full((n,), float(rank + 1))
        self.grad = torch.zeros(n)
        self.segments = {"decay": (0, n - 100), "no_decay": (n - 100, n), "frozen": (n, n)}

    def sync_shadow(self):
        pass


class _StubEngine:
    """calls the DP hooks where Engine.forward / Engine.backward do"""

    def __init__(self, n, rank):
        self.arena = _StubArena(n, rank)
        self.bn_flat = torch.full((37,), 100.0 + rank)
        self.before_forward = self.before_backward = self.on_grad_ready = self.after_backward = None

    def forward(self):
        if self.before_forward is not None:
            self.before_forward()

    def backward(self, g):
        if self.before_backward is not None:
            self.before_backward()
        self.arena.grad += g
        for off in (self.arena.segments["decay"][1] // 2, 0):     # per-layer readiness watermarks
            self.on_grad_ready(off)
        self.after_backward()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env(backend="gloo")
        n = 70001
        eng = _StubEngine(n, rank)
        model = types.SimpleNamespace(avsr=types.SimpleNamespace(engine=lambda: eng),
                                      buffers=lambda: [torch.tensor([rank], dtype=torch.int64)])
        ddp = parallel.ArenaDDP(model, bucket_bytes=4 * 8192, average=True, use_stream=False)
        res = {"bcast_params": bool((eng.arena.data == 1.0).all()), "bcast_bn": bool((eng.bn_flat == 100.0).all())}
        base = torch.arange(n, dtype=torch.float32)
        # GA = 2: micro-step 1 under no_sync (local accumulation), micro-step 2 synchronises
        eng.bn_flat.fill_(200.0 + rank)
        with ddp.no_sync():
            eng.forward()                       # previous state synced -> broadcast
            eng.backward(base * (rank + 1))
        res["bn_after_first_forward"] = float(eng.bn_flat[0])
        res["local_after_no_sync"] = bool(torch.equal(eng.arena.grad, base * (rank + 1)))
        eng.bn_flat.fill_(300.0 + rank)
        eng.forward()                           # previous forward was no_sync -> no broadcast
        res["bn_after_second_forward"] = float(eng.bn_flat[0])
        eng.backward(base * 10 * (rank + 1))
        want = (base * 11 * (1 + 2)) / 2       # mean over ranks of (mb1 + mb2)
        res["averaged"] = bool(torch.allclose(eng.arena.grad, want, rtol=1e-6))
        eng.bn_flat.fill_(400.0 + rank)
        eng.forward()                           # previous backward synchronised -> broadcast
        res["bn_after_third_forward"] = float(eng.bn_flat[0])
        res["broadcasts"] = ddp.buffer_broadcasts
        q.put((rank, res))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_arena_ddp_semantics_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        r = res[rank]
        assert r["bcast_params"] and r["bcast_bn"], r
        assert r["local_after_no_sync"] and r["averaged"], r
        assert r["bn_after_first_forward"] == 200.0, r            # rank 0's buffers win
        assert r["bn_after_second_forward"] == 300.0 + rank, r    # no broadcast after no_sync
        assert r["bn_after_third_forward"] == 400.0, r
        assert r["broadcasts"] == 2, r
