"""Data-parallel plumbing on CPU with the gloo backend, world_size 2:
the bucketed gradient all-reduce of the flat arena buffer (sum and average, buckets that
split the buffer unevenly) and the rank-0 parameter / buffer broadcast."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from avsr_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = parallel.init_from_env(backend="gloo")
        assert (r, w) == (rank, world)
        n = 1000003                                   # odd size: last bucket is short
        g = torch.arange(n, dtype=torch.float32) * (rank + 1)
        red = parallel.GradReducer(g, bucket_bytes=4 * 65536)
        assert len(red.buckets) == (n + 65535) // 65536
        red.allreduce(average=False)
        want = torch.arange(n, dtype=torch.float32) * sum(range(1, world + 1))
        ok_sum = torch.equal(g, want)
        red.allreduce(average=True)                   # sum over ranks of identical buffers / world
        ok_avg = torch.allclose(g, want, rtol=1e-6)
        # overlapped protocol: readiness watermarks over the decay segment, then finish();
        # every element must be reduced exactly once
        g2 = torch.arange(n, dtype=torch.float32) * (rank + 1)
        red2 = parallel.GradReducer(g2, bucket_bytes=4 * 50000, segment=(1000, 900000))
        red2.begin()
        for off in (850000, 850000, 600001, 400000, 1000):
            red2.ready(off)
        red2.finish(average=False)
        ok_sum = ok_sum and torch.equal(g2, want)
        params = torch.full((17,), float(rank))
        bufs = [torch.full((3,), 10.0 + rank), torch.tensor([rank], dtype=torch.int64)]
        parallel.broadcast_state(params, bufs)
        ok_bc = bool((params == 0).all()) and bool((bufs[0] == 10).all()) and int(bufs[1]) == 0
        q.put((rank, ok_sum, ok_avg, ok_bc))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_reducer_and_broadcast_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_sum, ok_avg, ok_bc in res:
        assert ok_sum and ok_avg and ok_bc, (rank, ok_sum, ok_avg, ok_bc)


def _worker_compress(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env(backend="gloo")
        n = 300007
        gen = torch.Generator().manual_seed(100 + rank)
        base = torch.randn(n, generator=gen) * torch.logspace(-6, 2, n)    # gradients over 8 decades
        exact = base.clone()
        parallel.GradReducer(exact, bucket_bytes=4 * 40000).allreduce(average=True)
        comp = base.clone()
        red = parallel.GradReducer(comp, bucket_bytes=4 * 40000, segment=(7, 250000), compress="bf16")
        red.begin()
        for off in (200000, 100000, 7):
            red.ready(off)
        red.finish(average=True)
        # bf16 keeps 8 significant bits: each rank's value is rounded once (2^-9 relative), the
        # two-rank sum once more; relative to the larger of the two summands
        scale = torch.maximum(base.abs(), (2 * exact - base).abs())
        err = ((comp - exact).abs() / scale.clamp_min(1e-30)).max().item()
        differs = not torch.equal(comp, exact)
        q.put((rank, err, differs))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_reducer_bf16_compression_world2():
    """GradReducer(compress="bf16"): every bucket (decay segment by readiness watermarks, then
    the tail) is exchanged in bf16 and decompressed into the fp32 arena; the result agrees with
    the fp32 exchange to bf16 rounding (and is not silently the uncompressed path)."""
    with pytest.raises(ValueError):
        parallel.GradReducer(torch.zeros(8), compress="fp8")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_compress, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, differs in res:
        assert err < 2 ** -7, (rank, err)
        assert differs, rank


def _ld_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from avsr_amd.optim import union_touched
        parallel.init_from_env(backend="gloo")
        local = {0, 3} if rank == 0 else {3, 5}         # LayerDrop kept different layers per rank
        q.put((rank, sorted(union_touched(local, 8))))
        dist.destroy_process_group()
    except Exception as e:                              # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


def test_layerdrop_touched_union_world2():
    """LayerDrop + DDP: every rank updates the layers that ANY rank's backward touched (the
    all-reduced gradient is nonzero there on every rank), so the replicas stay identical"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ld_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert out == {0: [0, 3, 5], 1: [0, 3, 5]}, out
