"""Data-parallel parity on the GPU: two ranks on cuda:0 over gloo with CUDA
tensors (the box has one GPU; the exchange protocol is the one RCCL runs at 8 GPUs), the tiny
model in fp32 parity mode, ArenaDDP on the communication stream with the engine's real
per-layer readiness watermarks.

  * one synchronising step: every rank's averaged gradient arena equals the mean of the two
    single-process per-shard gradients (the reference's DDP semantics: per-rank BatchNorm
    batch statistics, gradients averaged);
  * gradient accumulation 2 with no_sync() on the first micro-step: the result equals the mean
    over ranks of the accumulated micro-step gradients (no double reduction);
  * BatchNorm running statistics: rank 0's win at construction and are broadcast before a
    forward that follows a synchronising backward (DDP broadcast_buffers=True);
  * mixed modality draws: rank 0 draws video_off (its ResNet backward is skipped), rank 1 draws
    none, in the same synchronising step — what every C3 step with modality dropout does
    (avhubert.py:476-482); the averaged arena equals the mean of the per-shard gradients;
  * the reference's module-level encoder call (model.avsr.encoder(input_features=, video=),
    surface.py) trained under ArenaDDP: the same parity on its gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(state, cfg_kw):
    from avsr_amd.avhubert_avsr_model import AVHubertAVSR
    from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
    m = AVHubertAVSR(AVHubertAVSRConfig(**cfg_kw)).train()
    m.load_state_dict(state, strict=True)
    m.setup_engine("cuda:0", torch.float32)
    return m


def _shard(batch, r):
    return {k: v[r:r + 1].contiguous() for k, v in batch.items()}


def _grads(m, shards, scale, modality=None):
    eng = m.avsr.engine()
    eng.force_modality = None if modality is None else (modality,)
    m.zero_grad()
    for sh in shards:
        (m(**sh).loss * scale).backward()
    torch.cuda.synchronize()
    eng.force_modality = None
    return eng.arena.grad.clone()


def _enc_grads(m, sh, wout):
    """the surface encoder call in train mode, loss = <encoder output, wout>"""
    m.zero_grad()
    out = m.avsr.encoder(input_features=sh["audios"], video=sh["videos"]).last_hidden_state
    (out * wout[:out.shape[1]].to(out.device)).sum().backward()
    torch.cuda.synchronize()
    return m.avsr.engine().arena.grad.clone()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    res = {}
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        torch.cuda.set_device(0)
        from avsr_amd import parallel
        from oracle.weights import NO_DROPOUT, TINY_CONFIG
        from tests.oracle_util import golden_batch, golden_state, load_golden
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = load_golden()
        state = {k: torch.from_numpy(v) for k, v in golden_state(g).items()}
        batch = {k: torch.from_numpy(v) for k, v in golden_batch(g).items()}
        cfg_kw = dict(**TINY_CONFIG, **NO_DROPOUT)
        # single-process references: per-shard gradients of both shards
        ref_m = _model(state, cfg_kw)
        g0 = _grads(ref_m, [_shard(batch, 0)], 1.0)
        g1 = _grads(ref_m, [_shard(batch, 1)], 1.0)
        mean = (g0 + g1) / 2
        mix = ("video_off", None)                       # rank 0 / rank 1 draws of the mixed step
        gm = [_grads(ref_m, [_shard(batch, r)], 1.0, modality=mix[r]) for r in range(2)]
        mean_mix = (gm[0] + gm[1]) / 2
        wout = torch.randn(batch["videos"].shape[2], cfg_kw["hidden_size"],
                           generator=torch.Generator().manual_seed(3))
        ge = [_enc_grads(ref_m, _shard(batch, r), wout) for r in range(2)]
        mean_enc = (ge[0] + ge[1]) / 2
        del ref_m
        # DDP model: rank r trains on shard r
        m = _model(state, cfg_kw)
        eng = m.avsr.engine()
        bn0 = eng.bn_flat.clone()
        if rank == 1:                                   # diverged running statistics on rank 1
            eng.bn_flat.add_(1.0)
        ddp = parallel.ArenaDDP(m, bucket_bytes=1 << 20, average=True, use_stream=True)
        res["n_buckets"] = len(ddp.reducer.buckets)
        res["bn_equal_after_init"] = bool(torch.equal(eng.bn_flat, bn0))
        got = _grads(m, [_shard(batch, rank)], 1.0)
        scale = mean.abs().max().item()
        res["sync_err"] = (got - mean).abs().max().item() / scale
        # gradient accumulation: micro-steps (shard r, shard 1-r), loss / 2 each
        m.zero_grad()
        with m.no_sync():
            (m(**_shard(batch, rank)).loss * 0.5).backward()
        torch.cuda.synchronize()
        local = eng.arena.grad.clone()
        res["no_sync_local_err"] = (local - g0 * 0.5 if rank == 0 else local - g1 * 0.5).abs().max().item() / scale
        (m(**_shard(batch, 1 - rank)).loss * 0.5).backward()
        torch.cuda.synchronize()
        res["ga_err"] = (eng.arena.grad - mean).abs().max().item() / scale
        # BN statistics broadcasts (DDP rule): before the first forward and before the forward
        # that follows a synchronising backward; not after the no_sync micro-step
        res["broadcasts"] = ddp.buffer_broadcasts
        # mixed modality step: the ResNet gradient of rank 0's shard is exactly zero
        rn = [(mt["off"], mt["off"] + mt["numel"]) for n, mt in eng.arena.meta.items()
              if ".resnet." in n and n in eng.arena.grad_views]
        got = _grads(m, [_shard(batch, rank)], 1.0, modality=mix[rank])
        res["mix_err"] = (got - mean_mix).abs().max().item() / mean_mix.abs().max().item()
        res["mix_video_zero_r0"] = (len(rn) > 0 and all(gm[0][a:b].abs().max().item() == 0 for a, b in rn)
                                    and any(gm[1][a:b].abs().max().item() > 0 for a, b in rn))
        # surface encoder call under DDP (its forward broadcasts BN buffers, its backward reduces)
        got = _enc_grads(m, _shard(batch, rank), wout)
        res["enc_err"] = (got - mean_enc).abs().max().item() / mean_enc.abs().max().item()
        res["enc_nonzero"] = bool(mean_enc.abs().max().item() > 0)
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        res["error"] = traceback.format_exc()
    finally:
        q.put((rank, res))
        if dist.is_initialized():
            dist.destroy_process_group()


def test_dp_world2_gradient_parity():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank in range(world):
        r = res[rank]
        assert "error" not in r, r.get("error")
        assert r["n_buckets"] > 4, r
        assert r["bn_equal_after_init"], r
        assert r["sync_err"] < 1e-5, r
        assert r["no_sync_local_err"] < 1e-5, r
        assert r["ga_err"] < 1e-5, r
        assert r["broadcasts"] == 2, r
        assert r["mix_err"] < 1e-5 and r["mix_video_zero_r0"], r
        assert r["enc_err"] < 1e-5 and r["enc_nonzero"], r
    for p in procs:
        assert p.exitcode == 0
