"""Throughput benchmark of the AVSR hot path (BASELINE.json metric / config C2, C3).

One step = forward + backward + (RCCL gradient all-reduce) + fused clip/AdamW of the full
AVHubertAVSR model (24-layer AV-HuBERT-Large encoder, ResNet-18 lip frontend, 6-layer
decoder, joint CTC/attention loss) on 16 synthetic 15 s clips per GPU (T = 375 AV-frames,
L = 40 labels), train mode (dropouts on), bf16 compute / fp32 master weights.
Inputs are resident in HBM before the timed region (SURVEY.md §8(d) d1 recipe).

  python bench.py [--gpus N --steps K --warmup W]

With N > 1 and no torch.distributed.run environment (WORLD_SIZE unset) this process is only
a launcher: it never touches the GPU, starts N child ranks of itself with RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, relays rank 0's JSON line and exits
non-zero if any rank fails (reference: torchrun over script/train.py:23,259-308). Under
`python -m torch.distributed.run ... bench.py --gpus N` the ranks run directly.

Prints ONE JSON line (rank 0). `roofline` is measured live on the probe kernel (the encoder
FFN up-projection GEMM, 6000x4096x1024 bf16, 24 launches per step) from in-kernel
s_memrealtime stamps (first workgroup start to last workgroup end of each launch);
`cpu_baseline` times the repo's CPU restatement of the same model (oracle/, "port") on the
host cores on a bounded sample. `--cpu-selftest` (no GPU, gloo) exercises the launcher and the
bucketed all-reduce only — it measures nothing and is what the CPU test suite runs.
"""
import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "AV-frames/sec/GPU (fwd+bwd) on 15s clips; WER parity on LRS2 test"
BF16_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
# modality dropout (avhubert.py:476-482): p(drop a modality) = 0.5, then audio w.p. 0.5
MODALITY_P = {"none": 0.5, "audio_off": 0.25, "video_off": 0.25}


# ============================================================================ launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Spawn n ranks of this script (the parent never initialises HIP: it only imports torch).
    Rank 0's stdout is relayed; returns the exit code (first failing rank's, 0 if all pass,
    1 if rank 0 printed no JSON line)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    last_json = []

    def pump():
        for line in procs[0].stdout:
            sys.stdout.write(line)
            sys.stdout.flush()
            if line.startswith("{"):
                last_json.append(line)
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                sys.stderr.write(f"[bench] rank {procs.index(p)} exited with {code}; stopping the others\n")
                for q in live:
                    q.terminate()
                deadline = time.time() + 30
                for q in live:
                    try:
                        q.wait(timeout=max(1.0, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
        time.sleep(0.2)
    th.join(timeout=10)
    if rc == 0 and not last_json:
        sys.stderr.write("[bench] rank 0 printed no result line\n")
        rc = 1
    return rc


# ========================================================================= inputs, FLOPs
def synthetic_batch(B, T, L, seed=1234):
    """uint8 96x96 lip frames -> crop 88 -> /255 -> (x-0.421)/0.165;
    standard-normal 104-dim 'mel' frames with per-frame LayerNorm; labels U[1, 5047]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    frames = rng.integers(0, 256, size=(B, T, 96, 96), dtype=np.uint8)
    v = (frames[:, :, 4:92, 4:92].astype(np.float32) / 255.0 - 0.421) / 0.165
    rng2 = np.random.Generator(np.random.PCG64(seed + 1))
    a = rng2.standard_normal((B, T, 104)).astype(np.float32)
    a = (a - a.mean(-1, keepdims=True)) / np.sqrt(a.var(-1, keepdims=True) + 1e-5)
    rng3 = np.random.Generator(np.random.PCG64(seed + 2))
    lab = rng3.integers(1, 5048, size=(B, L)).astype(np.int64)
    return (torch.from_numpy(v[:, None]), torch.from_numpy(np.ascontiguousarray(a.transpose(0, 2, 1))),
            torch.full((B,), T, dtype=torch.int64), torch.from_numpy(lab))


def model_flops_per_frame(cfg, T, L, variant="none"):
    """algorithmic fwd+bwd FLOPs per AV-frame: 3x the forward MACs*2.
    variant "video_off" runs the ResNet forward only (its backward is skipped: the gradient is
    exactly zero, avhubert.py:480), so the ResNet's backward FLOPs are not counted for it."""
    D, F, nl = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    enc = nl * (2 * (4 * D * D + 2 * D * F) + 4 * T * D)            # per frame, forward
    # ResNet-18 frontend forward per frame (conv MACs * 2), stem + 4 stages + 512->D proj
    stem = 2 * 44 * 44 * 64 * 5 * 49
    res = 0
    for (hw, cin, cout, s) in [(22, 64, 64, 1), (22, 64, 64, 1), (22, 64, 128, 2), (11, 128, 128, 1),
                               (11, 128, 256, 2), (6, 256, 256, 1), (6, 256, 512, 2), (3, 512, 512, 1)]:
        ho = (hw + 2 - 3) // s + 1
        res += 2 * ho * ho * cout * cin * 9 + 2 * ho * ho * cout * cout * 9
        if s != 1 or cin != cout:
            res += 2 * ho * ho * cout * cin
    front = stem + res + 2 * 512 * D + 2 * 104 * D + 2 * 2 * D * D
    posconv = 2 * D * (D // cfg.num_conv_pos_embedding_groups) * cfg.num_conv_pos_embeddings
    ctc = 2 * D * cfg.odim
    dD, dF, dl = cfg.ddim, cfg.dunits, cfg.dlayers
    L1 = L + 1
    dec_tok = dl * (2 * (4 * dD * dD + 2 * dD * dF) + 4 * L1 * dD + 4 * T * dD) + 2 * dD * cfg.odim
    dec = (dec_tok * L1 + dl * 2 * 2 * T * dD * dD) / T               # memory K/V projections per frame
    fwd = enc + front + posconv + ctc + dec
    # backward = 2x forward except the stem (no data-grad): stem counted fwd + wgrad only
    total = 3 * fwd - stem
    if variant == "video_off":
        total -= 2 * res + stem
    return total


def stratified_variants(steps, rank):
    """modality variant of each timed step: the reference draws it per forward (p = 0.5 none,
    0.25 audio_off, 0.25 video_off; avhubert.py:476-482); the bench takes the same distribution
    stratified (period 4: none, video_off, none, audio_off; rotated per rank so ranks differ
    like independent draws), so `value` is the expected-mix throughput instead of one draw's"""
    pat = [None, "video_off", None, "audio_off"]
    return [pat[(i + rank) % 4] for i in range(steps)]


def expected_step_ms(variant_ms, world):
    """E[step time] when every rank draws its modality independently with the reference's
    probabilities and a step lasts as long as its slowest rank (the all-reduce joins them)."""
    lv = sorted((variant_ms[k], MODALITY_P[k]) for k in MODALITY_P)
    e, cum_prev = 0.0, 0.0
    for ms, p in lv:
        cum = cum_prev + p
        e += ms * (cum ** world - cum_prev ** world)
        cum_prev = cum
    return e


# ===================================================================== CPU baselines
def _oracle_cfg(model_cfg):
    from oracle import avsr_oracle as O
    return O.OracleConfig.from_dict(dict(odim=model_cfg.odim, hidden_size=model_cfg.hidden_size,
                                         num_attention_heads=model_cfg.num_attention_heads,
                                         intermediate_size=model_cfg.intermediate_size,
                                         num_hidden_layers=model_cfg.num_hidden_layers, ddim=model_cfg.ddim,
                                         dheads=model_cfg.dheads, dunits=model_cfg.dunits, dlayers=model_cfg.dlayers))


def cpu_baseline(model_cfg, state, T, threads, budget_s=10.0, max_clips=8):
    """Time the repo's CPU restatement (oracle/avsr_oracle.py) fwd+bwd on 15 s clips, one at a
    time, until budget_s of CPU work (at least one clip, at most max_clips)."""
    from oracle import avsr_oracle as O
    torch.set_num_threads(threads)
    cfg = _oracle_cfg(model_cfg)
    sd = {k: v.detach().float().cpu().clone() for k, v in state.items()}
    for k, v in sd.items():
        if v.is_floating_point() and not (k.endswith("running_mean") or k.endswith("running_var")):
            v.requires_grad_(True)
    clips, t0 = 0, time.perf_counter()
    while clips < max_clips and (clips == 0 or time.perf_counter() - t0 < budget_s):
        v, a, lens, lab = synthetic_batch(1, T, 40, seed=99 + clips)
        loss, *_ = O.e2e_forward(sd, cfg, v, a, lens, lab, train=True)
        loss.backward()
        clips += 1
    dt = time.perf_counter() - t0
    return clips * T / dt, dt, clips


def decode_cpu_baseline(model_cfg, state, T, beam, threads, steps=None):
    """oracle/decode_oracle.py beam search (the reference's BatchBeamSearch restated) on ONE
    utterance of T frames, all T output steps a random-weight search takes (each step scores the
    full T-frame CTC prefix); steps < T: the first `steps`, extrapolated (debug runs)."""
    from oracle import decode_oracle as D
    torch.set_num_threads(threads)
    cfg = _oracle_cfg(model_cfg)
    sd = {k: v.detach().float().cpu() for k, v in state.items()}
    W, b = sd["avsr.ctc.ctc_lo.weight"], sd["avsr.ctc.ctc_lo.bias"]
    x = torch.randn(T, model_cfg.hidden_size, generator=torch.Generator().manual_seed(5)) * 0.5
    steps = T if steps is None else min(steps, T)
    t0 = time.perf_counter()
    with torch.no_grad():
        lp = torch.log_softmax(x @ W.t() + b, -1)
        D.beam_search(sd, cfg, x, lp, beam, ctc_weight=0.1, maxlenratio=-steps)
    dt = time.perf_counter() - t0
    per_step = dt / steps
    return {"value": round(1.0 / (per_step * T), 4), "unit": "utt/s", "cores": threads, "kind": "port",
            "sample": f"1 utterance, T={T}, beam {beam}, fp32: {steps} of {T} decode steps in {dt:.1f} s"
                      + ("" if steps == T else f", extrapolated to {T} steps")}


# ======================================================================= side measurements
def frontend_timing(B, T, dev, reps=5):
    """Device front end on one C2 batch -- 16 x 240000-sample waveforms -> log-fbank /
    stack / LN, 16 x T x 96 x 96 uint8 frames -> crop / normalise. Reported beside the metric,
    not part of `value` (the reference runs these in CPU collator workers)."""
    from avsr_amd import frontend
    g = torch.Generator(device="cpu").manual_seed(99)
    wav = (0.1 * torch.randn(B, 640 * T, generator=g)).to(dev)
    ns = torch.full((B,), 640 * T, dtype=torch.int64)
    fr = torch.randint(0, 256, (B, T, 96, 96), generator=g, dtype=torch.uint8).to(dev)
    frontend.audio_features(wav, ns, T=T)
    frontend.video_transform(fr)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        frontend.audio_features(wav, ns, T=T)
        frontend.video_transform(fr)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    return {"ms_per_batch": round(ms, 3), "clips_per_s": round(B / ms * 1e3, 1),
            "what": f"{B} clips: log-fbank+stack4+LN of {640 * T} samples and crop/normalise of {T}x96x96 u8 frames"}


def encoder_gemm_table(dev, M, D, F):
    """the 12 GEMM shapes of one encoder layer (QKV, out-proj, FFN1, FFN2 x fwd / dgrad /
    wgrad with the engine's split-K policy), each timed alone (HIP graph, plain epilogue,
    N(0, 0.25) operands); outside the timed region. Returns per-shape TF/s and the worst."""
    from avsr_amd import ops
    from tools.gemm_table import timed, wgrad
    g = torch.Generator(device="cpu").manual_seed(0)
    from avsr_amd import engine
    rows, wg = [], {}
    for name, (N, K) in {"qkv": (3 * D, D), "out": (D, D), "ffn1": (F, D), "ffn2": (D, F)}.items():
        x = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
        W = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        dy = (torch.randn(M, N, generator=g) * 0.5).to(dev, torch.bfloat16)
        dW = torch.zeros(N, K, device=dev)
        wg[name] = (dy, x, dW)
        fl = 2.0 * M * N * K
        for op, fn in (("fwd", lambda: ops.linear_fwd(x, W)), ("dgrad", lambda: ops.linear_dgrad(dy, W)),
                       ("wgrad", lambda: wgrad(dy, x, dW))):
            us = timed(fn)
            tf = fl / us / 1e6
            rows.append({"gemm": f"{name} {op}", "us": round(us, 1), "tflops": round(tf, 1),
                         "frac": round(tf / BF16_PEAK_TFLOPS, 4),
                         "engine": not (engine.WGRAD_GROUP and op == "wgrad" and name in ("qkv", "out"))})
    # the engine's QKV + out-proj weight-gradients: one grouped launch (192 + 64 output tiles)
    us = timed(lambda: ops.wgrad_group([wg["qkv"] + (1.0,), wg["out"] + (1.0,)]))
    fl = 2.0 * M * (3 * D * D + D * D)
    tf = fl / us / 1e6
    rows.append({"gemm": "qkv+out wgrad (grouped)", "us": round(us, 1), "tflops": round(tf, 1),
                 "frac": round(tf / BF16_PEAK_TFLOPS, 4), "engine": bool(engine.WGRAD_GROUP)})
    used = [r for r in rows if r["engine"]]
    worst = min(used, key=lambda r: r["frac"])
    tot_us = sum(r["us"] for r in used)
    tot_fl = sum(2.0 * M * N * K for (N, K) in ((3 * D, D), (D, D), (F, D), (D, F))) * 3
    return {"per_shape": rows, "worst": worst, "layer_us": round(tot_us, 1),
            "layer_frac": round(tot_fl / tot_us / 1e6 / BF16_PEAK_TFLOPS, 4),
            "note": "isolated launches, plain epilogue (tools/gemm_table.py); worst / layer over the launches the "
                    "engine makes (engine: true); the in-step probe is `roofline`"}


def decode_throughput(dev, state_cpu, model_cfg, cpu_threads):
    """C1 (8 x 1 s, greedy), C4 (LRS2-length 4 s utterances, beam 3) and C5 (15 s chunks,
    beam 5) decode on the HIP engine, fp32 like the reference's evaluation
    (script/evaluation.py:89-108): random-init weights, so every search runs to maxlen = T.
    Batched over 8 utterances (decode_batch) and, for C1 / C4, the reference's one-utterance
    call form. cpu_baseline: the oracle's beam search on one utterance (bounded)."""
    from avsr_amd.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
    from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
    torch.manual_seed(0)
    model = AVHubertAVSR(AVHubertAVSRConfig(odim=5049)).eval()
    if state_cpu is not None:
        model.load_state_dict(state_cpu, strict=True)
    model.setup_engine(dev, torch.float32)
    tokens = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
    out = []
    for name, T, beam, seq in (("C1 greedy", 25, 1, True), ("C4 beam 3", 100, 3, True), ("C5 beam 5", 375, 5, False)):
        bs = get_beam_search_decoder(model.avsr, tokens, ctc_weight=0.1, beam_size=beam)
        g = torch.Generator().manual_seed(5)
        xs = [(torch.randn(T, 1024, generator=g) * 0.5).to(dev) for _ in range(8)]
        bs.decode_batch(xs[:2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bat = bs.decode_batch(xs)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rec = {"config": name, "utterances": 8, "frames_per_utt": T, "beam": beam, "dtype": "fp32",
               "batched_utt_per_s": round(8 / (t1 - t0), 2)}
        if seq:
            t0 = time.perf_counter()
            one = [bs(x) for x in xs]
            torch.cuda.synchronize()
            rec["sequential_utt_per_s"] = round(8 / (time.perf_counter() - t0), 2)
            rec["batched_equals_sequential"] = all(
                [h.asdict()["yseq"] for h in a] == [h.asdict()["yseq"] for h in b] for a, b in zip(one, bat))
        if state_cpu is not None:
            rec["cpu_baseline"] = decode_cpu_baseline(model_cfg, state_cpu, T, beam, cpu_threads)
        out.append(rec)
    del model
    torch.cuda.empty_cache()
    return out


# ===================================================================== CPU self-test
def cpu_selftest(args):
    """No GPU: the launcher, rendezvous, barrier + max-over-ranks timing and the bucketed
    all-reduce of a flat fp32 gradient arena (parallel.GradReducer over gloo, readiness
    watermarks like the engine's backward) are exercised and checked. Not a measurement."""
    from avsr_amd import parallel
    if os.environ.get("AVSR_BENCH_SELFTEST_FAIL_RANK") == os.environ.get("RANK", "0"):
        sys.exit(7)            # test hook: a rank dying before the rendezvous (tests/test_bench_launcher.py)
    rank, world, _ = parallel.init_from_env(backend="gloo")
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    n = 3_000_001
    flat = torch.zeros(n)
    seg = (1000, 2_500_000)
    red = parallel.GradReducer(flat, bucket_bytes=4 << 18, segment=seg, use_stream=False, compress=args.grad_compress)
    ok = True
    for _ in range(args.warmup):
        flat.fill_(rank + 1.0)
        red.begin()
        red.finish(average=True)
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        flat.copy_(torch.arange(n, dtype=torch.float32) * (rank + 1 + i))
        red.begin()
        for off in (2_000_000, 1_200_000, 400_000, seg[0]):     # layers finishing back to front
            red.ready(off)
        red.finish(average=True)
        want = torch.arange(n, dtype=torch.float32) * (sum(range(1, world + 1)) / world + i)
        ok = ok and torch.allclose(flat, want, rtol=1e-6 if args.grad_compress is None else 2 ** -7)
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    okt = torch.tensor([1 if ok else 0])
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    res = {"metric": "cpu-selftest (launcher + bucketed all-reduce; not a measurement)", "value": None,
           "unit": None, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(t.item() / max(1, args.steps) * 1e3, 3), "data": "synthetic",
           "allreduce": {"backend": dist.get_backend(), "ranks": dist.get_world_size(),
                         "buckets": len(red.buckets) + len(red.tail), "elements": n,
                         "compress": args.grad_compress or "none (fp32)",
                         "mean_ok": bool(okt.item())}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    return 0 if okt.item() else 3


# ============================================================================ GPU bench
def gpu_bench(args):
    from avsr_amd import parallel
    rank, world, local = parallel.init_from_env()
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from avsr_amd.engine import prioritize_step_stream
    prioritize_step_stream(dev)      # the step's stream above the weight-grad side stream (AVSR_MAIN_PRIO=0: off)
    from avsr_amd import ops
    from avsr_amd.avhubert_avsr_model import AVHubertAVSR
    from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
    from avsr_amd.optim import FusedAdamW

    torch.manual_seed(0)
    kw = {} if args.layers is None else {"num_hidden_layers": args.layers}
    cfg = AVHubertAVSRConfig(odim=5049, **kw)
    model = AVHubertAVSR(cfg).train()
    state_cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        state_cpu = {k: v.clone() for k, v in model.state_dict().items()}
    model.setup_engine(dev, torch.bfloat16)
    eng = model.avsr.engine()
    arena = eng.arena
    # DDP semantics on the arena: rank-0 broadcast of parameters + buffers, per-forward BN
    # statistics broadcast, bucketed RCCL all-reduce overlapped with the backward; the 1/world
    # average is folded into the AdamW kernel (average=False, grad_scale below)
    ddp = parallel.ArenaDDP(model, average=False, compress=args.grad_compress)
    from avsr_amd import engine as _engine
    opt = FusedAdamW(arena, lr=1e-4, weight_decay=0.005, max_grad_norm=1.0, overlap=_engine.OPT_OVERLAP)
    opt.overlap_blocks = _engine.OPT_OVERLAP_BLOCKS
    opt.clear_in_update = _engine.OPT_CLEAR_IN_UPDATE
    if world == 1 and _engine.EARLY_NORM:   # gradient norm of all but the ResNet beside the ResNet backward
        eng.pre_video_grads = opt.early_sumsq

    B, T, L = args.batch, args.seq, args.labels
    v, a, lens, lab = synthetic_batch(B, T, L, seed=args.seed + rank)
    v, a = v.to(dev), a.to(dev)
    mtl = cfg.mtlalpha
    d_ctc = torch.full((1,), mtl, device=dev)
    d_att = torch.full((1,), 1.0 - mtl, device=dev)

    # the import-time heap goes to the collector's permanent generation (a full collection
    # inside a step stalled the host for 0.1-0.15 s once per run)
    if os.environ.get("AVSR_BENCH_GCFREEZE", "1") == "1":
        gc.collect()
        gc.freeze()
    # untimed warm-up of each modality variant's step first (no RNG draws): every allocation
    # pattern the timed steps can take is in the caching allocator's pool before timing
    for forced in ((None, "video_off", "audio_off") if os.environ.get("AVSR_BENCH_PRIME", "1") == "1" else ()):
        eng.force_modality = (forced,)
        arena.zero_grad()
        _, ctx = eng.forward(v, a, lens, lab, train=True, need_grad=True, seed=1)
        eng.backward(ctx, d_ctc, d_att)
        del ctx
    eng.force_modality = None
    torch.cuda.synchronize()
    arena.zero_grad()

    # modality dropout (avhubert.py:476-482) draws from numpy's global RNG like the reference;
    # seeded here so that the timed steps' decisions are reproducible and reported
    np.random.seed(args.seed + 7919 * rank)
    drops = []
    step_seed = [args.seed * 1000003 + rank]

    forced_all = None if args.force_modality is None else (
        (None if args.force_modality == "none" else args.force_modality),)
    # per-step variants: stratified (default), or the reference's own random draw (--modality-draws random)
    strat = args.modality_draws == "stratified"
    sched = stratified_variants(args.warmup + args.steps, rank)

    def step(i=None, variant=False):
        if forced_all is not None and not variant:
            eng.force_modality = forced_all
        elif strat and not variant:
            eng.force_modality = (sched[i],)
        eng.zero_grad_async()                   # the gradient clear runs on the side stream
        step_seed[0] += 1
        out4, ctx = eng.forward(v, a, lens, lab, train=True, need_grad=True, seed=step_seed[0])
        drops.append(eng.last_modality)
        eng.backward(ctx, d_ctc, d_att)
        opt.step(grad_scale=1.0 / world)
        return out4

    for i in range(args.warmup):
        out4 = step(i)
    torch.cuda.synchronize()
    # probe: encoder FFN up-projection (M = B*T, N = F, K = D), forward, bf16
    M, N_, K_ = B * T, cfg.intermediate_size, cfg.hidden_size
    nprobe = args.steps * cfg.num_hidden_layers + 8
    stamps = torch.zeros(nprobe, 2, dtype=torch.int64, device=dev)
    stamps[:, 0] = -1                                   # {~0ull, 0}: min-start / max-end identities
    ops.PROBE["gemm"] = {"match": lambda m, n, k, ak, bk, dt: (m, n, k, ak, bk) == (M, N_, K_, True, True),
                         "events": [], "stamps": stamps.view(-1)}
    red = ddp.reducer
    red.timing = [] if world > 1 else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    drops.clear()
    ms0 = torch.cuda.memory_stats(dev)
    host_t = []
    step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    step_ev[0].record()
    for i in range(args.steps):
        h0 = time.perf_counter()
        out4 = step(args.warmup + i)
        step_ev[i + 1].record()
        host_t.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms1 = torch.cuda.memory_stats(dev)
    timed_drops = list(drops)
    probe = ops.PROBE.pop("gemm")
    ar_timing, red.timing = red.timing, None
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    losses = out4.cpu().tolist()
    frames = args.steps * B * T * world
    value = frames / elapsed
    # probe kernel duration from its in-kernel stamps (100 MHz ticks), events beside it
    nl = len(probe["events"])
    st = stamps[:nl].cpu()
    kern_ms = [(int(e) - int(s)) * 1e-5 for s, e in st.tolist()]
    kern_ms_sorted = sorted(kern_ms)
    avg_ms = sum(kern_ms) / max(1, nl)
    med_ms = kern_ms_sorted[nl // 2] if nl else 0.0
    ev_ms = [s.elapsed_time(e) for s, e in probe["events"]]
    ev_avg = sum(ev_ms) / max(1, len(ev_ms))
    flops = 2.0 * M * N_ * K_
    achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    # FLOPs the timed steps performed (video_off steps skip the ResNet backward)
    fpf = sum(model_flops_per_frame(cfg, T, L, d or "none") for d in timed_drops) / max(1, len(timed_drops))
    # HBM bytes per launch from the committed PMC passes of the current GEMM core (tools/pmc_traffic.py
    # via tools/gpu_counters.sh): the newest profiles/r*_pmc_traffic.json
    traffic, traffic_src = None, None
    cands = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc_traffic.json"))
    if cands:
        traffic_src = "profiles/" + cands[-1]
        rec = json.load(open(os.path.join(ROOT, traffic_src)))
        if rec.get("shape") == [M, N_, K_]:
            traffic = rec["traffic_bytes"]

    # per-modality-variant step time (outside the timed region; every rank forced alike)
    # back-to-back steps of one variant, like the timed loop (no synchronisation between them:
    # a synchronised step also pays the pipeline refill); the median of the last three intervals
    variant_ms = {}
    for name, forced in (("none", None), ("audio_off", "audio_off"), ("video_off", "video_off")):
        eng.force_modality = (forced,)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        evs[0].record()
        for j in range(4):
            step(variant=True)
            evs[j + 1].record()
        torch.cuda.synchronize()
        per = [evs[j].elapsed_time(evs[j + 1]) for j in range(1, 4)]
        variant_ms[name] = round(sorted(per)[1], 2)
    eng.force_modality = None
    exp_ms = expected_step_ms(variant_ms, world)
    # what one seeded draw of the reference's RNG would have given for the same K steps
    # (per-variant medians; the timed region itself runs the stratified schedule)
    rs = np.random.RandomState(args.seed + 7919 * rank)
    raw = []
    for _ in range(args.steps):
        pm, pa = rs.random_sample(), rs.random_sample()
        raw.append("none" if pm >= cfg.modality_dropout else ("audio_off" if pa < cfg.audio_dropout else "video_off"))
    raw_ms = sum(variant_ms[k] for k in raw)
    allreduce = None
    if world > 1:
        exposed = [j0.elapsed_time(j1) for (c0, c1, j0, j1) in ar_timing]
        comm = [c0.elapsed_time(c1) for (c0, c1, j0, j1) in ar_timing if c0 is not None]
        allreduce = {"backend": dist.get_backend(), "ranks": dist.get_world_size(),
                     "compress": args.grad_compress or "none (fp32)",
                     "buckets": len(red.buckets) + len(red.tail), "bucket_mib": parallel.BUCKET_BYTES >> 20,
                     "bytes_per_step": arena.grad.numel() * 4,
                     "exposed_ms_per_step": round(sum(exposed) / max(1, len(exposed)), 3),
                     "comm_ms_per_step": round(sum(comm) / max(1, len(comm)), 3),
                     "note": "exposed = compute-stream wait for the comm stream after the backward (rank 0); "
                             "comm = first bucket launch to last completion"}
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "AV-frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "warmup_note": "plus one untimed fwd+bwd per modality variant (none / video_off / audio_off) before the warm-up steps",
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (SURVEY d1 recipe: uint8 lip frames, normal+LN 104-d audio, U[1,5047] labels)",
        "config": {"workload": f"C2/C3: AVHubertAVSR fwd+bwd+AdamW, {B}x{T / 25:.0f}s clips per GPU "
                               f"(T={T}, L={L}), train mode, dropouts on",
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                   "encoder_layers": cfg.num_hidden_layers,
                   "optimizer": "fused clip+AdamW",
                   "modality_draws": ("stratified 0.5/0.25/0.25 (period 4, rotated per rank)" if strat and forced_all is None
                                      else "reference RNG draws" if forced_all is None else "forced")},
        "roofline": {"bound": "mfma", "kernel": f"dense_glds_kernel bf16 (encoder FFN1 fwd {M}x{N_}x{K_})",
                     "achieved": round(achieved, 1), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                     "traffic_unit": f"bytes/launch (rocprofv3 FETCH_SIZEx2+WRITE_SIZE, {traffic_src})",
                     "algorithmic_flops_per_launch": flops, "launches": nl,
                     "avg_launch_ms": round(avg_ms, 4), "median_launch_ms": round(med_ms, 4),
                     "timing": "in-kernel s_memrealtime stamps (first workgroup start -> last workgroup end)",
                     "event_avg_launch_ms": round(ev_avg, 4)},
        "model_tflops_per_s": round(value * fpf / world / 1e12, 1),
        "model_mfu": round(value * fpf / world / 1e12 / BF16_PEAK_TFLOPS, 4),
        "model_flops_note": "algorithmic FLOPs of the steps actually timed (video_off: no ResNet backward)",
        "modality_variants": {"step_ms": variant_ms, "p": MODALITY_P,
                              "expected_ms_per_step": round(exp_ms, 3),
                              "value_expected": round(B * T * world / exp_ms * 1e3, 2),
                              "value_seeded_draw": round(args.steps * B * T * world / raw_ms * 1e3, 2),
                              "seeded_draw_counts": {k: raw.count(k) for k in MODALITY_P},
                              "note": "median of 3 back-to-back forced steps per variant (after one lead-in step); value_expected weights them with "
                                      "the reference's draw probabilities (avhubert.py:476-482), slowest rank "
                                      "bounding a step for N > 1; value_seeded_draw: the same K steps under one "
                                      "numpy draw (seed --seed) instead of the stratified schedule"},
        "loss": [round(x, 4) for x in losses],
        "host_ms_per_step_timed": round(sum(host_t) / len(host_t) * 1e3, 2),
        "host_ms_steps": [round(t * 1e3, 1) for t in host_t],
        "stream_ms_steps": [round(step_ev[i].elapsed_time(step_ev[i + 1]), 1) for i in range(args.steps)],
        "allocator_timed": {k: ms1.get(k, 0) - ms0.get(k, 0) for k in
                            ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams")},
        "modality_drops": {"seed": args.seed, "video_off": timed_drops.count("video_off"),
                           "audio_off": timed_drops.count("audio_off"), "none": timed_drops.count(None),
                           "note": "rank 0's timed steps; video_off skips the ResNet backward "
                                   "(its gradient is exactly zero, avhubert.py:480)"},
        "allreduce": allreduce,
    }
    if forced_all is not None:
        result["forced_modality"] = f"every timed step forced to {args.force_modality} (profiling run, not the metric)"
    if rank == 0 and not args.quick:
        result["frontend"] = frontend_timing(B, T, dev)
        if args.layers is None:
            result["encoder_gemms"] = encoder_gemm_table(dev, B * T, cfg.hidden_size, cfg.intermediate_size)
            result["roofline"]["worst_encoder_gemm"] = result["encoder_gemms"]["worst"]
    threads = min(16, os.cpu_count() or 1)
    if state_cpu is not None:
        fps, dt, clips = cpu_baseline(cfg, state_cpu, T, threads)
        result["cpu_baseline"] = {"value": round(fps, 2), "unit": "AV-frames/s", "cores": threads, "kind": "port",
                                  "sample": f"{clips} x 15 s clips (T={T}, L=40) fwd+bwd one at a time, "
                                            f"oracle/avsr_oracle.py fp32, {dt:.1f} s"}
    if rank == 0 and world == 1 and args.layers is None and not args.quick and not args.no_decode:
        del eng, arena, opt, ddp, model
        gc.collect()
        torch.cuda.empty_cache()
        result["decode"] = decode_throughput(dev, state_cpu, cfg, threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=16, help="clips per GPU")
    ap.add_argument("--seq", type=int, default=375, help="AV-frames per clip (15 s at 25 fps)")
    ap.add_argument("--labels", type=int, default=40)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--modality-draws", choices=["stratified", "random"], default="stratified",
                    help="timed steps' modality variants: stratified to the reference's probabilities (default), "
                         "or drawn from numpy's global RNG per forward as the reference does")
    ap.add_argument("--grad-compress", choices=["bf16"], default=None,
                    help="N > 1: exchange gradients in bf16 (parallel.GradReducer; default fp32 for parity)")
    ap.add_argument("--no-decode", action="store_true", help="skip the C1/C4/C5 decode throughput section")
    ap.add_argument("--quick", action="store_true", help="only the step measurement (profiling runs)")
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer encoder layers (INVALID for the metric)")
    ap.add_argument("--seed", type=int, default=1234, help="seeds the inputs, dropout streams and the "
                    "modality-dropout draws (numpy global RNG, as the reference draws them)")
    ap.add_argument("--force-modality", choices=["none", "audio_off", "video_off"], default=None,
                    help="profiling only: every step uses this modality variant (the value is then not the metric)")
    ap.add_argument("--cpu-selftest", action="store_true", help="no GPU: launcher + gloo all-reduce check only")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:])
    if args.cpu_selftest:
        return cpu_selftest(args)
    return gpu_bench(args)


if __name__ == "__main__":
    sys.exit(main())
