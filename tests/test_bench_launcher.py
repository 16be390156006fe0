"""bench.py's own multi-rank entry point: `python bench.py --gpus N`
without a torch.distributed.run environment spawns N ranks itself (the parent never touches
the GPU), relays rank 0's JSON line and fails when any rank fails. CPU only: --cpu-selftest
runs the launcher, the gloo rendezvous and the bucketed gradient all-reduce
(parallel.GradReducer with readiness watermarks), with a tiny synthetic arena."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


@pytest.mark.parametrize("compress", [None, "bf16"])
def test_bench_self_launch_world2(compress):
    extra = [] if compress is None else ["--grad-compress", compress]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-selftest",
                        "--steps", "2", "--warmup", "1"] + extra, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2
    ar = d["allreduce"]
    assert ar["ranks"] == 2 and ar["backend"] == "gloo" and ar["mean_ok"] is True
    assert ar["buckets"] >= 4
    assert ar["compress"] == (compress or "none (fp32)")


def test_bench_launcher_fails_when_a_rank_fails():
    """rank 1 dies before the rendezvous: rank 0 would wait forever; the launcher must stop
    it and exit non-zero"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-selftest",
                        "--steps", "1", "--warmup", "0"], env=_env(AVSR_BENCH_SELFTEST_FAIL_RANK="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with 7" in r.stderr


def test_expected_step_ms():
    sys.path.insert(0, ROOT)
    import bench
    v = {"none": 55.0, "audio_off": 54.0, "video_off": 39.0}
    assert bench.expected_step_ms(v, 1) == pytest.approx(0.5 * 55 + 0.25 * 54 + 0.25 * 39)
    # two ranks: the step is video_off only if both draw it
    e2 = bench.expected_step_ms(v, 2)
    p_vo, p_le_ao = 0.25 ** 2, 0.5 ** 2
    assert e2 == pytest.approx(39 * p_vo + 54 * (p_le_ao - p_vo) + 55 * (1 - p_le_ao))


def test_stratified_variants_match_reference_probabilities():
    """bench.py's timed steps take the reference's modality distribution stratified: every 4
    consecutive steps hold 2 none, 1 video_off, 1 audio_off, on every rank; ranks are rotated"""
    sys.path.insert(0, ROOT)
    import bench
    for rank in range(3):
        s = bench.stratified_variants(20, rank)
        for i in range(0, 20, 4):
            blk = s[i:i + 4]
            assert blk.count(None) == 2 and blk.count("video_off") == 1 and blk.count("audio_off") == 1
    assert bench.stratified_variants(4, 0) != bench.stratified_variants(4, 1)
