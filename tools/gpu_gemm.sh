set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tg.log 2>&1
for T in 128 pp; do AVSR_GEMM_TILE=$T timeout -k 10 200 python tools/bench_gemm.py big >> gpurun_out/bg.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1
echo rc=$?
