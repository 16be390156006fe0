set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_gemm.py -x -q > gpurun_out/tg.log 2>&1
for T in pp 128; do AVSR_GEMM_TILE=$T timeout -k 10 200 python tools/bench_gemm.py big >> gpurun_out/bg.log 2>&1 || exit 1; done
echo rc=$?
