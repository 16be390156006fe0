set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_gemm.py -x -q > gpurun_out/tg.log 2>&1 && \
timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/bg.log 2>&1 && \
AVSR_GEMM_NOGLDS=1 timeout -k 10 200 python tools/bench_gemm.py >> gpurun_out/bg.log 2>&1
echo rc=$?
