set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py -x -q > gpurun_out/tg.log 2>&1
timeout -k 10 300 python -m pytest tests/test_gpu_decode.py -x -q > gpurun_out/td.log 2>&1
for T in 128 256x128 256; do AVSR_GEMM_TILE=$T timeout -k 10 200 python tools/bench_gemm.py >> gpurun_out/bg.log 2>&1 || exit 1; done
timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1
AVSR_CONV_NOGLDS=1 timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline >> gpurun_out/b.log 2>&1
echo rc=$?
