set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tg.log 2>&1
for K in fwd dgrad wgrad; do timeout -k 10 100 python tools/conv_one.py $K 6000 22 64 64 3 1 >> gpurun_out/conv.log 2>&1 || exit 1; done
for K in fwd dgrad wgrad; do timeout -k 10 100 python tools/conv_one.py $K 6000 11 128 128 3 1 >> gpurun_out/conv.log 2>&1 || exit 1; done
AVSR_GEMM_TILE=128 timeout -k 10 200 python tools/bench_gemm.py >> gpurun_out/bg.log 2>&1
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1
echo rc=$?
