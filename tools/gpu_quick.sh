# Quick GPU check: GEMM/conv parity tests + K-sweep of the auto tile. Usage: gpurun -- bash tools/gpu_quick.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-q}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python -u tools/gemm_k.py 6000 4096 > $O/k.log 2>&1 || { echo gemmk failed; exit 1; }
timeout -k 10 120 python -u tools/bench_gemm.py > $O/bg.log 2>&1 || { echo bench_gemm failed; exit 1; }
cat $O/tests.log | tail -2; cat $O/k.log $O/bg.log
echo rc=0
