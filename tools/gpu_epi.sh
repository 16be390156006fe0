set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-epi}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_model_parity.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/epi_bench.py > $O/epi.log 2>&1 || { echo failed; tail -20 $O/epi.log; exit 1; }
cat $O/epi.log
