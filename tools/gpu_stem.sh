set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-stem}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_rnprof.sh ${1:-stem}_rn || exit 1
echo rc=0
