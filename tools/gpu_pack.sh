set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pack}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss_misc.py tests/test_gpu_model_parity.py tests/test_gpu_norm.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_rnprof.sh ${1:-pack}_rn || exit 1
echo rc=0
