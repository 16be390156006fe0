set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ctcs}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_model_parity.py tests/test_gpu_fullsize_golden.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py tests/test_gpu_trainer.py tests/test_gpu_surface.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_env.sh ${1:-ctcs}_ab AVSR_CTC_SIDE "1 0" 3 || exit 1
echo rc=0
