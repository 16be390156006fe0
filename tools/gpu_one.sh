# one GPU test selection, e.g.: bash tools/gpu_one.sh TAG "tests/test_gpu_fullsize_golden.py -k t375"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-one}; mkdir -p $O
timeout -k 10 400 python -u -m pytest $2 -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo rc=0
