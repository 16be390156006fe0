# capped-grid dropout-mask kernel and the folded gradient clear: tests, then in-step A/B.
# Usage: gpurun -- bash tools/gpu_r6q5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6q5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_attention.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
REPS="1 2 3" bash tools/gpu_abx.sh ${1:-r6q5}/ab "base|-" "maskfull|-" "base|OPT_CLEAR_IN_UPDATE=0"
