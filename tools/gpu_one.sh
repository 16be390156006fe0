# one GPU pytest selection: gpurun -- bash tools/gpu_one.sh TAG pytest-args...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/one.log 2>&1; rc=$?
grep -E "^E |PASSED|FAILED" $O/one.log | head -40
exit $rc
