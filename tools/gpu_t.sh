# Given GPU test files only (fast feedback): gpurun -- bash tools/gpu_t.sh TAG tests/test_x.py ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-t}; shift; mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -40
exit $rc
