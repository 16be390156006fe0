# the whole -m gpu suite (every failure listed), then the batched-decode diagnostic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/dbg_batch_decode.py > $O/dbg.log 2>&1; rc=$?
grep worst $O/dbg.log
exit $rc
