# attention tests + micro-bench: gpurun -- bash tools/gpu_t2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-t2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py -q -x -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py > $O/attn.log 2>&1 || { cat $O/attn.log; exit 1; }
cat $O/attn.log
