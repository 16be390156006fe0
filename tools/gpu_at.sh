# attention tests + isolated attention timing. Usage: gpurun -- bash tools/gpu_at.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-at}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > $O/attn.log 2>&1 || { echo attn tests failed; tail -30 $O/attn.log; exit 1; }
tail -1 $O/attn.log
timeout -k 10 120 python -u tools/attn_bench.py > $O/ab.txt 2>&1 || { echo attn bench failed; tail -5 $O/ab.txt; exit 1; }
grep drop $O/ab.txt
echo rc=0
