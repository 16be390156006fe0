# attention parity tests + microbench (+ rocprof split). Usage: gpurun -- bash tools/gpu_attnt.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-at}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model_parity.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo tests failed; tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 120 python -u tools/attn_bench.py > $O/a.log 2>&1 || { echo attn bench failed; exit 1; }
AVSR_DKDV_WAVES=12 timeout -k 10 120 python -u tools/attn_bench.py >> $O/a.log 2>&1 || { echo attn bench12 failed; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/attn_bench.py > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
cat $O/a.log
echo rc=0
