# attention tests + microbench, then bench twice: default and with the weight-gradient side
# stream off (host / allocator diagnostics)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-b2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model_parity.py tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/attn_bench.py > $O/attn.log 2>&1 || { echo attn bench failed; exit 1; }
grep drop $O/attn.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/benchA.log 2>&1 || { echo bench failed; tail -20 $O/benchA.log; exit 1; }
AVSR_SIDE_STREAM=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/benchB.log 2>&1 || { echo bench B failed; exit 1; }
for f in A B; do tail -1 $O/bench$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], 'host', d['host_ms_per_step_timed'], d['host_issue_ms_per_step'], 'dev', d['device_ms_per_step_synced'], d['allocator_timed'], d['modality_drops']['video_off'])"; done
echo rc=0
