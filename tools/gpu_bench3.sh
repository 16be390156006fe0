# model parity tests + three default bench runs (box noise). Usage: gpurun -- bash tools/gpu_bench3.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-b3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_model_parity.py tests/test_gpu_fullsize_golden.py tests/test_gpu_surface.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.log 2>&1 || { echo bench failed; exit 1; }
  tail -1 $O/bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['device_ms_per_step_synced'], d['modality_drops']['video_off'])"
done
echo rc=0
