# full GPU suite, then default bench interleaved A/B against an env setting.
# Usage: gpurun -- bash tools/gpu_ab_env.sh TAG "ENV=VAL"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/benchA$i.log 2>&1 || { echo bench failed; exit 1; }
  echo -n "A: "; tail -1 $O/benchA$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['device_ms_per_step_synced'], d['modality_drops']['video_off'])"
  env $2 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/benchB$i.log 2>&1 || { echo bench B failed; exit 1; }
  echo -n "B ($2): "; tail -1 $O/benchB$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['device_ms_per_step_synced'], d['modality_drops']['video_off'])"
done
echo rc=0
