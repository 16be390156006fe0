# A/B of env settings on the full bench (default vs each "NAME=VALUE" argument), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
run() {  # label, env assignment
  env $2 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/$1.log 2>&1 || { echo "$1 failed"; tail -20 $O/$1.log; exit 1; }
  tail -1 $O/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', '$2', d['value'], d['ms_per_step'], d['host_ms_per_step_timed'], d['device_ms_per_step_synced'], d['host_issue_ms_per_step'])"
}
run base AVSR_NOP=1
i=0
for a in "$@"; do i=$((i+1)); run v$i "$a"; done
run base2 AVSR_NOP=1
