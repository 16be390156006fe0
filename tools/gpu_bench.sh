# the default bench line. Usage: gpurun -- bash tools/gpu_bench.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-bx}; mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['modality_variants']['value_expected'], d['modality_variants']['step_ms'])"
echo rc=0
