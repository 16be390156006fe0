# interleaved bench A/B of one env switch: bash tools/gpu_ab_env.sh TAG VAR "v1 v2" [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abenv}; mkdir -p $O
for i in $(seq ${4:-2}); do
for v in $3; do
env "$2=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode > $O/b_${v}_$i.log 2>&1 || { echo bench failed; tail -5 $O/b_${v}_$i.log; exit 1; }
echo "$2=$v $(tail -1 $O/b_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
echo rc=0
