set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-side}; mkdir -p $O
for i in 1 2; do
for s in 1 0; do
AVSR_SIDE_STREAM=$s timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_${s}_$i.log 2>&1 || { echo bench failed; tail -5 $O/b_${s}_$i.log; exit 1; }
echo "side=$s $(tail -1 $O/b_${s}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
echo rc=0
