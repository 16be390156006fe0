set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-prio}; mkdir -p $O
for i in 1 2; do
for p in 0 1; do
AVSR_MAIN_PRIO=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_$p_$i.log 2>&1 || { echo bench failed; tail -5 $O/b_$p_$i.log; exit 1; }
echo "prio=$p $(tail -1 $O/b_$p_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stream_ms_steps"])')"
done
done
echo rc=0
