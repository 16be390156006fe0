set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-long}; mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["modality_drops"], d["roofline"]["frac"])'
echo rc=0
