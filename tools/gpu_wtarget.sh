set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wt}; mkdir -p $O
for i in 1 2; do
for t in ${2:-512 256 1024}; do
env "${3:-AVSR_WGRAD_TARGET}=$t" timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_${t}_$i.log 2>&1 || { echo bench failed; tail -5 $O/b_${t}_$i.log; exit 1; }
echo "target=$t $(tail -1 $O/b_${t}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
echo rc=0
