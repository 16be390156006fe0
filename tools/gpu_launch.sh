set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lb}; mkdir -p $O
timeout -k 10 120 python -u tools/launch_bench.py > $O/lb.log 2>&1 || { echo failed; tail -20 $O/lb.log; exit 1; }
grep " us" $O/lb.log
echo rc=0
