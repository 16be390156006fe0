set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-st}; mkdir -p $O
timeout -k 10 120 python -u tools/attn_stamps.py $O/stamps.json > $O/stamps.log 2>&1 || { echo stamps failed; tail -20 $O/stamps.log; exit 1; }
grep drop $O/stamps.log
echo rc=0
