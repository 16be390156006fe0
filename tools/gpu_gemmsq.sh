set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gsq}; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_sq.py ${2:-128,pp,256} > $O/sq.log 2>&1 || { echo failed; tail -20 $O/sq.log; exit 1; }
cat $O/sq.log
