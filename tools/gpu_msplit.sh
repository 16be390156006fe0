set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ms}; mkdir -p $O
timeout -k 10 300 python -u tools/msplit_bench.py > $O/ms.log 2>&1 || { echo failed; tail -20 $O/ms.log; exit 1; }
cat $O/ms.log
