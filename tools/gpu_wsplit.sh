# encoder GEMM table with different weight-gradient split-K choices
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ws}; mkdir -p $O
for sp in default 1 2 4 16; do
  if [ $sp = default ]; then unset AVSR_WGRAD_SPLIT; else export AVSR_WGRAD_SPLIT=$sp; fi
  timeout -k 10 200 python -u tools/gemm_table.py $O/t_$sp.json auto > $O/t_$sp.log 2>&1 || { echo failed $sp; tail -5 $O/t_$sp.log; exit 1; }
  echo "split $sp:"; grep wgrad $O/t_$sp.log
done
echo rc=0
