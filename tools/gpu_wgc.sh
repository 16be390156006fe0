set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wgc}; mkdir -p $O
timeout -k 10 300 python -u tools/wgrad_cmp.py > $O/wgrad_cmp.txt 2>&1 || { echo failed; tail -20 $O/wgrad_cmp.txt; exit 1; }
cat $O/wgrad_cmp.txt
