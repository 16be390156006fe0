# rocprof kernel trace of the isolated ResNet fwd/bwd (tools/resnet_bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rnp}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn -o run -- python3 tools/resnet_bench.py 3 > $O/rn.log 2>&1 || { echo rn failed; tail -20 $O/rn.log; exit 1; }
grep video $O/rn.log
echo rc=0
