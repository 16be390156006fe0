# ResNet frontend isolated at C2 (round 4): fwd / bwd medians with the side stream (engine
# default) and without (every kernel alone), plus a kernel trace of the side-stream-off run.
# Usage: gpurun -- bash tools/gpu_rn4.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rn4}; mkdir -p $O
timeout -k 10 300 python -u tools/resnet_bench.py 5 > $O/rn_side.log 2>&1 || { echo rn failed; tail -20 $O/rn_side.log; exit 1; }
grep video $O/rn_side.log
AVSR_SIDE_STREAM=0 timeout -k 10 300 python -u tools/resnet_bench.py 5 > $O/rn_noside.log 2>&1 || { echo rn2 failed; tail -20 $O/rn_noside.log; exit 1; }
grep video $O/rn_noside.log
AVSR_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn -o run -- python3 tools/resnet_bench.py 1 > $O/rn.log 2>&1 || { echo rnprof failed; tail -20 $O/rn.log; exit 1; }
rm -rf $O/rn/*/ 2>/dev/null
echo rc=0
