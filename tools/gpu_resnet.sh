# ResNet fwd/bwd A/B (fused BN-backward reductions vs separate) + kernel trace of it.
# Usage: gpurun -- bash tools/gpu_resnet.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rn}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/resnet_bench.py 7 > $O/rn.log 2>&1 || { echo resnet bench failed; tail -20 $O/rn.log; exit 1; }
cat $O/rn.log
AVSR_SIDE_STREAM=0 timeout -k 10 300 python -u tools/resnet_bench.py 5 > $O/rn_noside.log 2>&1 || { echo resnet bench2 failed; exit 1; }
echo no-side-stream:; grep fuse $O/rn_noside.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/resnet_bench.py 1 > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
echo rc=0
