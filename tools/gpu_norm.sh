# norm/conv tests + isolated ResNet fwd/bwd
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-nrm}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/resnet_bench.py 5 > $O/rn.log 2>&1 || { echo rn failed; tail -20 $O/rn.log; exit 1; }
grep video $O/rn.log
echo rc=0
