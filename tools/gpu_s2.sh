# stride-2 data-grad parity classes: conv / BN-epilogue tests, ResNet fwd/bwd A/B, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_norm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_model_parity.py -x -q --timeout 240 --timeout-method thread > $O/tests2.log 2>&1 || { echo model tests failed; tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
timeout -k 10 300 python -u tools/resnet_bench.py 7 s2 > $O/rn.log 2>&1 || { echo resnet bench failed; tail -20 $O/rn.log; exit 1; }
cat $O/rn.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/resnet_bench.py 1 s2 > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
echo rc=0
