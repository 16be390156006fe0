# patch-resident stage-1 conv: equivalence tests, ResNet A/B timing, per-kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-patch}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/resnet_bench.py 5 new > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/resnet_bench.py 1 new > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
echo rc=0
