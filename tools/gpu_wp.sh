# conv tests (incl. the patch-resident weight-grad) + isolated ResNet conv kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-wp}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/conv_kbench.py 10 > $O/kb.log 2>&1 || { echo kb failed; tail -20 $O/kb.log; exit 1; }
tail -1 $O/kb.log
echo rc=0
