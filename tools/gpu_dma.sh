# kernel tests touching the LDS-DMA loaders + isolated conv kernels + encoder GEMM table
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dma}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gemm.py tests/test_gpu_norm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/conv_kbench.py 10 > $O/kb.log 2>&1 || { echo kb failed; tail -20 $O/kb.log; exit 1; }
tail -1 $O/kb.log
timeout -k 10 300 python -u tools/gemm_table.py $O/gemm_table.json auto > $O/gt.log 2>&1 || { echo gt failed; tail -20 $O/gt.log; exit 1; }
tail -14 $O/gt.log
echo rc=0
