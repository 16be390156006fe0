# GEMM parity (weight-grad / layouts) + the encoder GEMM table at the default tile choice.
# Usage: gpurun -- bash tools/gpu_gt.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gt}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -k "wgrad_dual or layouts_bf16" -x -q --timeout 120 --timeout-method thread > $O/gemm.log 2>&1 || { echo gemm tests failed; tail -30 $O/gemm.log; exit 1; }
tail -1 $O/gemm.log
timeout -k 10 300 python -u tools/gemm_table.py $O/table.json auto > $O/table.txt 2>&1 || { echo table failed; tail -20 $O/table.txt; exit 1; }
cat $O/table.txt
echo rc=0
