# per-shape encoder GEMM table. Usage: gpurun -- bash tools/gpu_gemmtab.sh TAG [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gt}; mkdir -p $O
timeout -k 10 600 python -u tools/gemm_table.py $O/gemm_table.json ${2:-auto,128,128s3,256x128,128x256,pp} > $O/gemm_table.txt 2>&1 || { echo table failed; tail -20 $O/gemm_table.txt; exit 1; }
cat $O/gemm_table.txt
echo rc=0
