set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gk}; mkdir -p $O
for c in 128 192; do
AVSR_GEMM_TILE=$c timeout -k 10 200 python -u tools/gemm_k.py 6000 4096 >> $O/gemm_k.txt 2>&1 || { echo failed; tail -20 $O/gemm_k.txt; exit 1; }
done
cat $O/gemm_k.txt
