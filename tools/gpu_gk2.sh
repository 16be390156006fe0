set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gk2}; mkdir -p $O
export DBGS=${2:-0 1 2 3}
for d in ${DBGS:-0 1 2}; do
echo "dbg=$d" >> $O/gemm_k.txt
AVSR_GEMM_DBG=$d AVSR_GEMM_TILE=128 timeout -k 10 200 python -u tools/gemm_k.py 6000 4096 >> $O/gemm_k.txt 2>&1 || { echo failed; tail -20 $O/gemm_k.txt; exit 1; }
done
grep -v amdgpu.ids $O/gemm_k.txt
