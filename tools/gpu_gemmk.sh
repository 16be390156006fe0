set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gemmk; mkdir -p $O
for T in 128 pp 256x128; do
  AVSR_GEMM_TILE=$T timeout -k 10 120 python tools/gemm_k.py 6000 4096 >> $O/k.log 2>&1 || exit 1
done
echo rc=0
