set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gemm2; mkdir -p $O
for T in auto 128 pp 256 128s3 256x128 128x256 128w8s3; do
  AVSR_GEMM_TILE=$T timeout -k 10 120 python tools/bench_gemm.py >> $O/bg.log 2>&1 || exit 1
done
echo rc=0
