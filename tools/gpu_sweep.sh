# Tile / split sweeps: conv weight-gradient split-K and dense GEMM tile configurations.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep; mkdir -p $O
timeout -k 10 300 python -u tools/wgrad_sweep.py 5 > $O/wgrad.log 2>&1 || { echo wgrad sweep failed; exit 1; }
for T in auto 128 256x128 128x256 pp 128s3 128w8s3; do
  if [ $T = auto ]; then E=""; else E="AVSR_GEMM_TILE=$T"; fi
  env $E timeout -k 10 120 python -u tools/bench_gemm.py >> $O/gemm.log 2>&1 || { echo gemm $T failed; exit 1; }
done
echo rc=0
