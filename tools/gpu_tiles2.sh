set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t2; mkdir -p $O
for T in auto 256x128w4 256x128w4s3 128x256w4; do
  if [ $T = auto ]; then E=""; else E="AVSR_GEMM_TILE=$T"; fi
  env $E timeout -k 10 120 python -u tools/bench_gemm.py >> $O/gemm.log 2>&1 || { echo gemm $T failed; exit 1; }
done
echo rc=0
