set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lw; mkdir -p $O
for T in auto 128 pp 128w8s3; do
  if [ $T = auto ]; then E=""; else E="AVSR_GEMM_TILE=$T"; fi
  env $E timeout -k 10 200 python -u tools/lin_wgrad_sweep.py >> $O/lw.log 2>&1 || { echo lw $T failed; exit 1; }
done
echo rc=0
