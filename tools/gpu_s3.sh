# validation (tests, smoke, bench, step profile) + encoder GEMM table over tile configs
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh ${1:-s3} || exit 1
bash tools/gpu_gemmtab.sh ${1:-s3}_gt ${2:-128,192,192x256,192s3} || exit 1
echo rc=0
