# GEMM tests (all tile configs incl. 64x64) + step A/B of the 64x64 small-grid tile.
# Usage: gpurun -- bash tools/gpu_g64.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-g64}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread > $O/gemm.log 2>&1 || { echo gemm tests failed; tail -30 $O/gemm.log; exit 1; }
tail -1 $O/gemm.log
bash tools/gpu_ab4.sh ${1:-g64}ab "AVSR_GEMM_NO64=0" "AVSR_GEMM_NO64=1"
