# per-encoder-layer gating of the overlapped update: tests, then in-step A/B. Usage: gpurun -- bash tools/gpu_r6g.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_opt_overlap.py tests/test_gpu_cfgvar.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS="1 2" bash tools/gpu_abx.sh ${1:-r6g}/ab "base|-" "base|OPT_LAYER_GATE=0" "base|OPT_OVERLAP_BLOCKS=64" "base|OPT_OVERLAP_BLOCKS=96"
