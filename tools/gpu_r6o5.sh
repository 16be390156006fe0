# encoder side-batch orders (engine.SIDE_ORDER): engine tests, then in-step A/B. Usage: gpurun -- bash tools/gpu_r6o5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6o5}; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_fullsize_golden.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $O/tests.log
REPS="1 2" bash tools/gpu_abx.sh ${1:-r6o5}/ab "base|-" "base|SIDE_ORDER=${V1:-o.c.f2.f1.q}" "base|SIDE_ORDER=${V2:-o.f2.f1.q.c}"
