# persistent weight-gradient blocks (AVSR_AB_WGRAD_CAP builds): GEMM / engine tests on the default and the
# capped library, then interleaved in-step A/B. Usage: gpurun -- bash tools/gpu_r6w.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6w}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_model_parity.py tests/test_gpu_c2_batch.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AVSR_LIB_PATH_AB=ab/wcap128/libavsr_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_c2_batch.py > $O/tests_cap.log 2>&1 || { echo cap tests failed; tail -40 $O/tests_cap.log; exit 1; }
tail -1 $O/tests_cap.log
REPS="1 2" bash tools/gpu_abx.sh ${1:-r6w}/ab "base|-" "wcap128|-" "wcap192|-"
