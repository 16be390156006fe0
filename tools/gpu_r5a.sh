# Round 5 first GPU call: the GPU tests touched by the option / workspace changes, then the
# counter passes (tools/gpu_counters.sh). A test failure (rc 1) does not stop the counters; a
# timeout, abort or crash does.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_surface.py tests/test_gpu_gemm.py \
  tests/test_gpu_attention.py tests/test_gpu_conv.py tests/test_gpu_norm.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/gpu_counters.sh ${1:-r5a}
