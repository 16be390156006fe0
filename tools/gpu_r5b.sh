# GEMM tests (main-loop change), batched-vs-single decode diagnostic, then the GEMM tile sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py tests/test_gpu_fullsize_golden.py -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/dbg_batch_decode.py > $O/dbg.log 2>&1; rc=$?
tail -20 $O/dbg.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_gemm_sweep.sh ${1:-r5b} auto,192,192w8s3,192w8s4,192x256,128
