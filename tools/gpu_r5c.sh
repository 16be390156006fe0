# tests of the changed kernels, GEMM table, then a short bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py tests/test_gpu_norm.py tests/test_gpu_decode.py -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_gemm_sweep.sh ${1:-r5c} auto,192,192w8s3,192x256,128 || exit 1
timeout -k 10 400 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-decode > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['modality_variants']['step_ms'], d['modality_variants']['value_expected'])"
