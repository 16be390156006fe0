# GPU tests (engine paths) then an in-box A/B of env settings on the bench.
# usage: gpurun -- bash tools/gpu_abt.sh TAG "ENV=a" "ENV=b" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abt}; shift; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_colsum.py tests/test_gpu_gemm.py tests/test_gpu_norm.py tests/test_gpu_model_parity.py tests/test_gpu_trainer.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/x.log 2>&1 || { echo "bench failed"; tail -20 $O/x.log; exit 1; }
  tail -1 $O/x.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'], d['stream_ms_steps'])"
done
