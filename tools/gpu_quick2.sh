# conv tests + model parity, wgrad split sweep, bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/q2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python -u tools/wgrad_sweep.py 5 > $O/wgrad.log 2>&1 || { echo sweep failed; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 $O/bench.log
echo rc=0
