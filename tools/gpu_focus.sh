# focused GPU tests (-k / files in $TESTS) + bench + per-kernel step profile.
# Usage: gpurun -- bash tools/gpu_focus.sh TAG "tests/test_a.py tests/test_b.py"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-focus}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${2:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/attn_bench.py > $O/attn.log 2>&1 && grep drop $O/attn.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 60 python tools/profsum.py $O/prof/run_kernel_trace.csv 3 45 > $O/steps.txt 2>&1 || { echo profsum failed; exit 1; }
echo rc=0
