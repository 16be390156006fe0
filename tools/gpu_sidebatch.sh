# batched side-stream handoffs (AVSR_SIDE_BATCH=1, default) vs one event per weight-gradient (=0):
# full GPU suite first, then alternating bench passes and a kernel trace of the batched run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sb}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for m in 1 0; do
    AVSR_SIDE_BATCH=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode > $O/b_${m}_$r.log 2>&1 || { echo bench $m failed; tail -20 $O/b_${m}_$r.log; exit 1; }
    tail -1 $O/b_${m}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch=$m', d['value'], d['ms_per_step'], d['modality_variants']['step_ms'], d['modality_variants']['value_expected'])"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-decode > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 60 python tools/profsum.py $O/prof/run_kernel_trace.csv 3 40 --skip 9 > $O/steps.txt 2>&1 || { echo profsum failed; exit 1; }
echo rc=0
