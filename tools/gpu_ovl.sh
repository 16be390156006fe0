# optimizer-overlap A/B on one box: new parity test, the trainer / DP tests, then bench with
# and without the overlap (twice each, alternating) and a short kernel trace of the overlapped run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ovl}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_opt_overlap.py tests/test_gpu_trainer.py tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode --opt-overlap > $O/ovl_$r.log 2>&1 || { echo bench ovl failed; tail -20 $O/ovl_$r.log; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode > $O/ser_$r.log 2>&1 || { echo bench ser failed; tail -20 $O/ser_$r.log; exit 1; }
  for f in ovl_$r ser_$r; do tail -1 $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['modality_variants']['step_ms'], d['modality_variants']['value_expected'])"; done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-decode --quick > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
echo rc=0
