# side-stream CU-mask A/B (AVSR_SIDE_CUS = k/n of the CUs for the weight-gradient stream):
# gpu tests of the masked stream first, then bench passes alternating the masks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cum}; mkdir -p $O
AVSR_SIDE_CUS=1/2 timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_trainer.py tests/test_gpu_opt_overlap.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for m in none 3/4 1/2 7/8; do
    t=$(echo $m | tr / _)
    if [ $m = none ]; then unset AVSR_SIDE_CUS; else export AVSR_SIDE_CUS=$m; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode > $O/b_${t}_$r.log 2>&1 || { echo bench $m failed; tail -20 $O/b_${t}_$r.log; exit 1; }
    tail -1 $O/b_${t}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d['modality_variants']['step_ms'], d['modality_variants']['value_expected'])"
  done
done
unset AVSR_SIDE_CUS
echo rc=0
