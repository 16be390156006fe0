# stem conv: the direct-conv and model tests, isolated kernel timing, bench, step profile.
# Usage: gpurun -- bash tools/gpu_stemc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-stemc}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_norm.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/stem_kbench.py 20 > $O/kb.txt 2>&1 || { echo kb failed; tail $O/kb.txt; exit 1; }
cat $O/kb.txt
timeout -k 10 120 python -u tools/stem_apply_kbench.py > $O/kba.txt 2>&1 || { echo kba failed; tail $O/kba.txt; exit 1; }
cat $O/kba.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --quick --no-cpu-baseline > $O/bench_$r.log 2>&1 || { echo bench failed; tail -20 $O/bench_$r.log; exit 1; }
  echo "run=$r $(tail -1 $O/bench_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); v=d['modality_variants']; print(d['value'], d['ms_per_step'], v['step_ms'], v['value_expected'])")"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --quick --no-cpu-baseline --force-modality none > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
timeout -k 10 60 python tools/profsum.py $O/prof/run_kernel_trace.csv 4 60 --skip 12 > $O/steps.txt 2>&1 || { echo profsum failed; exit 1; }
grep -i "stem_" $O/steps.txt
rm -rf $O/prof/*/ 2>/dev/null
PROGS=stem bash tools/gpu_pmc.sh ${1:-stemc}/pmc || exit 1
timeout -k 10 60 python tools/pmc_sum.py $O/pmc/pmc_sq.json $O/pmc/*/run_counter_collection.csv > $O/pmc_sum.log 2>&1 || { echo sum failed; tail -5 $O/pmc_sum.log; exit 1; }
grep stem_conv $O/pmc_sum.log
echo rc=0
