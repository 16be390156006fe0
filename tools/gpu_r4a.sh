# round-4 validation: changed tests first, whole GPU suite, smoke, bench, decode split A/B,
# step profile. Usage: gpurun -- bash tools/gpu_r4a.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4a}; mkdir -p $O
export AVSR_REPORT_DIR=$O/report
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_gemm.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread > $O/new.log 2>&1 || { echo new tests failed; tail -30 $O/new.log; exit 1; }
tail -1 $O/new.log
for v in 1 0; do AVSR_ATTN_SQ=$v timeout -k 10 120 python -u tools/attn_bench.py > $O/attn_sq$v.txt 2>&1 || { echo attn bench failed; exit 1; }; echo sq=$v; cat $O/attn_sq$v.txt; done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['modality_variants']['value_expected'], d['roofline']['frac'])"
for r in 1 2; do
  timeout -k 10 300 python -u tools/decode_bench.py split > $O/dec_split_$r.json 2> $O/dec.err || { echo dec failed; tail -20 $O/dec.err; exit 1; }
  timeout -k 10 300 python -u tools/decode_bench.py > $O/dec_nosplit_$r.json 2> $O/dec.err || { echo dec failed; tail -20 $O/dec.err; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dp -o run -- python3 tools/decode_c5.py split > $O/dprof.log 2>&1 || { echo dprof failed; tail -20 $O/dprof.log; exit 1; }
rm -f $O/dp/run_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --quick --no-cpu-baseline --force-modality none > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
timeout -k 10 60 python tools/profsum.py $O/prof/run_kernel_trace.csv 4 60 --skip 12 > $O/steps.txt 2>&1 || { echo profsum failed; exit 1; }
rm -rf $O/prof/*/ 2>/dev/null
echo rc=0
