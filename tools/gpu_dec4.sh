# decode parity (unit + full-size goldens), C1 / C4 / C5 throughput (split on / off), C5 profile.
# Usage: gpurun -- bash tools/gpu_dec4.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dec4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -k "skinny or wgrad_dual or layouts_bf16" -x -q --timeout 120 --timeout-method thread > $O/gemm.log 2>&1 || { echo gemm tests failed; tail -30 $O/gemm.log; exit 1; }
tail -1 $O/gemm.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize_golden.py tests/test_gpu_surface.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1; do
  timeout -k 10 300 python -u tools/decode_bench.py > $O/dec_nosplit_$r.json 2> $O/dec.err || { echo dec failed; tail -20 $O/dec.err; exit 1; }
  echo nosplit; cat $O/dec_nosplit_$r.json
  timeout -k 10 300 python -u tools/decode_bench.py split > $O/dec_split_$r.json 2> $O/dec.err || { echo dec failed; tail -20 $O/dec.err; exit 1; }
  echo split; cat $O/dec_split_$r.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/decode_c5.py split > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
grep C5 $O/prof.log
rm -f $O/p/run_kernel_trace.csv
echo rc=0
