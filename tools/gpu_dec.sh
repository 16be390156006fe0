# GEMM + decode parity tests, then decode throughput (C1 / C4 / C5) with the few-row GEMM K split
# on and off (tools/decode_bench.py split)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dec}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_decode.py tests/test_gpu_fullsize_golden.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/decode_bench.py split > $O/dec_split_$r.json 2> $O/dec.err || { echo dec failed; tail -20 $O/dec.err; exit 1; }
  echo split; cat $O/dec_split_$r.json
  timeout -k 10 300 python -u tools/decode_bench.py > $O/dec_nosplit_$r.json 2> $O/dec.err || { echo dec failed; tail -20 $O/dec.err; exit 1; }
  echo nosplit; cat $O/dec_nosplit_$r.json
done
echo rc=0
