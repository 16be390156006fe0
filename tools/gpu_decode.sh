# decode tests + decode throughput. Usage: gpurun -- bash tools/gpu_decode.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dec}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize_golden.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo tests failed; tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u tools/decode_bench.py 8 100 3 float32 > $O/d.log 2>&1 || { echo decode bench failed; tail $O/d.log; exit 1; }
timeout -k 10 300 python -u tools/decode_bench.py 8 375 5 bfloat16 >> $O/d.log 2>&1 || { echo decode bench2 failed; tail $O/d.log; exit 1; }
cat $O/d.log
echo rc=0
