# gemm tests + encoder GEMM table + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s3b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/gemm_table.py $O/gemm_table.json ${2:-auto,128,192} > $O/gemm_table.txt 2>&1 || { echo table failed; tail -20 $O/gemm_table.txt; exit 1; }
cat $O/gemm_table.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'])"
echo rc=0
