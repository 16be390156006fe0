# attention tests + microbench + model parity + bench (dropout-hash change)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/at2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model_parity.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
timeout -k 10 120 python -u tools/attn_bench.py > $O/a.log 2>&1 || { echo attn bench failed; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/b.log 2>&1 || { echo bench failed; exit 1; }
tail -2 $O/t.log; cat $O/a.log; grep -o '"ms_per_step": [0-9.]*' $O/b.log
echo rc=0
