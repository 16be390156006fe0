set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ctc3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss_misc.py tests/test_gpu_model_parity.py tests/test_gpu_fullsize.py -x -q -s --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo tests failed; grep -a "Error\|assert" $O/t.log | head; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
tail -1 $O/t.log; grep -a "parity (" $O/t.log; grep ctc_fwd $O/prof/run_kernel_stats.csv | cut -c1-120
echo rc=0
