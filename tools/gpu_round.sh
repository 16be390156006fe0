# Full GPU cycle: parity tests, smoke, bench (with CPU baseline), rocprof kernel stats,
# HBM PMC passes on the roofline probe GEMM. Usage: gpurun -- bash tools/gpu_round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 60 python tools/probe_trace.py $O/prof/run_kernel_trace.csv > $O/probe.txt 2>&1 || { echo probe failed; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_fetch -o run --pmc FETCH_SIZE -- python3 tools/gemm_one.py 6000 4096 1024 ffn1 20 > $O/pmc.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_write -o run --pmc WRITE_SIZE -- python3 tools/gemm_one.py 6000 4096 1024 ffn1 20 >> $O/pmc.log 2>&1 || { echo pmc2 failed; exit 1; }
timeout -k 10 60 python tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv 6000 4096 1024 $O/pmc_traffic.json >> $O/pmc.log 2>&1 || { echo pmc_traffic failed; exit 1; }
echo rc=0
