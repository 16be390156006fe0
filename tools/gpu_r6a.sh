# attention backward (unrolled tile loops): tests, isolated kernel stats, SQ counters.
# Usage: gpurun -- bash tools/gpu_r6a.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6a}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_model_parity.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/attn_bench.py > $O/bench.log 2>&1 || { echo prof failed; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log | grep -v amdgpu.ids
python - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in rows:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us avg  n={int(r['Calls']):5d}  {r['Name'][:110]}")
PY
rm -f $O/prof/run_kernel_trace.csv
PROGS=attn bash tools/gpu_counters.sh $T > $O/counters.log 2>&1 || { echo counters failed; tail -20 $O/counters.log; exit 1; }
grep -A8 "== attn" $O/counters.log
