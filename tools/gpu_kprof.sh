# Per-kernel durations (rocprofv3 --kernel-trace --stats) and two SQ counter passes over one
# microbench command. Usage: gpurun -- bash tools/gpu_kprof.sh TAG "python3 tools/attn_bench.py"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-kprof}; shift; mkdir -p $O
CMD="$1"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $CMD > $O/kt.log 2>&1 || { echo trace failed; tail -5 $O/kt.log; exit 1; }
python3 - $O/kt/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us avg  n={r['Calls']:>5}  {r['Name'][:110]}")
PY
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY"
for pass in A B; do
  if [ $pass = A ]; then P="$PA"; else P="$PB"; fi
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/sq$pass -o run -- $CMD > $O/sq$pass.log 2>&1 || { echo "sq $pass failed"; tail -5 $O/sq$pass.log; exit 1; }
done
timeout -k 10 60 python3 tools/pmc_sum.py $O/sq.json $O/sqA/run_counter_collection.csv $O/sqB/run_counter_collection.csv > $O/sq.txt 2>&1 || { echo sum failed; exit 1; }
head -30 $O/sq.txt
rm -rf $O/sqA $O/sqB
