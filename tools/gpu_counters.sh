# Counter evidence at HEAD (verdict r4 item 1): HBM traffic of the roofline probe (FETCH_SIZE /
# WRITE_SIZE passes), the probe's per-launch durations, and two SQ passes over the isolated
# microbenches of the named kernels and over two video-on training steps.
# Usage: gpurun -- bash tools/gpu_counters.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cnt}; mkdir -p $O
PROBE="python3 tools/gemm_one.py 6000 4096 1024 ffn1 20"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_fetch -o run --pmc FETCH_SIZE -- $PROBE > $O/pmc.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_write -o run --pmc WRITE_SIZE -- $PROBE >> $O/pmc.log 2>&1 || { echo write failed; exit 1; }
timeout -k 10 60 python tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv 6000 4096 1024 $O/pmc_traffic.json >> $O/pmc.log 2>&1 || { echo pmc_traffic failed; exit 1; }
echo "traffic: $(tail -1 $O/pmc.log)"
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY"
for prog in ${PROGS:-probe wgrad attn stem cwgrad step}; do
  case $prog in
    probe) CMD="$PROBE";;
    wgrad) CMD="python3 tools/gemm_one.py 4096 1024 6000 wgrad 20";;
    attn) CMD="python3 tools/attn_bench.py";;
    stem) CMD="python3 tools/stem_kbench.py 5";;
    stemw) CMD="python3 tools/stem_wgrad_kbench.py 3";;
    cwgrad) CMD="python3 tools/wgrad_kb.py";;
    step) CMD="python3 bench.py --steps 2 --warmup 1 --quick --no-cpu-baseline --force-modality none";;
  esac
  for pass in A B; do
    if [ $pass = A ]; then P="$PA"; else P="$PB"; fi
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/$prog$pass -o run -- $CMD > $O/$prog$pass.log 2>&1 || { echo "$prog $pass failed"; tail -5 $O/$prog$pass.log; exit 1; }
  done
  timeout -k 10 60 python tools/pmc_sum.py $O/sq_$prog.json $O/${prog}A/run_counter_collection.csv $O/${prog}B/run_counter_collection.csv > $O/sq_$prog.txt 2>&1 || { echo "sum $prog failed"; exit 1; }
  echo "== $prog"; head -12 $O/sq_$prog.txt
  [ $prog = step ] && rm -rf $O/${prog}A $O/${prog}B     # the per-dispatch step CSVs exceed what gpurun copies back
done
echo rc=0
