# SQ counter passes (MFMA busy, VALU / LDS / VMEM issue, waits, LDS conflicts) over the attention,
# ResNet and GEMM microbenches. Usage: gpurun -- bash tools/gpu_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}; mkdir -p $O
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY"
for prog in ${PROGS:-attn resnet gemm}; do
  case $prog in
    attn) CMD="python3 tools/attn_bench.py";;
    resnet) CMD="python3 tools/resnet_bench.py 1";;
    gemm) CMD="python3 tools/gemm_sq.py ${GEMM_CFGS:-128}";;
    wgrad) CMD="python3 tools/wgrad_kb.py";;
    stem) CMD="python3 tools/stem_kbench.py 5";;
  esac
  for pass in A B; do
    if [ $pass = A ]; then P="$PA"; else P="$PB"; fi
    timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/$prog$pass -o run -- $CMD > $O/$prog$pass.log 2>&1 || { echo "$prog $pass failed"; tail -5 $O/$prog$pass.log; exit 1; }
  done
done
echo rc=0
