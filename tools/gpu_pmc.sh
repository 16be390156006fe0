set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for T in pp; do
  AVSR_GEMM_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$T/a -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -- python tools/gemm_one.py 8192 8192 8192 fwd 5 > gpurun_out/pmc_$T.log 2>&1 || exit 1
  AVSR_GEMM_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$T/b -o run --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM -- python tools/gemm_one.py 8192 8192 8192 fwd 5 >> gpurun_out/pmc_$T.log 2>&1 || exit 1
  AVSR_GEMM_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$T/c -o run --pmc FETCH_SIZE -- python tools/gemm_one.py 8192 8192 8192 fwd 5 >> gpurun_out/pmc_$T.log 2>&1 || exit 1
  AVSR_GEMM_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$T/d -o run --pmc TCC_HIT_sum TCC_MISS_sum -- python tools/gemm_one.py 8192 8192 8192 fwd 5 >> gpurun_out/pmc_$T.log 2>&1 || exit 1
done
echo rc=$?
