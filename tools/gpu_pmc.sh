set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for T in 256 256x128; do
  AVSR_GEMM_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$T/a -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -- python tools/gemm_one.py 6000 4096 1024 fwd 10 > gpurun_out/pmc_$T.log 2>&1 || exit 1
  AVSR_GEMM_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$T/b -o run --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU -- python tools/gemm_one.py 6000 4096 1024 fwd 10 >> gpurun_out/pmc_$T.log 2>&1 || exit 1
done
AVSR_GEMM_TILE=128 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_128/c -o run --pmc FETCH_SIZE -- python tools/gemm_one.py 6000 4096 1024 fwd 10 >> gpurun_out/pmc_128.log 2>&1 || exit 1
AVSR_GEMM_TILE=128 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_128/d -o run --pmc TCC_HIT_sum TCC_MISS_sum -- python tools/gemm_one.py 6000 4096 1024 fwd 10 >> gpurun_out/pmc_128.log 2>&1 || exit 1
echo rc=$?
