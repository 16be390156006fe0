set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for K in fwd dgrad wgrad; do timeout -k 10 100 python tools/conv_one.py $K 6000 22 64 64 3 1 >> gpurun_out/conv.log 2>&1 || exit 1; done
for K in fwd dgrad wgrad; do timeout -k 10 100 python tools/conv_one.py $K 6000 11 128 128 3 1 >> gpurun_out/conv.log 2>&1 || exit 1; done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_conv/a -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES -- python tools/conv_one.py fwd 6000 22 64 64 3 1 5 > gpurun_out/pmc_conv.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_conv/b -o run --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM -- python tools/conv_one.py fwd 6000 22 64 64 3 1 5 >> gpurun_out/pmc_conv.log 2>&1 || exit 1
echo rc=$?
