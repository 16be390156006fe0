set -o pipefail
cd $GRAFT_REPO_ROOT
export PROGS="attn gemm" GEMM_CFGS="128,192"
bash tools/gpu_pmc.sh ${1:-pmc2} || exit 1
timeout -k 10 60 python tools/pmc_sum.py gpurun_out/${1:-pmc2}/pmc_sq.json gpurun_out/${1:-pmc2}/*/run_counter_collection.csv > gpurun_out/${1:-pmc2}/sum.log 2>&1 || { echo sum failed; tail -5 gpurun_out/${1:-pmc2}/sum.log; exit 1; }
echo rc=0
