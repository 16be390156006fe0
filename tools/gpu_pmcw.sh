set -o pipefail
cd $GRAFT_REPO_ROOT
export PROGS="wgrad"
bash tools/gpu_pmc.sh ${1:-pmcw} || exit 1
timeout -k 10 60 python tools/pmc_sum.py gpurun_out/${1:-pmcw}/pmc_sq.json gpurun_out/${1:-pmcw}/*/run_counter_collection.csv > gpurun_out/${1:-pmcw}/sum.log 2>&1 || { echo sum failed; tail -5 gpurun_out/${1:-pmcw}/sum.log; exit 1; }
cat gpurun_out/${1:-pmcw}/sum.log
echo rc=0
