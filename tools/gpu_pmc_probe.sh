# HBM PMC passes on the roofline probe GEMM (FFN1 fwd at C2, engine tile choice)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcp}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_fetch -o run --pmc FETCH_SIZE -- python3 tools/gemm_one.py 6000 4096 1024 ffn1 20 > $O/pmc.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_write -o run --pmc WRITE_SIZE -- python3 tools/gemm_one.py 6000 4096 1024 ffn1 20 >> $O/pmc.log 2>&1 || { echo pmc2 failed; exit 1; }
timeout -k 10 60 python tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv 6000 4096 1024 $O/pmc_traffic.json >> $O/pmc.log 2>&1 || { echo pmc_traffic failed; exit 1; }
tail -1 $O/pmc.log
echo rc=0
