# Encoder GEMM table under the given tile configurations (tools/gemm_table.py, HIP-graph timed,
# random data). Usage: gpurun -- bash tools/gpu_gemm_sweep.sh TAG cfg,cfg,...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gs}; mkdir -p $O
timeout -k 10 600 python -u tools/gemm_table.py $O/table.json ${2:-auto,192,192w8s3,192w8s4,192x256} > $O/table.txt 2>&1 || { echo table failed; tail -20 $O/table.txt; exit 1; }
cat $O/table.txt
