# encoder GEMM table under several tile configurations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gt}; mkdir -p $O
timeout -k 10 500 python -u tools/gemm_table.py $O/gemm_table.json ${2:-auto,128,192,192s3,192x256,256,256x128,128s3} > $O/gt.log 2>&1 || { echo gt failed; tail -20 $O/gt.log; exit 1; }
cat $O/gt.log | grep -v amdgpu.ids
echo rc=0
