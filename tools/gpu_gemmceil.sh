# library-GEMM ceiling on the encoder shapes + our per-shape table (auto tiles)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gc}
mkdir -p $O
timeout -k 10 300 python -u tools/blas_ref.py $O/blas_ref.json > $O/blas.log 2>&1 || { echo blas failed; tail -20 $O/blas.log; exit 1; }
timeout -k 10 300 python -u tools/gemm_table.py $O/gemm_table.json auto > $O/gt.log 2>&1 || { echo gt failed; tail -20 $O/gt.log; exit 1; }
echo rc=0
