# kernel names / durations of the library GEMMs on the encoder shapes + isolated ResNet fwd/bwd kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-nm}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blas -o run -- python3 tools/blas_ref.py > $O/blas.log 2>&1 || { echo blas failed; tail -20 $O/blas.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn -o run -- python3 tools/resnet_bench.py 3 > $O/rn.log 2>&1 || { echo rn failed; tail -20 $O/rn.log; exit 1; }
echo rc=0
