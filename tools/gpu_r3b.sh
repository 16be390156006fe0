# library-GEMM ceiling on the encoder shapes + a video-on step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3b}
mkdir -p $O
timeout -k 10 300 python -u tools/blas_ref.py $O/blas_ref.json > $O/blas.log 2>&1 || { echo blas failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --quick --no-cpu-baseline --force-modality none > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
echo rc=0
