set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ln}; mkdir -p $O
timeout -k 10 200 python -u tools/ln_bench.py > $O/ln.txt 2>&1 || { echo ln failed; tail -20 $O/ln.txt; exit 1; }
grep -v amdgpu.ids $O/ln.txt
