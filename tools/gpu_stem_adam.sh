set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sa}; mkdir -p $O
timeout -k 10 120 python -u tools/adamw_bench.py > $O/adamw.txt 2>&1 || { echo adamw failed; tail -20 $O/adamw.txt; exit 1; }
grep -v amdgpu.ids $O/adamw.txt
bash tools/gpu_stem.sh ${1:-sa}_stem || exit 1
echo rc=0
