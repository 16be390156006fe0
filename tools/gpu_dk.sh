# decode kernels in isolation. Usage: gpurun -- bash tools/gpu_dk.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dk}; mkdir -p $O
timeout -k 10 200 python -u tools/dec_kbench.py > $O/dk.txt 2>&1 || { echo bench failed; tail -20 $O/dk.txt; exit 1; }
cat $O/dk.txt
echo rc=0
