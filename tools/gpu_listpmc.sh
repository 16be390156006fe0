set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/list.txt 2>&1 || { echo list failed; exit 1; }
grep -c . gpurun_out/pmc/list.txt
