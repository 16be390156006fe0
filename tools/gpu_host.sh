set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-host}; mkdir -p $O
timeout -k 10 400 python -u tools/host_profile.py > $O/host.txt 2>&1 || { echo host failed; tail -20 $O/host.txt; exit 1; }
grep "host enqueue" $O/host.txt
echo rc=0
