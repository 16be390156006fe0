set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-hp}; mkdir -p $O
timeout -k 10 300 python -u tools/host_profile.py > $O/hp.log 2>&1 || { echo failed; tail -20 $O/hp.log; exit 1; }
echo rc=0
