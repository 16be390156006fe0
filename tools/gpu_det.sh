set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det}; mkdir -p $O
timeout -k 10 200 python -u tools/stem_det.py > $O/sdet.log 2>&1; cat $O/sdet.log; timeout -k 10 400 python -u tools/det_check.py > $O/det.log 2>&1 || { echo det failed; tail -20 $O/det.log; exit 1; }
tail -1 $O/det.log
echo rc=0
