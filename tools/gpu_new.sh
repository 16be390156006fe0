# Run only the given GPU test files (fast iteration). Usage: gpurun -- bash tools/gpu_new.sh TAG files...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-n}
shift
O=gpurun_out/$TAG
mkdir -p $O
export AVSR_REPORT_DIR=$O/report
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/new.log 2>&1 || { echo new tests failed; exit 1; }
echo rc=0
