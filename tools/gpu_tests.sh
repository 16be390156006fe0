# GPU parity pass: the given test files first (fast feedback), then the whole -m gpu suite,
# smoke and a default bench line. Usage: gpurun -- bash tools/gpu_tests.sh TAG [test files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-t}
shift
O=gpurun_out/$TAG
mkdir -p $O
export AVSR_REPORT_DIR=$O/report
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/new.log 2>&1 || { echo new tests failed; exit 1; }
fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; exit 1; }
echo rc=0
