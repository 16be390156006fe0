set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ln}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_norm.py -m gpu -x -q -k layernorm --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/ln_bench.py > $O/ln.log 2>&1 || { echo ln bench failed; tail -20 $O/ln.log; exit 1; }
grep rows $O/ln.log
echo rc=0
