# conv tests + stem weight-grad A/B (64x512 vs 64x256 tiles). Usage: gpurun -- bash tools/gpu_cw.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cw}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread > $O/conv.log 2>&1 || { echo conv tests failed; tail -30 $O/conv.log; exit 1; }
tail -1 $O/conv.log
for r in 1 2; do for v in 1 0; do
  AVSR_CONV_WGRAD512=$v timeout -k 10 120 python -u tools/conv_one.py wgrad 6000 88 8 64 7 2 10 > $O/w$v.txt 2>&1 || { echo conv_one failed; tail -5 $O/w$v.txt; exit 1; }
  echo "wgrad512=$v $(tail -1 $O/w$v.txt)"
done; done
echo rc=0
