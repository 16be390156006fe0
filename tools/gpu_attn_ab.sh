# attention tests + A/B microbench (ab/libavsr_base.so vs the tree's library), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-atab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model_parity.py tests/test_gpu_fullsize_golden.py tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  echo "base:" >> $O/attn.log
  AVSR_LIB_PATH_AB=$GRAFT_REPO_ROOT/ab/libavsr_base.so timeout -k 10 120 python -u tools/attn_bench.py >> $O/attn.log 2>&1 || { echo attn bench failed; exit 1; }
  echo "new:" >> $O/attn.log
  timeout -k 10 120 python -u tools/attn_bench.py >> $O/attn.log 2>&1 || { echo attn bench failed; exit 1; }
done
grep -v amdgpu.ids $O/attn.log
echo rc=0
