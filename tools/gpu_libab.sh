# same-box A/B of two builds of the library: attention microbench (old, new, old, new),
# then the attention tests on the new build. usage: gpu_libab.sh OUT
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lab}; mkdir -p $O
L=avsr_amd/libavsr_hip.so
for v in old new old new; do
  cp avsr_amd/libavsr_hip_$v.so $L
  echo "== $v" >> $O/attn.log
  timeout -k 10 120 python -u tools/attn_bench.py >> $O/attn.log 2>&1 || { echo attn bench failed; tail $O/attn.log; exit 1; }
done
cat $O/attn.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo rc=0
