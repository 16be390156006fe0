# attention tests, encoder-backward phase stamps, micro-bench: gpurun -- bash tools/gpu_stamps.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-st}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py -q -x -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_stamps.py bwd $O/bwd.json 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
