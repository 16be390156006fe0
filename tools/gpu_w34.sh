# stage-3/4 patch weight-grads + pipelined LayerNorm backward: parity tests, isolated timing,
# then an interleaved in-step A/B against the ab/r6h build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-w34}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_norm.py -k "wgrad_patch or layernorm or ln_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u tools/wgrad34_bench.py $O/bench.json 2>&1 | grep -v amdgpu.ids
REPS="1 2" bash tools/gpu_abx.sh ${1:-w34}/ab "base|-" "r6h|-"
