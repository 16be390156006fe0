set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_t.sh r6p/t tests/test_gpu_attention.py tests/test_lib_abi.py || exit 1
REPS="1 2" bash tools/gpu_abx.sh r6p/ab "base|-" "base|opt:attn_sq_bwd=1"
