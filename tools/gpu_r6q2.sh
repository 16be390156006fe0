# overlapped update grid cap, second sweep. Usage: gpurun -- bash tools/gpu_r6q2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
REPS="1 2" bash tools/gpu_abx.sh ${1:-r6q2}/ab "base|-" "base|OPT_OVERLAP_BLOCKS=128" "base|OPT_OVERLAP_BLOCKS=192" "base|OPT_OVERLAP_BLOCKS=384"
