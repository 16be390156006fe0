# position of the out-proj weight-gradient in each encoder layer's side-stream batch: in-step A/B.
# Usage: gpurun -- bash tools/gpu_r6o2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
REPS="${REPS:-1 2}" bash tools/gpu_abx.sh ${1:-r6o2}/ab "base|-" "base|SIDE_OUT_POS=first" ${LAST:-"base|SIDE_OUT_POS=last"}
