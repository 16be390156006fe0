set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/layout
timeout -k 10 300 python -u tools/arena_layout.py gpurun_out/layout/arena_layout.json 2>&1 | grep -v amdgpu.ids
