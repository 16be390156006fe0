# attention tests, micro-bench, then per-kernel trace + SQ counters of the micro-bench:
# gpurun -- bash tools/gpu_attn.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-attn}
bash tools/gpu_t2.sh $T && bash tools/gpu_kprof.sh $T/prof "python3 tools/attn_bench.py"
