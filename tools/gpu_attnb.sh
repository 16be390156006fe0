# attention microbench (+ rocprof per-kernel split). Usage: gpurun -- bash tools/gpu_attnb.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 120 python -u tools/attn_bench.py > $O/a.log 2>&1 || { echo attn bench failed; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/attn_bench.py > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
cat $O/a.log
echo rc=0
