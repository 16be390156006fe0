# rocprof kernel trace of video-on training steps (bench --force-modality none)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sp}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --quick --no-cpu-baseline --force-modality none > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
python tools/profsum.py $O/prof/run_kernel_trace.csv 3 45 > $O/sum.txt
cat $O/sum.txt
echo rc=0
