# rocprof kernel trace of video-on training steps (bench --force-modality none): per-kernel step
# breakdown (tools/profsum.py) and stream phases (tools/stream_phases.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sp}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --quick --no-cpu-baseline --force-modality none > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
python tools/profsum.py $O/prof/run_kernel_trace.csv 3 60 > $O/sum.txt
python tools/stream_phases.py $O/prof/run_kernel_trace.csv > $O/phases.txt 2>&1 || true
head -62 $O/sum.txt
tail -12 $O/phases.txt
gzip -c $O/prof/run_kernel_trace.csv > $O/trace.csv.gz
rm -f $O/prof/run_kernel_trace.csv
echo rc=0
