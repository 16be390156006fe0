# Round evidence: default bench line, a rocprofv3 kernel trace of video-on steps (per-kernel table,
# probe durations), then the counter passes (tools/gpu_counters.sh). Usage: ... TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ev}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['modality_variants']['step_ms'], d['modality_variants']['value_expected'], d.get('cpu_baseline'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --quick --no-cpu-baseline --force-modality none > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
timeout -k 10 60 python tools/profsum.py $O/prof/run_kernel_trace.csv 4 60 --skip 8 > $O/steps.txt 2>&1 || { echo profsum failed; exit 1; }
timeout -k 10 60 python tools/stream_phases.py $O/prof/run_kernel_trace.csv 4 --skip 8 > $O/phases.txt 2>&1 || echo phases failed
timeout -k 10 60 python tools/probe_trace.py $O/prof/run_kernel_trace.csv > $O/probe.txt 2>&1 || echo probe_trace failed
cat $O/probe.txt; head -25 $O/steps.txt
gzip -9 $O/prof/run_kernel_trace.csv; rm -f $O/prof/run_agent_info.csv
bash tools/gpu_counters.sh $T
