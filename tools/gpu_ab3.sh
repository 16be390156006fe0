set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
for cfg in "AVSR_BENCH_GCFREEZE=1" "AVSR_BENCH_GCFREEZE=0" "AVSR_BENCH_GCFREEZE=1" "AVSR_BENCH_GCFREEZE=1"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/x.log 2>&1 || { echo "bench failed"; tail -20 $O/x.log; exit 1; }
  tail -1 $O/x.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'], d['host_ms_per_step_timed'], d['allocator_timed']['num_device_alloc']); print(' host', d['host_ms_steps']); print(' strm', d['stream_ms_steps'])"
done
