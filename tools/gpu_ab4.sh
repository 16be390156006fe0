# step-time A/B of kernel switches on video-on steps (bench --quick --force-modality none),
# interleaved: bash tools/gpu_ab4.sh TAG "ENV1=a ENV2=b" "ENV1=c" ... (each arg one config)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab4}; mkdir -p $O; shift
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 240 python -u bench.py --quick --no-cpu-baseline --force-modality none --steps 12 --warmup 3 > $O/c${i}_$rep.log 2>&1 || { echo "bench failed: $cfg"; tail -5 $O/c${i}_$rep.log; exit 1; }
    echo "[$cfg] $(tail -1 $O/c${i}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
echo rc=0
