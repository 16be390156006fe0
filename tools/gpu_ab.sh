# In-step A/B of library variants (tools/build_variant.py): short bench lines, interleaved.
# Usage: gpurun -- bash tools/gpu_ab.sh TAG variant[,variant...]   ("base" = the product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
for rep in ${REPS:-1 2}; do
  for v in $(echo ${2:-base} | tr , ' '); do
    if [ $v = base ]; then unset AVSR_LIB_PATH_AB; else export AVSR_LIB_PATH_AB=ab/$v/libavsr_hip.so; fi
    timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --quick --no-cpu-baseline --no-decode > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.$rep.log; exit 1; }
    tail -1 $O/$v.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['modality_variants']; print('$v', $rep, d['value'], d['ms_per_step'], m['step_ms'], m['value_expected'], d['roofline']['avg_launch_ms'])"
  done
done
