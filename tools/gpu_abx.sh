# Interleaved in-step A/B over variants "lib|flags": lib = base or an ab/NAME build, flags = engine
# constants / opt:OPTION for tools/bench_flags.py (comma separated, "-" for none).
# Usage: gpurun -- bash tools/gpu_abx.sh TAG "base|-" "r5|ATTN_MASK=0" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abx}; shift; mkdir -p $O
for rep in ${REPS:-1 2}; do
  for v in "$@"; do
    lib=${v%%|*}; fl=${v#*|}
    if [ "$lib" = base ]; then unset AVSR_LIB_PATH_AB; else export AVSR_LIB_PATH_AB=ab/$lib/libavsr_hip.so; fi
    [ "$fl" = "-" ] && fl=""
    tag=$(echo "$lib.$fl" | tr '=,|:' '-_._')
    timeout -k 10 300 python -u tools/bench_flags.py $(echo $fl | tr ',' ' ') -- --steps 12 --warmup 3 --quick --no-cpu-baseline --no-decode > $O/$tag.$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/$tag.$rep.log; exit 1; }
    tail -1 $O/$tag.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['modality_variants']; print('$v', $rep, d['value'], d['ms_per_step'], m['step_ms'], m['value_expected'])"
  done
done
