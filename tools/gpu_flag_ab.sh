# In-step A/B of engine module constants (tools/bench_flags.py): short bench lines, interleaved.
# Usage: gpurun -- bash tools/gpu_flag_ab.sh TAG "NAME=V[,NAME=V]" ...   ("base" = product settings)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fab}; shift; mkdir -p $O
for rep in ${REPS:-1 2}; do
  for v in "$@"; do
    tag=$(echo $v | tr '=,' '-_')
    timeout -k 10 300 python -u tools/bench_flags.py $(echo $v | sed 's/^base$//' | tr ',' ' ') -- --steps 12 --warmup 3 --quick --no-cpu-baseline --no-decode > $O/$tag.$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/$tag.$rep.log; exit 1; }
    tail -1 $O/$tag.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['modality_variants']; print('$v', $rep, d['value'], d['ms_per_step'], m['step_ms'], m['value_expected'])"
  done
done
