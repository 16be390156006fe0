# A/B: slab vs atomic conv weight-gradient, bench + kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/a1.log 2>&1 || exit 1
AVSR_WGRAD_SLAB=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/b1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/a2.log 2>&1 || exit 1
AVSR_WGRAD_SLAB=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/b2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
for f in a1 b1 a2 b2; do echo $f; grep -o '"ms_per_step": [0-9.]*' $O/$f.log; done
echo rc=0
