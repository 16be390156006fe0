set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof5a -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/p5a.log 2>&1
AVSR_CONV_NOGLDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof5b -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/p5b.log 2>&1
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b5.log 2>&1
AVSR_CONV_NOGLDS=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline >> gpurun_out/b5.log 2>&1
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline >> gpurun_out/b5.log 2>&1
echo rc=$?
