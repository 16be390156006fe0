# ResNet fwd+bwd kernel trace with the side stream off (isolated per-kernel durations)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rnprof}; mkdir -p $O
export AVSR_SIDE_STREAM=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/resnet_bench.py 2 > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
grep -v amdgpu.ids $O/prof.log | tail -5
echo rc=0
