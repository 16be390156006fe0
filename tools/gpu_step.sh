# quick in-step measurement: bench (step only, all modality variants reported) + isolated ResNet fwd/bwd
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-st}; mkdir -p $O
timeout -k 10 400 python -u bench.py --quick --no-cpu-baseline --no-decode > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['modality_variants']['step_ms'],d['modality_variants']['value_expected'],d['roofline']['frac'])"
timeout -k 10 300 python -u tools/resnet_bench.py 5 > $O/rn.log 2>&1 || { echo rn failed; tail -20 $O/rn.log; exit 1; }
grep video $O/rn.log
echo rc=0
