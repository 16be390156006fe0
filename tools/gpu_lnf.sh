# norm tests + model parity tests touching the encoder backward + quick step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lnf}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_model_parity.py tests/test_gpu_c2_batch.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py --quick --no-cpu-baseline --no-decode > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['modality_variants']['step_ms'],d['modality_variants']['value_expected'],d['roofline']['frac'])"
AVSR_LN_EW_FUSE=0 timeout -k 10 400 python -u bench.py --quick --no-cpu-baseline --no-decode > $O/bench0.json 2> $O/bench0.err || { echo bench0 failed; tail -20 $O/bench0.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench0.json'));print('fuse=0', d['value'],d['ms_per_step'],d['modality_variants']['step_ms'],d['modality_variants']['value_expected'])"
echo rc=0
