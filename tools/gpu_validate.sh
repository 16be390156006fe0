# full GPU suite + smoke + default bench line. Usage: gpurun -- bash tools/gpu_validate.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['modality_variants']['value_expected'], d.get('cpu_baseline')); [print(x['config'], x.get('batched_utt_per_s'), x.get('cpu_baseline')) for x in d.get('decode', [])]"
