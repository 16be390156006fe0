# GEMM tests + GEMM table (auto) + quick step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-gs}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/gemm_table.py $O/gemm_table.json auto > $O/gt.log 2>&1 || { echo gt failed; tail -20 $O/gt.log; exit 1; }
grep -v amdgpu.ids $O/gt.log
timeout -k 10 400 python -u bench.py --quick --no-cpu-baseline --no-decode > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['modality_variants']['step_ms'],d['modality_variants']['value_expected'],d['roofline']['frac'])"
echo rc=0
