# stream-K GEMM: parity tests, then time vs K and the encoder table against whole-tile grids
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 60 --timeout-method thread -k "stream_k or bit_identical" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in ${2:-128 128sk 192 192sk}; do
AVSR_GEMM_TILE=$c timeout -k 10 200 python -u tools/gemm_k.py 6000 4096 >> $O/gemm_k.txt 2>&1 || { echo gemm_k failed; tail -20 $O/gemm_k.txt; exit 1; }
done
grep -v amdgpu.ids $O/gemm_k.txt
timeout -k 10 600 python -u tools/gemm_table.py $O/gemm_table.json ${3:-auto,128,128sk,192sk} > $O/gemm_table.txt 2>&1 || { echo table failed; tail -20 $O/gemm_table.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_table.txt
echo rc=0
