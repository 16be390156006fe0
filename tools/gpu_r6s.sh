# round-6 session check: GPU tests touched by the decoder LayerNorm/dropout fusion and the dQ kernel
# removal, the host-lead trace, and the out-proj / qkv tile sweep. Usage: gpurun -- bash tools/gpu_r6s.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6s}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_fullsize_golden.py tests/test_gpu_model_parity.py tests/test_gpu_cfgvar.py tests/test_lib_abi.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/host_lead.py 10 > $O/host_lead.txt 2>&1 || { echo host_lead failed; tail -20 $O/host_lead.txt; exit 1; }
cat $O/host_lead.txt
GEMM_TABLE_LAYERS=out GEMM_TABLE_PROBE=0 timeout -k 10 300 python -u tools/gemm_table.py $O/table.json auto,128,96,128x64,64,192,256x128,192w8 > $O/table.txt 2>&1 || { echo table failed; tail -20 $O/table.txt; exit 1; }
cat $O/table.txt
