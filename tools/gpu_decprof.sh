# rocprof kernel trace of the C5 decode (few-row GEMM K split on)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-decp}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/decode_c5.py split > $O/dec.log 2>&1 || { echo dec failed; tail -20 $O/dec.log; exit 1; }
grep C5 $O/dec.log
rm -f $O/p/run_kernel_trace.csv
echo rc=0
