# few-row GEMM microbenchmark (decoder shapes, M = 40 and 10). Usage: gpurun -- bash tools/gpu_sk2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sk2}; mkdir -p $O
for m in 40 10; do
  timeout -k 10 200 python -u tools/skinny_bench.py $m > $O/sk_$m.txt 2>&1 || { echo bench failed; tail -20 $O/sk_$m.txt; exit 1; }
  echo M=$m; cat $O/sk_$m.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/skinny_bench.py 40 > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
rm -f $O/p/run_kernel_trace.csv
echo rc=0
