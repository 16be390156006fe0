set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6k}; mkdir -p $O
bash tools/gpu_t.sh ${1:-r6k}/t tests/test_gpu_gemm.py -k wgrad || exit 1
timeout -k 10 300 python -u -c "
import json, torch, bench
t = bench.encoder_gemm_table(torch.device('cuda'), 6000, 1024, 4096)
for r in t['per_shape']: print(r)
print('worst', t['worst'], 'layer_us', t['layer_us'], 'layer_frac', t['layer_frac'])
json.dump(t, open('$O/gemms.json', 'w'), indent=1)
" 2>&1 | grep -v amdgpu.ids || exit 1
REPS="1 2" bash tools/gpu_abx.sh ${1:-r6k}/ab "base|-" "base|WGRAD_GROUP=0"
