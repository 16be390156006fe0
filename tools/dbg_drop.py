import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops
dev = torch.device("cuda")
R, N = 300, 3072
dy = torch.randn(R, N, device=dev, dtype=torch.bfloat16)
y = torch.empty_like(dy)
ops.dropout_fwd(dy, y, 0.3, 99)
out = torch.empty_like(dy)
ops.ew_bwd(torch.ones_like(dy), out=out, drop_p=0.3, seed=99)
a = (y != 0); b = (out != 0)
d = (a != b).nonzero()
print("mismatch", d.shape[0], "zeros in dy", (dy == 0).sum().item())
for r, c in d[:10].tolist():
    print(r, c, dy[r, c].item(), y[r, c].item(), out[r, c].item())
