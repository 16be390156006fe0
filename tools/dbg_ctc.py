import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from avsr_amd import ops
dev = torch.device("cuda")
B, T, V, Vp = 4, 50, 5049, 5056
x = torch.randn(B * T, Vp, device=dev)
lse = torch.empty(B * T, device=dev)
print("row_lse", flush=True)
ops.row_lse(x, V, lse); torch.cuda.synchronize(); print("ok", lse[:3].tolist(), flush=True)
lab = torch.tensor([[5, 5, 17, 301, 4000, 17] + [-1] * 24, [77, 5047, 1, 2] + [-1] * 26, [9] * 30, [3, 4] + [-1] * 28], dtype=torch.int32, device=dev)
ll = torch.tensor([6, 4, 30, 2], dtype=torch.int32, device=dev)
il = torch.tensor([50, 41, 20, 7], dtype=torch.int32, device=dev)
S = 61
alpha = torch.empty(B, T, S, device=dev); gamma = torch.empty(B, T, S, device=dev); nll = torch.empty(B, device=dev)
p = ops.ctc_params(x, B, T, V, lab, ll, il, lse, alpha, gamma, nll)
print("ctc_fwd", flush=True)
ops.ctc_fwd(p); torch.cuda.synchronize(); print("ok", nll.tolist(), flush=True)
