"""Per-workgroup timelines (diagnostic) at C2 from in-kernel s_memrealtime stamps (100 MHz):
start / first round landed / compute done / end, for the resident attention forward (`fwd`) or
the encoder backward's dQ and dK / dV kernels (`bwd`, stored dropout mask). Prints launch span,
median phase durations and workgroups per CU. usage: python tools/attn_stamps.py fwd|bwd [out.json]"""
import ctypes
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import _lib as L, ops  # noqa: E402

dev = torch.device("cuda")
B, H, Lq, D = 16, 16, 375, 64
mode = sys.argv[1] if len(sys.argv) > 1 else "fwd"
qkv = torch.randn(B * Lq, 3 * H * D, device=dev, dtype=torch.bfloat16)
q, k, v = qkv[:, :1024], qkv[:, 1024:2048], qkv[:, 2048:]
o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
do = torch.randn_like(o)
dq, dk, dv = torch.empty_like(o), torch.empty_like(o), torch.empty_like(o)
lse = torch.empty(B * H * Lq, device=dev)
delta = torch.empty(B * H * Lq, device=dev)
klen = torch.full((B,), Lq, device=dev, dtype=torch.int32)
mask = torch.empty(ops.attn_mask_words(B, H, Lq, Lq), device=dev, dtype=torch.int64)
parts = 1 if mode == "fwd" else 2
buf = torch.zeros(parts * B * H * 6, dtype=torch.int64, device=dev)
lib = L.load()


def run(p, m):
    if mode == "fwd":
        ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lq, klen=klen, drop_p=p, seed=3, mask=m)
    else:
        ops.attn_bwd(do, q, k, v, o, lse, None, dk, dv, delta, B=B, H=H, Lq=Lq, Lk=Lq, klen=klen, drop_p=p, seed=3,
                     dq=dq, mask=m)


def summary(st):
    t0 = min(r[0] for r in st)
    med = lambda x: sorted(x)[len(x) // 2]
    tot = [(r[3] - r[0]) * 10 / 1e3 for r in st]
    cu = Counter(((r[5] & 0xF), (r[4] >> 13) & 7, (r[4] >> 12) & 1, (r[4] >> 8) & 0xF) for r in st)
    start = sorted((r[0] - t0) * 10 / 1e3 for r in st)
    return {"span_us": round((max(r[3] for r in st) - t0) * 10 / 1e3, 2), "start_us_max": round(start[-1], 2),
            "wg_total_us": {"min": round(min(tot), 2), "median": round(med(tot), 2), "max": round(max(tot), 2)},
            "phase_median_us": {"first_round": round(med([(r[1] - r[0]) * 10 / 1e3 for r in st]), 2),
                                "compute": round(med([(r[2] - r[1]) * 10 / 1e3 for r in st]), 2),
                                "store": round(med([(r[3] - r[2]) * 10 / 1e3 for r in st]), 2)},
            "distinct_cus": len(cu), "max_wg_per_cu": max(cu.values())}


res = {}
ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lq, klen=klen, drop_p=0.1, seed=3)
for p in (0.0, 0.1):
    m = ops.attn_dropmask(mask, B=B, H=H, Lq=Lq, Lk=Lq, drop_p=p, seed=3) if p > 0 else None
    for rep in range(3):
        run(p, m)
    torch.cuda.synchronize()
    buf.zero_()
    L.check(lib.avsr_debug_attn_stamps(ctypes.c_void_p(buf.data_ptr())), "stamps on")
    run(p, m)
    torch.cuda.synchronize()
    L.check(lib.avsr_debug_attn_stamps(None), "stamps off")
    allst = buf.view(parts, -1, 6).cpu().tolist()
    for i, st in enumerate(allst):
        name = f"{mode}{'' if parts == 1 else ('_dq' if i == 0 else '_dkdv')}_drop{p}"
        res[name] = summary(st)
        print(name, json.dumps(res[name]), flush=True)
if len(sys.argv) > 2:
    json.dump(res, open(sys.argv[2], "w"), indent=1)
