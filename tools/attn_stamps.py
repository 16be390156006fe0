"""Per-workgroup timeline of the resident attention forward at C2 (diagnostic): s_memrealtime
stamps (100 MHz) at start / after the first K/V round / compute done / end, plus HW_ID and
XCC_ID, for one launch. Prints the launch span, per-WG phase durations and how many
workgroups each CU ran. usage: python tools/attn_stamps.py [out.json]"""
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
qkv = torch.randn(B * Lq, 3 * H * D, device=dev, dtype=torch.bfloat16)
q, k, v = qkv[:, :1024], qkv[:, 1024:2048], qkv[:, 2048:]
o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * H * Lq, device=dev)
klen = torch.full((B,), Lq, device=dev, dtype=torch.int32)
buf = torch.zeros(B * H * 6, dtype=torch.int64, device=dev)
lib = L.load()
res = {}
for p in (0.0, 0.1):
    for rep in range(3):
        ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lq, klen=klen, drop_p=p, seed=3)
    torch.cuda.synchronize()
    buf.zero_()
    L.check(lib.avsr_debug_attn_stamps(ctypes.c_void_p(buf.data_ptr())), "stamps on")
    ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lq, klen=klen, drop_p=p, seed=3)
    torch.cuda.synchronize()
    L.check(lib.avsr_debug_attn_stamps(None), "stamps off")
    st = buf.view(-1, 6).cpu().tolist()
    t0 = min(r[0] for r in st)
    span = (max(r[3] for r in st) - t0) * 10 / 1e3
    start = sorted((r[0] - t0) * 10 / 1e3 for r in st)
    load = [(r[1] - r[0]) * 10 / 1e3 for r in st]
    comp = [(r[2] - r[1]) * 10 / 1e3 for r in st]
    store = [(r[3] - r[2]) * 10 / 1e3 for r in st]
    tot = [(r[3] - r[0]) * 10 / 1e3 for r in st]
    # HW_ID (gfx9): wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]; XCC_ID low bits
    cu = Counter(((r[5] & 0xF), (r[4] >> 13) & 7, (r[4] >> 12) & 1, (r[4] >> 8) & 0xF) for r in st)
    med = lambda x: sorted(x)[len(x) // 2]
    rec = {"drop_p": p, "span_us": round(span, 2), "start_us_max": round(start[-1], 2),
           "start_us_p90": round(start[int(len(start) * 0.9)], 2),
           "wg_total_us": {"min": round(min(tot), 2), "median": round(med(tot), 2), "max": round(max(tot), 2)},
           "phase_median_us": {"first_round": round(med(load), 2), "compute": round(med(comp), 2), "store": round(med(store), 2)},
           "distinct_cus": len(cu), "max_wg_per_cu": max(cu.values())}
    res[f"drop{p}"] = rec
    print(json.dumps(rec), flush=True)
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
