"""Per-shape table of the encoder GEMMs at C2 (M = B*T = 6000 tokens, d = 1024, F = 4096):
QKV, out-proj, FFN1, FFN2 x forward / data-grad / weight-grad, each under every GEMM tile
configuration (library option gemm_tile), with the engine's own split-K choice for weight-grads.
Launches are captured in a HIP graph (device time only). Prints a table and writes JSON.

  python tools/gemm_table.py [out.json] [cfg,cfg,...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402
from avsr_amd.engine import wgrad_splitk  # noqa: E402

PEAK = 2500.0
dev = torch.device("cuda")
M, D, F = 6000, 1024, 4096
LAYERS = {"qkv": (3 * D, D), "out": (D, D), "ffn1": (F, D), "ffn2": (D, F)}   # (N, K) of y = x W^T


def timed(fn, n=10, reps=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.reserve_stream_workspaces(dev)      # zeroed split-K counters exist before the capture
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (n * reps) * 1e3      # us


def wgrad(dy, x, dW):
    """the engine's weight-grad launch (Engine._wgrad: split-K into a slab when the output
    grid is at or below one block per CU)"""
    Mt, N = dy.shape
    K = x.shape[1]
    splitk = wgrad_splitk(Mt, N, K)
    ws = torch.empty(ops.slab_ws(1, splitk, N, K), device=dy.device, dtype=torch.float32) if splitk > 1 else None
    ops.gemm(dy, x, dW, M=N, N=K, K=Mt, a_kmajor=False, b_kmajor=False, lda=dy.stride(0), ldb=x.stride(0),
             ldc=dW.stride(0), beta=1.0, splitk=splitk, ws=ws)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["auto", "128", "128s3", "256x128", "128x256", "pp"]
    g = torch.Generator(device="cpu").manual_seed(0)
    rows = []
    only = os.environ.get("GEMM_TABLE_LAYERS")       # e.g. "out": a subset of the layers
    for name, (N, K) in LAYERS.items():
        if only and name not in only.split(","):
            continue
        x = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
        W = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        dy = (torch.randn(M, N, generator=g) * 0.5).to(dev, torch.bfloat16)
        dW = torch.zeros(N, K, device=dev)
        fl = 2.0 * M * N * K
        ops_ = {"fwd": lambda: ops.linear_fwd(x, W),
                "dgrad": lambda: ops.linear_dgrad(dy, W),
                "wgrad": lambda: wgrad(dy, x, dW)}
        if name == "ffn1" and os.environ.get("GEMM_TABLE_PROBE", "1") == "1":
            # the bench roofline probe: FFN1 forward with its full epilogue (bias, GELU, pre-activation
            # store, dropout); not counted in the layer totals below
            bias = torch.zeros(N, device=dev)
            h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops_["probe"] = lambda: ops.linear_fwd(x, W, bias, act=1, preact=h, drop_p=0.1, seed=7)
        for op, fn in ops_.items():
            rec = {"layer": name, "op": op, "M": M, "N": N if op != "dgrad" else K, "K": K if op != "dgrad" else N,
                   "gflop": round(fl / 1e9, 2), "us": {}, "tflops": {}}
            if op == "wgrad":
                rec.update(M=N, N=K, K=M)
            for c in cfgs:
                if c == "auto":
                    ops.L.set_option("gemm_tile", "auto")
                else:
                    ops.L.set_option("gemm_tile", c)
                try:
                    us = timed(fn)
                except Exception as e:          # a config may refuse a shape
                    print(f"  {name} {op} {c}: {e}", flush=True)
                    continue
                rec["us"][c] = round(us, 2)
                rec["tflops"][c] = round(fl / us / 1e6, 1)
            ops.L.set_option("gemm_tile", "auto")
            best = max(rec["tflops"], key=rec["tflops"].get)
            rec["best"] = best
            rec["best_frac"] = round(rec["tflops"][best] / PEAK, 4)
            rows.append(rec)
            print(f"{name:5s} {op:5s} M{rec['M']:5d} N{rec['N']:5d} K{rec['K']:5d} " +
                  " ".join(f"{c}:{rec['us'].get(c, float('nan')):7.1f}us/{rec['tflops'].get(c, 0):5.0f}" for c in cfgs) +
                  f"  best {best} {rec['best_frac']:.3f}", flush=True)
    layer = [r for r in rows if r["op"] != "probe"]
    tot_auto = sum(r["us"].get("auto", 0) for r in layer)
    tot_best = sum(min(r["us"].values()) for r in layer)
    fl_all = sum(r["gflop"] for r in layer) * 1e9
    print(f"one encoder layer, 12 GEMMs: auto {tot_auto:.0f} us ({fl_all / tot_auto / 1e6:.0f} TF/s), "
          f"best-per-shape {tot_best:.0f} us ({fl_all / tot_best / 1e6:.0f} TF/s)", flush=True)
    if out:
        json.dump({"shape_note": "encoder GEMMs at C2, M=6000 tokens", "peak_tflops": PEAK, "rows": rows,
                   "layer_total_us": {"auto": tot_auto, "best_per_shape": tot_best}}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
