"""Host cost per launch of a few ops (tiny shapes, so the GPU never limits): microseconds of
Python + C-ABI per call, and the stream-pointer query alone. usage: python tools/launch_bench.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import _lib as L, ops  # noqa: E402

dev = torch.device("cuda")
x = torch.randn(256, 256, device=dev, dtype=torch.bfloat16)
W = torch.randn(256, 256, device=dev, dtype=torch.bfloat16)
g = torch.ones(256, device=dev)
db = torch.zeros(256, device=dev)


def per_call(fn, n=2000):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        fn()
        if i % 200 == 199:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


print(f"stream_ptr        {per_call(lambda: L.stream_ptr(), 20000):6.2f} us", flush=True)
print(f"torch current_stream {per_call(lambda: torch.cuda.current_stream().cuda_stream, 20000):6.2f} us", flush=True)
print(f"linear_fwd 256^3  {per_call(lambda: ops.linear_fwd(x, W)):6.2f} us", flush=True)
print(f"ew_bwd + db       {per_call(lambda: ops.ew_bwd(x, db=db)):6.2f} us", flush=True)
print(f"layernorm_fwd     {per_call(lambda: ops.layernorm_fwd(x, g, db, 1e-5)):6.2f} us", flush=True)
print(f"torch.empty 1MB   {per_call(lambda: torch.empty(1 << 18, device=dev)):6.2f} us", flush=True)
