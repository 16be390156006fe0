"""C1 / C4 / C5 decode throughput on the HIP engine (bench.decode_throughput without the CPU
baseline): python tools/decode_bench.py [split]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from avsr_amd import ops  # noqa: E402

# A/B of the few-row GEMM K split: python tools/decode_bench.py [split]
ops.SKINNY_SPLIT = len(sys.argv) > 1 and sys.argv[1] == "split"
print(json.dumps(bench.decode_throughput(torch.device("cuda"), None, None, 0)))
