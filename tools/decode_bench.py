"""C1 / C4 / C5 decode throughput on the HIP engine (bench.decode_throughput without the CPU
baseline): python tools/decode_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.decode_throughput(torch.device("cuda"), None, None, 0)))
