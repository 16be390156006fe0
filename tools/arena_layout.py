"""Dump the flat parameter arena's layout of the full-size model (C2 engine, bf16) as JSON: the
segments, every parameter's (offset, numel), and the encoder layers' decay-segment offsets the
gradient reducer's readiness hook uses (input of tools/ddp_buckets.py).
usage: python tools/arena_layout.py out.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd.avhubert_avsr_model import AVHubertAVSR  # noqa: E402
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig  # noqa: E402

m = AVHubertAVSR(AVHubertAVSRConfig(odim=5049)).train()
m.setup_engine(torch.device("cuda"), torch.bfloat16)
eng = m.avsr.engine()
a = eng.arena
out = {"segments": {k: list(v) for k, v in a.segments.items()},
       "layer_decay_off": list(eng._layer_decay_off),
       "params": {n: {"off": int(v["off"]), "numel": int(v["numel"]) if "numel" in v else None} for n, v in a.meta.items()},
       "total": int(a.grad.numel())}
json.dump(out, open(sys.argv[1], "w"), indent=0)
print("segments", out["segments"], "total", out["total"], "layers", out["layer_decay_off"][:3], "...")
