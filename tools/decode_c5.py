"""C5 decode only (8 x 15 s utterances, beam 5, fp32, random-init weights), for profiling:
python tools/decode_c5.py [split]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from avsr_amd import ops  # noqa: E402
from avsr_amd.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder  # noqa: E402
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig  # noqa: E402

ops.SKINNY_SPLIT = len(sys.argv) > 1 and sys.argv[1] == "split"
dev = torch.device("cuda")
torch.manual_seed(0)
model = AVHubertAVSR(AVHubertAVSRConfig(odim=5049)).eval()
model.setup_engine(dev, torch.float32)
tokens = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
bs = get_beam_search_decoder(model.avsr, tokens, ctc_weight=0.1, beam_size=5)
g = torch.Generator().manual_seed(5)
xs = [(torch.randn(375, 1024, generator=g) * 0.5).to(dev) for _ in range(8)]
bs.decode_batch(xs[:2])
torch.cuda.synchronize()
t0 = time.perf_counter()
bs.decode_batch(xs)
torch.cuda.synchronize()
print(f"C5 batched {8 / (time.perf_counter() - t0):.2f} utt/s")
