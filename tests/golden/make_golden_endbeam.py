"""Golden vectors for beam searches that END BEFORE maxlen, produced by
running the REFERENCE (quanpn90/avsr, read-only at /root/reference) on CPU, fp32, in this
container. Never run on the GPU box; only the .npz output is committed:
  tests/golden/avsr_endbeam.npz

With the recipe weights every C1 search runs to maxlen (random decoder logits never favour
<eos>), so end_detect (src/nets/e2e_asr_common.py:18-48) and the ranking of hypotheses that
ended at different lengths (src/nets/beam_search.py:330-406, post_process :408-456) were never
exercised against the reference. Here the full-size model's recipe weights get
`avsr.decoder.output_layer.bias[eos] += EOS_BIAS` for a few offsets, and the reference's own C1
encoder output (avsr_full.npz "c1_enc") is decoded with beams 3 and 5
(get_beam_search_decoder, ctc_weight 0.1). Stored per (offset, beam, clip): EVERY returned
hypothesis (the reference returns all ended hypotheses, best first) — token sequences and
total / decoder / ctc scores — and the step at which the search stopped.

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_endbeam.py   (≈ 4 min, ≈ 10 GB RAM)
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from oracle.weights import NO_DROPOUT, gen_tensor  # noqa: E402
from tests.golden.full_inputs import ENDBEAM  # noqa: E402


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    from src.avhubert_avsr.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
    from src.avhubert_avsr.configuration_avhubert_avsr import AVHubertAVSRConfig

    t0 = time.time()
    model = AVHubertAVSR(AVHubertAVSRConfig(odim=5049, **NO_DROPOUT))
    sd = model.state_dict()
    model.load_state_dict({k: torch.from_numpy(gen_tensor(k, v.shape, seed=0)) for k, v in sd.items()}, strict=True)
    model.eval()
    enc = torch.from_numpy(np.load(os.path.join(HERE, "avsr_full.npz"), allow_pickle=False)["c1_enc"])
    token_list = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
    eos = model.avsr.eos
    bias = model.avsr.decoder.output_layer.bias
    base = bias.detach().clone()
    out = {}
    print(f"model built in {time.time() - t0:.1f} s")
    for off in ENDBEAM["offsets"]:
        with torch.no_grad():
            bias.copy_(base)
            bias[eos] += off
        for beam in ENDBEAM["beams"]:
            bs = get_beam_search_decoder(model.avsr, token_list, ctc_weight=0.1, beam_size=beam)
            for c in ENDBEAM["clips"]:
                with torch.no_grad():
                    hyps = bs(enc[c])
                d = [h.asdict() for h in hyps]
                key = f"eb_{off:g}_b{beam}_{c}"
                out[key + "_len"] = np.array([len(h["yseq"]) for h in d])
                out[key + "_yseq"] = np.concatenate([np.array([int(t) for t in h["yseq"]]) for h in d])
                out[key + "_score"] = np.array([float(h["score"]) for h in d])
                out[key + "_dec"] = np.array([float(h["scores"]["decoder"]) for h in d])
                out[key + "_ctc"] = np.array([float(h["scores"]["ctc"]) for h in d])
                print(f"{key}: {len(d)} ended, lengths {out[key + '_len'].tolist()[:8]}, best {d[0]['score']:.3f}",
                      flush=True)
    path = os.path.join(HERE, "avsr_endbeam.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes in", round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
