"""Golden vectors for the beam-search configurations at the ends of the CTC-weight range
(VERDICT r04 item 8), produced by running the REFERENCE (quanpn90/avsr, read-only at
/root/reference) on CPU, fp32, in this container. Never run on the GPU box; only the .npz output
is committed: tests/golden/avsr_ctcw.npz

get_beam_search_decoder(model, token_list, ctc_weight, beam_size)
(src/avhubert_avsr/avhubert_avsr_model.py:12-36) builds, for
  ctc_weight = 0.0: the decoder scorer alone (a scorer of weight 0 is dropped,
                    src/nets/beam_search.py:69-73; no partial scorer, so no pre-beam: :96-100);
  ctc_weight = 1.0: the CTC prefix scorer alone over the FULL vocabulary
                    (pre_beam_score_key=None; the decoder's weight is 0).
Model: the tiny recipe (oracle/weights.py TINY_CONFIG, gen_tensor weights, seed 0, dropouts 0,
eval); inputs: the reference's own encoder outputs stored in avsr_tiny.npz (dec_enc_0 / _1).
Stored per (ctc weight, beam, clip): EVERY returned hypothesis (token sequence, total score,
per-scorer scores).

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ctcw.py   (≈ 1 min)
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

from oracle.weights import NO_DROPOUT, TINY_CONFIG, gen_tensor  # noqa: E402

WEIGHTS = (0.0, 1.0)
BEAMS = (1, 3)


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    from src.avhubert_avsr.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
    from src.avhubert_avsr.configuration_avhubert_avsr import AVHubertAVSRConfig

    t0 = time.time()
    model = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT))
    sd = model.state_dict()
    model.load_state_dict({k: torch.from_numpy(gen_tensor(k, v.shape, seed=0)) for k, v in sd.items()}, strict=True)
    model.eval()
    g = np.load(os.path.join(HERE, "avsr_tiny.npz"), allow_pickle=False)
    token_list = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
    out = {}
    for w in WEIGHTS:
        for beam in BEAMS:
            bs = get_beam_search_decoder(model.avsr, token_list, ctc_weight=w, beam_size=beam)
            for c in range(2):
                x = torch.from_numpy(g[f"dec_enc_{c}"])
                with torch.no_grad():
                    hyps = bs(x)
                d = [h.asdict() for h in hyps]
                key = f"w{w:g}_b{beam}_{c}"
                out[key + "_len"] = np.array([len(h["yseq"]) for h in d])
                out[key + "_yseq"] = np.concatenate([np.array([int(t) for t in h["yseq"]]) for h in d])
                out[key + "_score"] = np.array([float(h["score"]) for h in d])
                for s in ("decoder", "ctc"):
                    if s in d[0]["scores"]:
                        out[key + "_" + s] = np.array([float(h["scores"][s]) for h in d])
                print(f"{key}: {len(d)} hyps, lengths {out[key + '_len'].tolist()[:8]}, best {d[0]['score']:.4f}, "
                      f"scorers {sorted(d[0]['scores'])}", flush=True)
    path = os.path.join(HERE, "avsr_ctcw.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes in", round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
