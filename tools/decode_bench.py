"""Decode throughput (C1 / C4 / C5-shaped synthetic utterances, full-size model, random-init
weights so every search runs to maxlen = T): utterances per second for the one-utterance
search (the reference's call form, script/evaluation.py:280-296) and the batched search.
  python tools/decode_bench.py [n_utts] [T] [beam] [dtype]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(n_utts=8, T=100, beam=3, dtype="float32", model=None):
    from avsr_amd.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
    from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
    dt = getattr(torch, dtype)
    if model is None:
        torch.manual_seed(0)
        model = AVHubertAVSR(AVHubertAVSRConfig(odim=5049)).eval()
        model.setup_engine("cuda", dt)
    tokens = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
    bs = get_beam_search_decoder(model.avsr, tokens, ctc_weight=0.1, beam_size=beam)
    g = torch.Generator().manual_seed(5)
    xs = [(torch.randn(T - 7 * (u % 3), 1024, generator=g) * 0.5).cuda() for u in range(n_utts)]
    bs(xs[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seq = [bs(x) for x in xs]
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    bat = bs.decode_batch(xs)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    same = all([h.asdict()["yseq"] for h in a] == [h.asdict()["yseq"] for h in b] for a, b in zip(seq, bat))
    return {"utterances": n_utts, "frames_per_utt": T, "beam": beam, "dtype": dtype,
            "sequential_utt_per_s": round(n_utts / (t1 - t0), 2), "batched_utt_per_s": round(n_utts / (t2 - t1), 2),
            "batched_equals_sequential": same}


if __name__ == "__main__":
    a = sys.argv[1:]
    print(json.dumps(run(int(a[0]) if a else 8, int(a[1]) if len(a) > 1 else 100, int(a[2]) if len(a) > 2 else 3,
                         a[3] if len(a) > 3 else "float32")))
