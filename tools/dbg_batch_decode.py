"""diagnostic: batched vs per-utterance decode on the tiny golden model (beam 5): max score
difference and the first decoder-step log-prob rows of the same hypothesis in both launches"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from avsr_amd import decode as Dm  # noqa: E402
from avsr_amd.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder  # noqa: E402
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig  # noqa: E402
from oracle.weights import NO_DROPOUT, TINY_CONFIG  # noqa: E402
from tests.oracle_util import golden_state, load_golden  # noqa: E402

TOKENS = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
g = load_golden()
m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT)).eval()
m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
m.setup_engine("cuda", torch.float32)
xs = [torch.from_numpy(g["dec_enc_0"]).cuda(), torch.from_numpy(g["dec_enc_1"]).cuda(),
      torch.from_numpy(g["dec_enc_0"][:11]).cuda(), torch.from_numpy(g["dec_enc_1"][3:17]).cuda()]
for fold in (True, False):
    Dm.FOLD_LN = fold
    for beam in (3, 5):
        bs = get_beam_search_decoder(m.avsr, TOKENS, ctc_weight=0.1, beam_size=beam)
        got = bs.decode_batch(xs)
        worst = 0.0
        for x, hyps in zip(xs, got):
            want = bs(x)
            same = [h.asdict()["yseq"] for h in hyps] == [h.asdict()["yseq"] for h in want]
            d = max(abs(float(a.score) - float(b.score)) for a, b in zip(hyps, want))
            worst = max(worst, d)
            print(f"fold={fold} beam={beam} T={x.shape[0]} yseq_equal={same} max|dscore|={d:.3e}", flush=True)
        print(f"fold={fold} beam={beam} worst {worst:.3e}", flush=True)
