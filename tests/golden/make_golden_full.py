"""Generate the FULL-SIZE golden vectors of tests/golden/ by running the REFERENCE (quanpn90/avsr,
mounted read-only at /root/reference) on CPU, fp32, in this container.

Never run on the GPU box (the reference does not travel); only its outputs are committed:
  tests/golden/avsr_full.npz

Model: the BASELINE configs' model, AVHubertAVSRConfig(odim=5049) (24 encoder layers, 6
decoder layers, 428 M parameters), weights from oracle/weights.py gen_tensor(key, shape,
seed=0). Inputs are regenerated from their seeds by the tests (they are
too large to commit); their checksums are stored to prove the regeneration is the same.

  C1 (BASELINE configs[0]): eval mode, 8 clips x 1 s (T=25), encoder without mask
      (script/evaluation.py:96-101 call form), then per clip greedy (beam 1), beam 3 (C4) and
      beam 5 (C5) decoding (get_beam_search_decoder, ctc_weight 0.1): yseq + score of the best
      hypothesis, a decoder batch_score and the CTC log-softmax of clip 0.
  C2-shaped train step: train mode, all dropouts 0, B=2 x 15 s (T=375) with the second row
      padded to 300 frames, labels of 40 and 31 tokens: losses, slices of the encoder output /
      CTC logits / decoder logits, every parameter-gradient norm + head, BN running stats.

The one shim SURVEY.md §8(c) c2 documents is applied on the instance
(encoder.encoder._use_flash_attention_2 = False).

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_full.py   (≈ 3 min, ≈ 20 GB RAM)
"""
import hashlib
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

from oracle.weights import NO_DROPOUT, collate, gen_tensor, make_inputs  # noqa: E402
from tests.golden.full_inputs import C1, DEC_ROWS, ENC_ROWS, TR, TR_LABELS  # noqa: E402

def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    torch.manual_seed(0)
    np.random.seed(0)
    torch.set_num_threads(8)
    from src.avhubert_avsr.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
    from src.avhubert_avsr.configuration_avhubert_avsr import AVHubertAVSRConfig

    t0 = time.time()
    cfg = AVHubertAVSRConfig(odim=5049, **NO_DROPOUT)
    model = AVHubertAVSR(cfg)
    sd = model.state_dict()
    model.load_state_dict({k: torch.from_numpy(gen_tensor(k, v.shape, seed=0)) for k, v in sd.items()}, strict=True)
    model.avsr.encoder.encoder._use_flash_attention_2 = False  # SURVEY §8(c) c2 shim
    out = {"param_keys": np.array(list(sd.keys())),
           "param_shapes": np.array([",".join(map(str, v.shape)) for v in sd.values()])}
    print(f"model built in {time.time() - t0:.1f} s")

    # ---------------------------------------------------------------- C1: eval + decode
    frames, feats, lengths, _ = make_inputs(B=C1["B"], T=C1["T"], lengths=C1["lengths"], seed=C1["seed"])
    b1 = collate(frames, feats, lengths, [(1,)] * C1["B"])
    out["c1_digest"] = np.array(digest(b1["videos"], b1["audios"]))
    model.eval()
    with torch.no_grad():
        enc = model.avsr.encoder(input_features=torch.from_numpy(b1["audios"]),
                                 video=torch.from_numpy(b1["videos"])).last_hidden_state
    out["c1_enc"] = enc.numpy()
    token_list = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
    for beam in (1, 3, 5):
        t1 = time.time()
        for c in range(C1["B"]):
            with torch.no_grad():
                hyps = get_beam_search_decoder(model.avsr, token_list, ctc_weight=0.1, beam_size=beam)(enc[c])
            best = hyps[0].asdict()
            out[f"c1_yseq_b{beam}_{c}"] = np.array([int(t) for t in best["yseq"]])
            out[f"c1_score_b{beam}_{c}"] = np.array([float(best["score"])])
        print(f"beam {beam}: {time.time() - t1:.1f} s, clip0 yseq {out[f'c1_yseq_b{beam}_0'][:8]}")
    with torch.no_grad():
        ys = torch.tensor([[5048, 5, 17, 301], [5048, 4000, 4000, 2]])
        logp, _ = model.avsr.decoder.batch_score(ys, [None, None], enc[:2])
        out["c1_batch_score"] = logp.numpy()
        out["c1_ctc_logp0"] = model.avsr.ctc.log_softmax(enc[:1]).numpy()

    # ---------------------------------------------------------------- C2-shaped train step
    frames, feats, lengths, _ = make_inputs(B=TR["B"], T=TR["T"], lengths=TR["lengths"], seed=TR["seed"])
    b2 = {k: torch.from_numpy(v) for k, v in collate(frames, feats, lengths, TR_LABELS).items()}
    del frames
    out["tr_digest"] = np.array(digest(b2["videos"].numpy(), b2["audios"].numpy(), b2["labels"].numpy()))
    model.train()
    caps = {}
    hooks = [model.avsr.encoder.register_forward_hook(
                 lambda m, i, o: caps.__setitem__("enc", o.last_hidden_state.detach().clone())),
             model.avsr.ctc.ctc_lo.register_forward_hook(lambda m, i, o: caps.__setitem__("ctc", o.detach().clone())),
             model.avsr.decoder.register_forward_hook(lambda m, i, o: caps.__setitem__("dec", o[0].detach().clone()))]
    t1 = time.time()
    res = model(**b2)
    for h in hooks:
        h.remove()
    res.loss.backward()
    print(f"train fwd+bwd {time.time() - t1:.1f} s, loss {res.loss.item():.6f}")
    out["tr_loss"] = np.array([res.loss.item(), res.loss_ctc.item(), res.loss_att.item(), float(res.acc)])
    enc = caps["enc"]
    out["tr_enc_rows"] = enc[:, list(ENC_ROWS)].numpy()                    # (2, 7, 1024)
    out["tr_enc_rownorm"] = enc.norm(dim=-1).numpy()                      # (2, 375)
    out["tr_ctc_rows"] = caps["ctc"][:, list(ENC_ROWS)].numpy()           # (2, 7, 5049)
    out["tr_dec_rows"] = caps["dec"][:, list(DEC_ROWS)].numpy()           # (2, 5, 5049)
    gkeys, gnorm, ghead = [], [], []
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        gkeys.append(k)
        gnorm.append(p.grad.double().norm().item())
        ghead.append(p.grad.flatten()[:8].numpy())
    out["grad_keys"] = np.array(gkeys)
    out["grad_norm"] = np.array(gnorm)
    out["grad_head"] = np.stack([np.pad(g, (0, 8 - len(g))) for g in ghead])
    bufs = model.state_dict()
    rkeys = [k for k in bufs if k.endswith("running_mean") or k.endswith("running_var")]
    out["bn_keys"] = np.array(rkeys)
    out["bn_after"] = np.stack([np.pad(bufs[k].flatten()[:8].numpy(), (0, 8 - min(8, bufs[k].numel()))) for k in rkeys])

    path = os.path.join(HERE, "avsr_full.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes in", round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
