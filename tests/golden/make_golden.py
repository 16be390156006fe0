"""Generate the golden vectors of tests/golden/ by running the REFERENCE (quanpn90/avsr,
mounted read-only at /root/reference) on CPU, fp32, in this container.

Never run on the GPU box (the reference does not travel); only its outputs are committed:
  tests/golden/avsr_tiny.npz   — see the `out[...]` keys below.

Recipe: tiny AVHubertAVSRConfig (oracle/weights.py TINY_CONFIG) with all
dropouts 0, weights from oracle/weights.py gen_tensor(key, shape, seed=0), inputs from
make_inputs()/collate() (B=2, T=25, lengths [25, 19]). The one shim SURVEY.md §8(c) c2
documents is applied on the instance: encoder.encoder._use_flash_attention_2 = False.

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from oracle.weights import NO_DROPOUT, TINY_CONFIG, collate, gen_tensor, make_inputs  # noqa: E402


def main():
    torch.manual_seed(0)
    np.random.seed(0)
    torch.set_num_threads(8)
    from src.avhubert_avsr.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
    from src.avhubert_avsr.configuration_avhubert_avsr import AVHubertAVSRConfig

    cfg = AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT)
    model = AVHubertAVSR(cfg)
    sd = model.state_dict()
    new = {k: torch.from_numpy(gen_tensor(k, v.shape, seed=0)) for k, v in sd.items()}
    model.load_state_dict(new, strict=True)
    model.avsr.encoder.encoder._use_flash_attention_2 = False  # SURVEY §8(c) c2 shim

    frames, feats, lengths, labels = make_inputs()
    batch = {k: torch.from_numpy(v) for k, v in collate(frames, feats, lengths, labels).items()}
    out = {"frames": frames, "feats": feats, "lengths": lengths,
           "labels": batch["labels"].numpy()}
    out["param_keys"] = np.array(list(sd.keys()))
    out["param_shapes"] = np.array([",".join(map(str, v.shape)) for v in sd.values()])

    # 1) eval-mode encoder forward without mask (script/evaluation.py:96-101 call form)
    model.eval()
    with torch.no_grad():
        enc = model.avsr.encoder(input_features=batch["audios"], video=batch["videos"]).last_hidden_state
    out["enc_eval"] = enc.numpy()

    # 2) train-mode forward + backward (dropouts 0; BN uses batch statistics)
    model.train()
    caps = {}
    h1 = model.avsr.encoder.register_forward_hook(lambda m, i, o: caps.__setitem__("enc", o.last_hidden_state.detach().clone()))
    h2 = model.avsr.ctc.ctc_lo.register_forward_hook(lambda m, i, o: caps.__setitem__("ctc_logits", o.detach().clone()))
    h3 = model.avsr.decoder.register_forward_hook(lambda m, i, o: caps.__setitem__("dec_logits", o[0].detach().clone()))
    res = model(**batch)
    for h in (h1, h2, h3):
        h.remove()
    res.loss.backward()
    out["loss"] = np.array([res.loss.item(), res.loss_ctc.item(), res.loss_att.item(), float(res.acc)])
    out["enc_train"] = caps["enc"].numpy()
    out["ctc_logits"] = caps["ctc_logits"].numpy()       # (B, T, V)
    out["dec_logits"] = caps["dec_logits"].numpy()       # (B, L+1, V)
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
    out["bn_after"] = np.stack([bufs[k].flatten()[:8].numpy() for k in rkeys])

    # 3) decoding: per utterance, B=1 encoder (no mask) + greedy (beam 1) and beam 3
    model.eval()
    token_list = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]
    for b in range(2):
        Tb = int(lengths[b])
        v = batch["videos"][b:b + 1, :, :Tb]
        a = batch["audios"][b:b + 1, :, :Tb]
        with torch.no_grad():
            x = model.avsr.encoder(input_features=a, video=v).last_hidden_state.squeeze(0)
            out[f"dec_enc_{b}"] = x.numpy()
            for beam in (1, 3):
                bs = get_beam_search_decoder(model.avsr, token_list, ctc_weight=0.1, beam_size=beam)
                hyps = bs(x)
                out[f"yseq_b{beam}_{b}"] = np.array([int(t) for t in hyps[0].asdict()["yseq"]])
                out[f"score_b{beam}_{b}"] = np.array([float(hyps[0].asdict()["score"])])
            # decoder one-step log-probs for a fixed prefix (decoder.py:153-227 batch_score)
            ys = torch.tensor([[5048, 5, 17, 301]])
            logp, _ = model.avsr.decoder.batch_score(ys, [None], x.unsqueeze(0))
            out[f"onestep_{b}"] = logp.numpy()
            out[f"ctc_logp_{b}"] = model.avsr.ctc.log_softmax(x.unsqueeze(0)).numpy()

    path = os.path.join(HERE, "avsr_tiny.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")
    print("loss", out["loss"], "yseq", out["yseq_b1_0"][:10], out["yseq_b3_1"][:10])


if __name__ == "__main__":
    main()
