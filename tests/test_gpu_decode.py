"""Beam-search decode on the HIP engine against the CPU oracle
(oracle/decode_oracle.py, itself pinned to the reference's own yseq / scores in
tests/golden/avsr_tiny.npz) and torch fp32 references of the individual kernels."""
import numpy as np
import pytest
import torch

from avsr_amd import ops
from avsr_amd.avhubert_avsr_model import AVHubertAVSR, get_beam_search_decoder
from avsr_amd.configuration_avhubert_avsr import AVHubertAVSRConfig
from oracle import avsr_oracle as O
from oracle import decode_oracle as DO
from oracle.weights import NO_DROPOUT, TINY_CONFIG
from tests.oracle_util import golden_batch, golden_state, load_golden, tiny_cfg

pytestmark = pytest.mark.gpu

TOKENS = ["<blank>"] + [f"u{i}" for i in range(1, 5048)] + ["<eos>"]


@pytest.fixture(scope="module")
def g():
    return load_golden()


@pytest.fixture(scope="module")
def model(g):
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT)).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
    m.setup_engine("cuda", torch.float32)
    return m


def test_dec_attn_matches_torch(dev):
    g = torch.Generator().manual_seed(3)
    n, H, L, D, Lmax = 3, 4, 37, 256, 50
    q = torch.randn(n, 3 * D, generator=g).to(dev)
    kc = torch.randn(n, Lmax, D, generator=g).to(dev)
    vc = torch.randn(n, Lmax, D, generator=g).to(dev)
    o = torch.empty(n, D, device=dev)
    ops.dec_attn(q[:, :D], kc, vc, o, n=n, H=H, klen_max=L, k_bstride=Lmax * D, v_bstride=Lmax * D)
    qh = q[:, :D].view(n, H, 1, 64)
    kh = kc[:, :L].view(n, L, H, 64).transpose(1, 2)
    vh = vc[:, :L].view(n, L, H, 64).transpose(1, 2)
    ref = torch.softmax(qh @ kh.transpose(-1, -2) * 0.125, -1) @ vh
    torch.testing.assert_close(o, ref.reshape(n, D), rtol=1e-5, atol=1e-5)
    # shared keys (bstride 0), bf16 storage
    mem = torch.randn(L, 2 * D, generator=g).to(dev)
    ops.dec_attn(q[:, :D], mem[:, :D], mem[:, D:], o, n=n, H=H, klen_max=L, k_bstride=0, v_bstride=0)
    km = mem[:, :D].view(L, H, 64).transpose(0, 1)
    vm = mem[:, D:].view(L, H, 64).transpose(0, 1)
    ref = torch.softmax(qh @ km.transpose(-1, -2).unsqueeze(0) * 0.125, -1) @ vm.unsqueeze(0)
    torch.testing.assert_close(o, ref.reshape(n, D), rtol=1e-5, atol=1e-5)


def test_row_topk_and_log_softmax(dev):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(5, 5056, generator=g).to(dev)
    lp = torch.empty(5, 5049, device=dev)
    ops.log_softmax_rows(x, 5049, lp)
    torch.testing.assert_close(lp, torch.log_softmax(x[:, :5049], -1), rtol=1e-5, atol=1e-5)
    ids = torch.empty(5, 7, device=dev, dtype=torch.int32)
    ops.row_topk(lp, 5049, 7, ids)
    assert torch.equal(ids.long().cpu(), torch.topk(lp.cpu(), 7, dim=-1)[1])


@pytest.mark.parametrize("V", [5049, 7000])
def test_log_softmax_topk_equals_separate_kernels(dev, V):
    """the fused decode-step kernel (V <= 6144 in registers; 7000 takes the two-pass path) is
    bit-identical to log_softmax_rows + row_topk, ties included"""
    g = torch.Generator().manual_seed(6)
    x = (torch.randn(9, V + 7, generator=g) * 4).round() / 4      # many exact ties
    x = x.to(dev)
    lp_a = torch.empty(9, V, device=dev)
    ids_a = torch.empty(9, 7, device=dev, dtype=torch.int32)
    ops.log_softmax_rows(x, V, lp_a)
    ops.row_topk(lp_a, V, 7, ids_a)
    lp_b = torch.full((9, V), float("nan"), device=dev)
    ids_b = torch.full((9, 7), -1, device=dev, dtype=torch.int32)
    ops.log_softmax_topk(x, V, lp_b, 7, ids_b)
    assert torch.equal(lp_a, lp_b)
    assert torch.equal(ids_a, ids_b)


@pytest.mark.parametrize("first,T,P", [(True, 40, 4), (False, 40, 4), (False, 375, 7)])
def test_ctc_prefix_matches_oracle(dev, first, T, P):
    g = torch.Generator().manual_seed(5)
    V, n = 300, 3
    logp = torch.log_softmax(torch.randn(T, V, generator=g) * 3, -1)
    eos = V - 1
    if first:
        yseqs = [[eos]] * n
        states = [None] * n
    else:
        yseqs = [[eos, 5, 7], [eos, 7, 7], [eos, 9, 2]]
        states = [(torch.log_softmax(torch.randn(T, 2, generator=g), -1) - 3.0, -2.5) for _ in range(n)]
    ids = torch.stack([torch.randperm(V - 2, generator=g)[:P] + 1 for _ in range(n)])
    ids[1, 0] = yseqs[1][-1]          # repeated-label path
    ids[2, 1] = eos
    ids[0, 2] = 0                     # blank among the scored ids
    ref_sc, ref_r, ref_psi = DO.ctc_prefix_scores(logp.double(), yseqs, [None if s is None else (s[0].double(), s[1]) for s in states],
                                                  ids, 0, eos)
    r_prev = None if first else torch.stack([s[0] for s in states]).to(dev).contiguous()
    last = torch.tensor([y[-1] for y in yseqs], dtype=torch.int32, device=dev)
    r_new = torch.empty(n, P, T, 2, device=dev)
    psi = torch.empty(n, P + 1, device=dev)
    ops.ctc_prefix(logp.to(dev), r_prev, last, ids.to(dev, torch.int32), r_new, psi, n=n, out_len=len(yseqs[0]) - 1,
                   blank=0, eos=eos)
    for h in range(n):
        for j in range(P):
            want = ref_psi[h, ids[h, j]].item()
            assert abs(psi[h, j].item() - want) <= 1e-5 * abs(want) + 1e-4, (h, j, psi[h, j].item(), want)
        assert abs(psi[h, P].item() - ref_psi[h, eos].item()) <= 1e-5 * abs(ref_psi[h, eos].item()) + 1e-4
    rr = ref_r.permute(2, 3, 0, 1).float()     # (n, P, T, 2)
    ok = rr > -1e9
    torch.testing.assert_close(r_new.cpu()[ok], rr[ok], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("b", [0, 1])
@pytest.mark.parametrize("beam", [1, 3])
def test_beam_search_on_reference_encoder_output(g, model, b, beam):
    """the HIP decode of the reference's own encoder output reproduces the reference's best
    hypothesis exactly (token ids) and its score (1e-4 relative)."""
    x = torch.from_numpy(g[f"dec_enc_{b}"]).cuda()
    bs = get_beam_search_decoder(model.avsr, TOKENS, ctc_weight=0.1, beam_size=beam)
    hyps = bs(x)
    best = hyps[0].asdict()
    assert best["yseq"] == g[f"yseq_b{beam}_{b}"].tolist()
    ref = float(g[f"score_b{beam}_{b}"][0])
    assert abs(best["score"] - ref) <= 1e-4 * abs(ref)


@pytest.fixture(scope="module")
def trained_model(g):
    """make_golden.py decodes AFTER its train-mode forward, which moved the BatchNorm running
    statistics: replay that forward (it updates the running statistics the same way)."""
    m = AVHubertAVSR(AVHubertAVSRConfig(**TINY_CONFIG, **NO_DROPOUT)).train()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(g).items()}, strict=True)
    m.setup_engine("cuda", torch.float32)
    batch = {k: torch.from_numpy(v) for k, v in golden_batch(g).items()}
    with torch.no_grad():
        m(**batch)
    return m.eval()


@pytest.mark.parametrize("b", [0, 1])
def test_encode_then_decode_end_to_end(g, trained_model, b):
    """script/evaluation.py:96-107 call form on the engine: encoder (B=1, no mask) + beam 3."""
    batch = golden_batch(g)
    Tb = int(g["lengths"][b])
    v = torch.from_numpy(np.ascontiguousarray(batch["videos"][b:b + 1, :, :Tb]))
    a = torch.from_numpy(np.ascontiguousarray(batch["audios"][b:b + 1, :, :Tb]))
    x = trained_model.avsr.engine().encode(a, v)[0]
    ref = torch.from_numpy(g[f"dec_enc_{b}"])
    assert float((x.cpu() - ref).abs().max() / ref.abs().max()) < 2e-4
    hyps = get_beam_search_decoder(trained_model.avsr, TOKENS, ctc_weight=0.1, beam_size=3)(x)
    assert hyps[0].asdict()["yseq"] == g[f"yseq_b3_{b}"].tolist()


@pytest.mark.parametrize("beam", [1, 3, 5])
def test_batched_decode_equals_per_utterance(g, model, beam):
    """decode_batch over utterances of different lengths returns, per utterance, exactly the
    hypotheses of the one-utterance search: tokens identical, total and per-scorer scores equal
    as floats (bit for bit, no rounding)."""
    bs = get_beam_search_decoder(model.avsr, TOKENS, ctc_weight=0.1, beam_size=beam)
    xs = [torch.from_numpy(g["dec_enc_0"]).cuda(), torch.from_numpy(g["dec_enc_1"]).cuda(),
          torch.from_numpy(g["dec_enc_0"][:11]).cuda(), torch.from_numpy(g["dec_enc_1"][3:17]).cuda()]
    got = bs.decode_batch(xs)
    for x, hyps in zip(xs, got):
        want = bs(x)
        assert [h.asdict()["yseq"] for h in hyps] == [h.asdict()["yseq"] for h in want]
        assert [float(h.score) for h in hyps] == [float(h.score) for h in want]
        for hb, hw in zip(hyps, want):
            sb, sw = hb.asdict()["scores"], hw.asdict()["scores"]
            assert sorted(sb) == sorted(sw) and all(float(sb[k]) == float(sw[k]) for k in sw), (sb, sw)
    if beam in (1, 3):                       # and the reference's own best hypothesis
        assert got[0][0].asdict()["yseq"] == g[f"yseq_b{beam}_0"].tolist()


@pytest.mark.parametrize("G,T,lens", [(3, 37, [37, 20, 5]), (5, 37, [37, 20, 5]), (5, 400, [400, 193, 150])])
def test_dec_attn_grouped_equals_single(G, T, lens):
    """avsr_dec_attn with group = G (the beams of one utterance read each memory row once)
    equals the per-hypothesis launch bit for bit, with ragged key lengths per utterance, and
    matches an fp64 softmax attention; with ksplit = 2 (keys of rows >= 193 split over two
    workgroups, merged by the last to arrive) grouped equals single too, and a row's result
    does not depend on the other utterances in the launch"""
    from avsr_amd import ops
    dev = torch.device("cuda")
    U, H = 3, 4
    D = 64 * H
    gen = torch.Generator().manual_seed(G + T)
    mem = torch.randn(U * T, 2 * D, generator=gen).to(dev)
    q = torch.randn(U * G, D, generator=gen).to(dev)
    uidx = torch.arange(U * G, dtype=torch.int32).div(G, rounding_mode="floor").to(dev, torch.int32)
    klen = torch.tensor([lens[u] for u in range(U) for _ in range(G)], dtype=torch.int32, device=dev)
    qd, md = q.double().cpu(), mem.double().cpu()
    for ks in (1, 2):
        outs = []
        for grp in (1, G):
            o = torch.empty(U * G, D, device=dev)
            ops.dec_attn(q, mem[:, :D], mem[:, D:], o, n=U * G, H=H, klen_max=T, k_bstride=T * mem.stride(0),
                         v_bstride=T * mem.stride(0), kidx=uidx, klen=klen, group=grp, ksplit=ks)
            outs.append(o)
        assert torch.equal(outs[0], outs[1])
        # the last utterance alone (its own launch, smaller klen_max) gives the same rows
        o1 = torch.empty(G, D, device=dev)
        u = U - 1
        ops.dec_attn(q[u * G:].contiguous(), mem[u * T:, :D], mem[u * T:, D:], o1, n=G, H=H, klen_max=lens[u],
                     k_bstride=0, v_bstride=0, klen=klen[u * G:].contiguous(), group=G, ksplit=ks)
        assert torch.equal(o1, outs[1][u * G:])
        for i in range(U * G):
            u = i // G
            k = md[u * T:u * T + lens[u], :D].view(-1, H, 64)
            v = md[u * T:u * T + lens[u], D:].view(-1, H, 64)
            s = torch.einsum("hd,jhd->hj", qd[i].view(H, 64), k) * 0.125
            ref = torch.einsum("hj,jhd->hd", torch.softmax(s, -1), v).reshape(D)
            assert (outs[1][i].double().cpu() - ref).abs().max().item() < 1e-5


def test_dec_attn_group_beyond_lds_limit_falls_back():
    """a cross-attention memory longer than the grouped kernel's LDS bound (about 2.7 k frames
    at group 5) runs ungrouped instead of raising, with the same rows bit for bit"""
    dev = torch.device("cuda")
    G, T, H = 5, 3000, 4
    D = 64 * H
    assert not ops.dec_attn_group_fits(T, G) and ops.dec_attn_group_fits(T, 1)
    gen = torch.Generator().manual_seed(11)
    mem = torch.randn(T, 2 * D, generator=gen).to(dev)
    q = torch.randn(G, D, generator=gen).to(dev)
    klen = torch.tensor([T, 2999, 1500, 7, 2800], dtype=torch.int32, device=dev)
    for ks in (1, 2):
        outs = []
        for grp in (1, G):
            o = torch.empty(G, D, device=dev)
            ops.dec_attn(q, mem[:, :D], mem[:, D:], o, n=G, H=H, klen_max=T, k_bstride=0, v_bstride=0, klen=klen,
                         group=grp, ksplit=ks)
            outs.append(o)
        assert torch.equal(outs[0], outs[1])
    qd, md = q.double().cpu(), mem.double().cpu()
    for i in range(G):
        n = int(klen[i])
        s = torch.einsum("hd,jhd->hj", qd[i].view(H, 64), md[:n, :D].view(-1, H, 64)) * 0.125
        ref = torch.einsum("hj,jhd->hd", torch.softmax(s, -1), md[:n, D:].view(-1, H, 64)).reshape(D)
        assert (outs[1][i].double().cpu() - ref).abs().max().item() < 1e-5


def test_decode_graph_workspaces_zeroed_before_capture(g, model):
    """the captured decode step's split-K arrival counters live in the capture stream's
    workspace; it is created (zeroed) eagerly before capture, so a first replay of graph 1 on
    recycled allocator memory full of garbage still decodes the reference's hypotheses, and
    the counters are back at zero afterwards"""
    from avsr_amd import decode as Dm
    dev = torch.device("cuda")
    for s in list(Dm._CAPTURE_STREAMS.values()):         # force a fresh capture stream + workspaces
        for key in [k for k in ops._SKINNY_WS if k[1] == s.cuda_stream]:
            del ops._SKINNY_WS[key]
    Dm._CAPTURE_STREAMS.clear()
    torch.cuda.synchronize()
    junk = torch.full((1 << 26,), -1, dtype=torch.int32, device=dev)      # 256 MiB of 0xFFFFFFFF
    del junk                                                                  # back to the caching allocator
    bs = get_beam_search_decoder(model.avsr, TOKENS, ctc_weight=0.1, beam_size=3)
    got = bs.decode_batch([torch.from_numpy(g["dec_enc_0"]).cuda(), torch.from_numpy(g["dec_enc_1"]).cuda()])
    assert got[0][0].asdict()["yseq"] == g["yseq_b3_0"].tolist()
    assert got[1][0].asdict()["yseq"] == g["yseq_b3_1"].tolist()
    s = Dm._CAPTURE_STREAMS[dev]
    ws = ops._SKINNY_WS[(ops._norm_dev(dev), s.cuda_stream)]
    torch.cuda.synchronize()
    assert int(ws[ops.SKINNY_WS:].view(torch.int32).abs().sum()) == 0


@pytest.mark.parametrize("w", [0.0, 1.0])
@pytest.mark.parametrize("beam", [1, 3])
def test_one_scorer_searches_match_reference(g, model, w, beam):
    """ctc_weight = 0 (decoder alone, no pre-beam) and ctc_weight = 1 (CTC prefix scorer alone
    over the full vocabulary, no decoder step) reproduce every hypothesis the reference returns
    (tests/golden/avsr_ctcw.npz from make_golden_ctcw.py): token sequences in order, total and
    per-scorer scores; batched over both clips = per clip"""
    import os
    c = np.load(os.path.join(os.path.dirname(__file__), "golden", "avsr_ctcw.npz"))
    bs = get_beam_search_decoder(model.avsr, TOKENS, ctc_weight=w, beam_size=beam)
    xs = [torch.from_numpy(g[f"dec_enc_{b}"]).cuda() for b in range(2)]
    batched = bs.decode_batch(xs)
    scorer = "decoder" if w == 0.0 else "ctc"
    for b in range(2):
        key = f"w{w:g}_b{beam}_{b}"
        lens = c[key + "_len"]
        ys = [y.tolist() for y in np.split(c[key + "_yseq"], np.cumsum(lens)[:-1])]
        hyps = [h.asdict() for h in bs(xs[b])]
        assert [h["yseq"] for h in hyps] == ys
        assert set(hyps[0]["scores"]) == {scorer}
        for h, s, s1 in zip(hyps, c[key + "_score"], c[key + "_" + scorer]):
            assert abs(h["score"] - s) <= 1e-4 * abs(s)
            assert abs(h["scores"][scorer] - s1) <= 1e-4 * abs(s1)
        assert [h.asdict()["yseq"] for h in batched[b]] == ys
