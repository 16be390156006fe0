"""Sharded evaluation bookkeeping: jiwer-equivalent WER known answers, the
reference's aggregation lines, and a world_size-2 gloo run whose gathered hypotheses and WER
equal the single-process result."""
import os
import socket
from collections import OrderedDict

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from avsr_amd import evaluate as E


@pytest.mark.parametrize("ref,hyp,want", [
    ("a b c", "a b c", 0.0),
    ("a b c", "a x c", 1 / 3),
    ("a b c", "a c", 1 / 3),                 # deletion
    ("a b c", "a b c d e", 2 / 3),           # insertions
    ("the cat sat", "", 1.0),
    ("  a   b ", "a b", 0.0),                # whitespace collapsed / stripped
])
def test_wer_known_answers(ref, hyp, want):
    assert E.wer(ref, hyp) == pytest.approx(want)


def test_wer_corpus_ratio_not_mean():
    # jiwer with lists: total edits / total reference words
    assert E.wer(["a b c d", "e"], ["a b c d", "x"]) == pytest.approx(1 / 5)
    with pytest.raises(ValueError):
        E.wer([""], ["a"])


def test_avcocktail_sorting_and_unk():
    segs = [(3.0, "c d"), (1.0, "a <unk>b")]
    assert E.avcocktail_chunk_wer("a b c d", segs) == pytest.approx(0.0)


def test_aggregation_lines():
    lines, avg = E.lrs2_average(OrderedDict([("test", 0.1), ("test_snr_0_interferer_2", 0.3)]))
    assert lines == ["WER test: 0.1000", "WER test_snr_0_interferer_2: 0.3000", "Average WER: 0.2000"]
    lines, avgs = E.avcocktail_average(OrderedDict([
        ("video_0", ({"asd_chunk": 0.5, "gold_chunk": 0.25}, 10)),
        ("video_1", ({"asd_chunk": 0.2, "gold_chunk": 0.1}, 30))]))
    assert avgs["asd_chunk"] == pytest.approx((0.5 * 10 + 0.2 * 30) / 40)
    assert lines[-2:] == [f"Average WER asd_chunk: {avgs['asd_chunk']:.4f}",
                          f"Average WER gold_chunk: {avgs['gold_chunk']:.4f}"]
    assert lines[0] == "WER video_0 asd_chunk: 0.5000"


UNITS = [f"u{i}" for i in range(11)]          # 11 units over 2 ranks: uneven shards


def _infer(u):
    return f"hyp {u}"


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = E.shard(UNITS, rank, world)
        out = E.run_sharded(UNITS, _infer, rank, world)
        q.put((rank, [i for i, _ in mine], out))
    finally:
        dist.destroy_process_group()


def test_sharded_eval_gloo_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (idx, out)) for r, idx, out in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(res[0][0] + res[1][0]) == list(range(len(UNITS)))      # every unit exactly once
    assert set(res[0][0]).isdisjoint(res[1][0])
    assert res[1][1] is None
    single = E.run_sharded(UNITS, _infer)
    assert res[0][1] == single
    refs = [f"hyp {u}" for u in UNITS]
    assert E.wer(refs, res[0][1]) == E.wer(refs, single) == 0.0


def test_avcocktail_window_and_label_order():
    """eval_avcocktail (script/evaluation.py:406-453): empty captions skipped, labels sorted by
    (start, text), segments outside [start - 1, end + 1] dropped, outputs sorted by (start, text)."""
    caps = [(5.0, 7.0, "c d"), (1.0, 3.0, "a b"), (4.0, 4.5, ""), (1.0, 2.0, "a a")]
    text, win = E.avcocktail_labels(caps)
    assert text == "a a a b c d" and win == (1.0, 7.0)
    assert E.in_window(0.5, 3.0, win) and not E.in_window(-0.5, 3.0, win)
    assert E.in_window(6.0, 8.0, win) and not E.in_window(6.0, 8.5, win)
    segs = [(5.0, 7.0, "c d"), (1.0, 2.0, "a a a b"), (-2.0, 0.0, "zz"), (6.0, 9.0, "yy")]
    assert E.avcocktail_chunk_wer(text, segs, window=win) == pytest.approx(0.0)
    assert E.avcocktail_chunk_wer(text, segs) > 0.0
    # ties on start time are broken by the text, like sorted(zip(starts, outputs))
    assert E.avcocktail_chunk_wer("a b", [(1.0, "b"), (1.0, "a")]) == pytest.approx(0.0)


def test_run_sharded_batched_single_process():
    units = list(range(11))
    got = E.run_sharded(units, None, infer_batch=lambda us: [str(u * 2) for u in us], batch=4)
    assert got == [str(u * 2) for u in units]
