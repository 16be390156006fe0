"""Data-parallel inference bookkeeping for the evaluation configs (BASELINE
configs C4 / C5): units (LRS2 utterances, AVCocktail session x chunk segments) are independent,
so ranks take them round-robin, decode them with the HIP engine (`avsr_amd.decode`), and ONE
object gather brings the hypotheses to rank 0, which scores them exactly as
script/evaluation.py does. No collective touches the data path.

Mirrors (script/evaluation.py):
  * `eval_lrs2` (:380-404): corpus WER over normalised (reference, hypothesis) lists
    (jiwer.wer with lists = total word edits / total reference words);
  * `eval_avcocktail` (:405-451): per chunk type, segment outputs sorted by start time, joined,
    `<unk>` removed, one WER against the joined labels; `len(label_text.split())` words;
  * `main` aggregation: LRS2 '*' = plain mean of the 9 set WERs (:539-547); AVCocktail '*' =
    word-count weighted mean per chunk type (`extend([wer] * num_words)`, :556-570);
  * stdout lines `WER {set_id}: x.xxxx`, `Average WER: x.xxxx`, `WER {set_id} {chunk}: x.xxxx`,
    `Average WER {chunk}: x.xxxx`.
jiwer (pinned by the reference's requirements, absent here) is restated as word-level
Levenshtein distance after its default transform (collapse whitespace, strip, split on spaces).
"""
from collections import OrderedDict

import torch.distributed as dist


def _words(s):
    return " ".join(s.split()).split(" ") if s.strip() else []


def word_edits(reference, hypothesis):
    """(substitutions + deletions + insertions, reference words) of one sentence pair."""
    r, h = _words(reference), _words(hypothesis)
    prev = list(range(len(h) + 1))
    for i in range(1, len(r) + 1):
        cur = [i] + [0] * len(h)
        for j in range(1, len(h) + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (r[i - 1] != h[j - 1]))
        prev = cur
    return prev[len(h)], len(r)


def wer(reference, hypothesis):
    """jiwer.wer semantics: strings or equal-length lists of strings (corpus-level ratio)."""
    if isinstance(reference, str):
        reference, hypothesis = [reference], [hypothesis]
    if len(reference) != len(hypothesis):
        raise ValueError("reference and hypothesis lists differ in length")
    e = n = 0
    for r, h in zip(reference, hypothesis):
        de, dn = word_edits(r, h)
        e, n = e + de, n + dn
    if n == 0:
        raise ValueError("one or more references are empty strings")
    return e / n


def shard(units, rank, world):
    """round-robin assignment of independent units (order-preserving within a rank)."""
    return [(i, u) for i, u in enumerate(units) if i % world == rank]


def gather_to_rank0(local, world):
    """local: list of (unit index, result). Rank 0 gets every result in unit order; others None."""
    if world == 1:
        return [r for _, r in sorted(local, key=lambda t: t[0])]
    parts = [None] * world if dist.get_rank() == 0 else None
    dist.gather_object(local, parts, dst=0)
    if dist.get_rank() != 0:
        return None
    return [r for _, r in sorted((t for p in parts for t in p), key=lambda t: t[0])]


def run_sharded(units, infer, rank=0, world=1, infer_batch=None, batch=8):
    """decode this rank's share with `infer(unit) -> text` (or `infer_batch(list of units) ->
    texts`, `batch` units at a time: the engine's batched beam search); rank 0 returns all
    texts in unit order."""
    mine = shard(units, rank, world)
    if infer_batch is None:
        local = [(i, infer(u)) for i, u in mine]
    else:
        local = []
        for s in range(0, len(mine), batch):
            chunk = mine[s:s + batch]
            local += list(zip([i for i, _ in chunk], infer_batch([u for _, u in chunk])))
    return gather_to_rank0(local, world)


def lrs2_set_wer(labels, outputs, norm=lambda s: s):
    """eval_lrs2: normalise (after removing <unk>) and score the lists."""
    return wer([norm(l.replace("<unk>", "")) for l in labels], [norm(o.replace("<unk>", "")) for o in outputs])


def avcocktail_labels(captions, norm=lambda s: s):
    """eval_avcocktail's label side (script/evaluation.py:410-434): captions = [(start, end,
    text)] in file order; empty texts skipped; the session window is [min start, max end];
    label texts sorted by (start, text) as `sorted(zip(...))` does, joined and normalised.
    Returns (label_text, (window_start, window_end))."""
    kept = [(a, b, t) for a, b, t in captions if t != ""]
    if not kept:
        raise ValueError("no non-empty caption")
    start, end = min(a for a, _, _ in kept), max(b for _, b, _ in kept)
    text = norm(" ".join(t for _, t in sorted((a, t) for a, _, t in kept)))
    return text, (start, end)


def in_window(seg_start, seg_end, window):
    """a segment is scored unless it starts more than 1 s before the labelled span or ends more
    than 1 s after it (script/evaluation.py:443-444)"""
    return not (seg_start + 1 < window[0] or seg_end - 1 > window[1])


def avcocktail_chunk_wer(label_text, segments, norm=lambda s: s, window=None):
    """eval_avcocktail for one chunk type: segments = [(start_time, output text)] or
    [(start_time, end_time, output text)]; with `window` (see avcocktail_labels) segments outside
    it are dropped (callers should not decode them at all). Outputs are ordered as
    `sorted(zip(start_times, outputs))`: by start, ties by text."""
    segs = [(s[0], s[1], s[2]) if len(s) == 3 else (s[0], None, s[1]) for s in segments]
    if window is not None:
        segs = [x for x in segs if in_window(x[0], x[1] if x[1] is not None else x[0], window)]
    outs = [o for _, o in sorted((a, o) for a, _, o in segs)]
    return wer(reference=label_text, hypothesis=norm(" ".join(outs).replace("<unk>", "")))


def lrs2_average(set_wers):
    """set_wers: OrderedDict set_id -> WER. Returns (lines, average) as the reference prints."""
    lines = [f"WER {k}: {v:.4f}" for k, v in set_wers.items()]
    avg = sum(set_wers.values()) / len(set_wers)
    return lines + [f"Average WER: {avg:.4f}"], avg


def avcocktail_average(per_set):
    """per_set: OrderedDict set_id -> ({chunk_type: WER}, num_words). Word-weighted averages."""
    lines, acc = [], OrderedDict()
    for set_id, (wers, nw) in per_set.items():
        for chunk, w in wers.items():
            acc.setdefault(chunk, []).extend([w] * nw)     # same summation as the reference
            lines.append(f"WER {set_id} {chunk}: {w:.4f}")
    avgs = OrderedDict((c, sum(v) / len(v)) for c, v in acc.items())
    return lines + [f"Average WER {c}: {v:.4f}" for c, v in avgs.items()], avgs
