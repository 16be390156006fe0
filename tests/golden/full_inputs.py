"""Input recipe of the full-size golden vectors (tests/golden/make_golden_full.py): the tests
regenerate these inputs from their seeds (too large to commit) and check the stored digests."""
C1 = dict(B=8, T=25, lengths=(25,) * 8, seed=2025)
TR = dict(B=2, T=375, lengths=(375, 300), seed=2026)
TR_LABELS = (tuple((7 * i * i + 13 * i + 5) % 5047 + 1 for i in range(40)),
             tuple((11 * i * i + 3 * i + 29) % 5047 + 1 for i in range(31)))
ENC_ROWS = (0, 1, 74, 150, 299, 300, 374)          # frames whose full encoder rows are kept
DEC_ROWS = (0, 1, 20, 31, 40)                      # decoder positions whose logits are kept


# early-ending beam searches (make_golden_endbeam.py): <eos> logit bias offsets, beams, C1 clips
ENDBEAM = dict(offsets=(4.0, 6.0, 8.0), beams=(3, 5), clips=(0, 3, 6))
