"""Deferred column-sum finalisation (avsr_colsum_defer / avsr_colsum_flush): bias and
LayerNorm parameter gradients finalised by one batched launch equal the immediate per-call
finalise passes bit for bit (same reduction order), across more passes than one batch holds."""
import pytest
import torch

from avsr_amd import ops

pytestmark = pytest.mark.gpu


def _run(dev, defer):
    g = torch.Generator().manual_seed(3)
    dys = [torch.randn(777, n, generator=g).to(dev, torch.bfloat16) for n in (1024, 3072, 256) * 12]
    x = torch.randn(777, 1024, generator=g).to(dev, torch.bfloat16)
    gamma, beta = torch.randn(1024, generator=g).to(dev), torch.randn(1024, generator=g).to(dev)
    dbs = [torch.zeros(d.shape[1], device=dev) for d in dys]
    dg, dbt = torch.zeros(1024, device=dev), torch.zeros(1024, device=dev)
    prev = ops.colsum_defer(defer)
    try:
        for d, db in zip(dys, dbs):
            ops.ew_bwd(d, db=db, drop_p=0.1, seed=5)
        _, mean, rstd = ops.layernorm_fwd(x, gamma, beta, 1e-5)
        ops.layernorm_bwd(dys[0], x, gamma, mean, rstd, dgamma=dg, dbeta=dbt)
        if defer:
            assert float(dbs[0].abs().sum()) == 0.0     # nothing finalised before the flush
        ops.colsum_flush()
    finally:
        ops.colsum_defer(prev)
    torch.cuda.synchronize()
    return dbs + [dg, dbt]


def test_deferred_colsum_matches_immediate(dev):
    a, b = _run(dev, False), _run(dev, True)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
