"""FlatGrads' stale-view protocol (CPU): after invalidate() the next gradient producer stores instead of
adding; autograd producers zero a stale view first; views nothing wrote hold zero at settle(); gradients
written by hand with no backward stand as written."""
from __future__ import annotations

import torch


def _params():
    return [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(5, 1))]


def test_claim_store_then_add():
    from gsd_amd.parallel import FlatGrads
    ps = _params()
    f = FlatGrads(ps)
    f.slab.fill_(7.0)
    f.invalidate()
    assert f.claim(ps) is False          # all stale: the producer stores
    assert f.claim(ps) is True           # a second producer in the same step adds
    f.invalidate()
    assert f.claim(ps[:1]) is False
    f.settle()                            # ps[1] got nothing: zero gradient
    assert torch.equal(ps[1].grad, torch.zeros(5, 1)) and float(ps[0].grad.sum()) == 7.0 * 15


def test_mixed_claim_zeroes_stale_views():
    from gsd_amd.parallel import FlatGrads
    ps = _params()
    f = FlatGrads(ps)
    f.slab.fill_(3.0)
    f.invalidate()
    assert f.claim(ps[:1]) is False
    assert f.claim(ps) is True            # ps[0] valid, ps[1] stale -> ps[1] zeroed, then added into
    assert torch.equal(ps[1].grad, torch.zeros(5, 1))


def test_autograd_producer_after_invalidate():
    from gsd_amd.parallel import FlatGrads
    ps = _params()
    f = FlatGrads(ps)
    f.slab.fill_(5.0)
    f.invalidate()
    (ps[0] * 2.0).sum().backward()        # AccumulateGrad into a stale view: zeroed by the hook first
    assert torch.equal(ps[0].grad, torch.full((5, 3), 2.0))
    assert ps[0].grad.data_ptr() == f.views[0].data_ptr()
    f.settle()
    assert torch.equal(ps[1].grad, torch.zeros(5, 1))


def test_hand_written_gradients_stand():
    from gsd_amd.parallel import FlatGrads
    ps = _params()
    f = FlatGrads(ps)
    f.invalidate()
    ps[0].grad.copy_(torch.ones(5, 3))
    ps[1].grad.copy_(torch.ones(5, 1))
    f.settle()
    assert float(f.slab.sum()) == 20.0


def test_settle_reports_parameters_without_gradient():
    """settle() returns the parameters nothing wrote (torch's grad None: FusedAdam skips them and does not
    advance their step); they stay "no gradient" until a producer writes them, also across a second settle()
    in the same step and across steps without invalidate()."""
    from gsd_amd.parallel import FlatGrads
    ps = _params()
    f = FlatGrads(ps)
    f.slab.fill_(4.0)
    f.invalidate()
    (ps[0] * 3.0).sum().backward()
    assert f.settle() == {id(ps[1])}
    assert torch.equal(ps[1].grad, torch.zeros(5, 1))
    assert f.settle() == {id(ps[1])}      # idempotent: its zeroing is not a hand-written gradient
    (ps[0] * 1.0).sum().backward()        # no invalidate: ps[0] accumulates, ps[1] still has none
    assert f.settle() == {id(ps[1])} and float(ps[0].grad.sum()) == 4.0 * 15
    (ps[1] * 2.0).sum().backward()
    assert f.settle() == set() and torch.equal(ps[1].grad, torch.full((5, 1), 2.0))
