"""The deformation network (gsd_amd.deform_mlp) against an independent float64
restatement (oracle/deform_mlp_ref.py) and the reference's parameter layout (offset_model.pth keys and
shapes, scene/gaussian_model.py:242-276).  The reference module itself cannot be imported here (its file
needs plyfile / FrEIA / simple_knn), so parity is pinned by restatement; CPU."""
from __future__ import annotations

import torch

from conftest import PKG  # noqa: F401


def test_parameter_layout_matches_reference():
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    sd = DirectTemporalNeRF().state_dict()
    expect = {"_time.0.weight": (256, 84)}
    for i in range(1, 8):
        expect[f"_time.{i}.weight"] = (256, 256 + (63 if i == 5 else 0))
    for n, o in (("_time_out", 3), ("_time_out_scale", 3), ("_time_out_rot", 4), ("_time_out_shs", 48)):
        expect[f"{n}.weight"] = (o, 256)
    for k, shape in expect.items():
        assert tuple(sd[k].shape) == shape, k
        assert tuple(sd[k.replace("weight", "bias")].shape) == (shape[0],)
    assert len(sd) == 2 * len(expect)
    assert sum(v.numel() for k, v in sd.items() if k.endswith("weight")) == 84 * 256 + 6 * 256 * 256 + 319 * 256 + 58 * 256


def test_forward_matches_restatement_and_zero_phase():
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    from oracle import deform_mlp_ref
    torch.manual_seed(0)
    net = DirectTemporalNeRF()
    x = torch.randn(300, 3)
    t = torch.full((300, 1), 0.37)
    for it in (0, 2999):
        outs = net(x, t, it)
        assert [tuple(o.shape) for o in outs] == [(300, 3), (300, 3), (300, 4), (300, 48)]
        assert all(float(o.abs().max()) == 0.0 for o in outs)
    got = net(x, t, 5000)
    ref = deform_mlp_ref.forward(net.state_dict(), x, t, 5000)
    for g, r in zip(got, ref):
        assert float((g.double() - r).abs().max()) <= 1e-5 * max(1.0, float(r.abs().max()))
