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


def test_split_k_gradients_match_plain_linear_layers():
    """The module's backward (gsd_amd.deform_mlp._Linear: bias + ReLU fused, split-K weight gradient over
    8192-row chunks plus a remainder, the four heads as one GEMM) against the same network written with
    torch.nn.functional.linear and autograd, on more rows than two chunks."""
    import torch.nn.functional as F

    from gsd_amd.deform_mlp import DirectTemporalNeRF, positional_encoding
    torch.manual_seed(1)
    net = DirectTemporalNeRF().double()
    P = 2 * 8192 + 37
    x = torch.randn(P, 3, dtype=torch.float64)
    t = torch.full((P, 1), 0.21, dtype=torch.float64)
    w = [torch.randn(P, n, dtype=torch.float64) for n in (3, 3, 4, 48)]

    def plain(xx):
        ex, et = positional_encoding(xx), positional_encoding(t)
        h = torch.cat((ex, et), -1)
        for i, layer in enumerate(net._time):
            h = F.relu(F.linear(h, layer.weight, layer.bias))
            if i in net.skips:
                h = torch.cat((ex, h), -1)
        return [F.linear(h, m.weight, m.bias) for m in (net._time_out, net._time_out_scale, net._time_out_rot,
                                                        net._time_out_shs)]

    grads = {}
    for name, fn in (("fused", lambda xx: net(xx, t, 5000)), ("plain", plain)):
        net.zero_grad()
        xx = x.clone().requires_grad_(True)
        outs = fn(xx)
        sum((o * wi).sum() for o, wi in zip(outs, w)).backward()
        grads[name] = [xx.grad] + [p.grad.clone() for p in net.parameters()]
    # the module returns float32 outputs (as the reference's .float()), so its gradients carry float32 rounding
    for a, b in zip(grads["fused"], grads["plain"]):
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max())
