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


def _emulate_fused_mlp(frags, bias, x, t):
    """The arithmetic of k_mlp_fwd (gsd_mlp.hip) lane by lane on the CPU, from the packed buffers alone:
    v_mfma_f32_32x32x16_bf16's operand maps (lane l = 32 h + r holds A[r][8 h + j] and B[8 h + j][r]; register
    `reg` of the accumulator is D[(reg&3) + 8 (reg>>2) + 4 h][r]), the accumulator registers 8 s .. 8 s + 7
    reused as the next layer's B fragment of k-step 2 rb + s, bf16 rounding where the kernel rounds.  x (32,3),
    t (32,): one wave."""
    import numpy as np

    from gsd_amd.deform_mlp import positional_encoding
    bf = lambda a: torch.as_tensor(a, dtype=torch.float32).to(torch.bfloat16).float().numpy()  # noqa: E731
    F = frags.float().numpy().reshape(-1, 64, 8)   # [fragment][lane][j]
    Bz = bias.numpy()
    ks_of = [6, 16, 16, 16, 16, 20, 16, 16, 16]
    rb_of = [8] * 8 + [2]
    enc = torch.cat((positional_encoding(torch.as_tensor(x)), positional_encoding(torch.as_tensor(t)[:, None])), -1)
    enc = np.concatenate((bf(enc), np.zeros((32, 12), np.float32)), 1)   # (32 Gaussians, 96)
    lanes = np.arange(64)
    h, r = lanes >> 5, lanes & 31
    # B fragments: bfr[ks][lane][j]
    enc_fr = np.stack([enc[r[:, None], 16 * ks + 8 * h[:, None] + np.arange(8)[None, :]] for ks in range(6)])
    act = enc_fr
    fo = bo = 0
    regs = np.arange(16)
    for L in range(9):
        KS, RB = ks_of[L], rb_of[L]
        B = np.concatenate((enc_fr[:4], act)) if L == 5 else act
        acc = np.zeros((RB, 64, 16), np.float64)
        for ks in range(KS):
            # B matrix (16 x 32) of this k-step from the lanes' fragments
            Bm = np.zeros((16, 32))
            Bm[8 * h[:, None] + np.arange(8)[None, :], r[:, None]] = B[ks]
            for rb in range(RB):
                A = np.zeros((32, 16))
                A[r[:, None], 8 * h[:, None] + np.arange(8)[None, :]] = F[fo + ks * RB + rb]
                D = A @ Bm                                   # (32 rows, 32 Gaussians)
                acc[rb] += D[(regs[None, :] & 3) + 8 * (regs[None, :] >> 2) + 4 * h[:, None], r[:, None]]
        fo += KS * RB
        bl = Bz[bo: bo + RB * 32].reshape(RB, 2, 16)
        bo += RB * 32
        v = acc.astype(np.float32) + bl[:, h, :]            # (RB, lane, reg)
        if L < 8:
            v = bf(np.maximum(v, 0.0))
            act = np.stack([v[rb, :, 8 * s: 8 * s + 8] for rb in range(RB) for s in range(2)])   # (16, lane, 8)
        else:
            out = np.zeros((32, 64), np.float32)
            f = 32 * np.arange(RB)[:, None, None] + ((regs & 3) + 8 * (regs >> 2))[None, None, :] + 4 * h[None, :, None]
            out[np.broadcast_to(r[None, :, None], f.shape), f] = bf(v)
            return out[:, :58]


def test_fused_mlp_packing_emulated():
    """pack_fused_mlp's layout and k permutation, checked by emulating the kernel's MFMA operand maps on the CPU
    (no GPU needed): the emulated outputs equal the module's float32 forward within bf16 rounding."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF, pack_fused_mlp
    torch.manual_seed(3)
    net = DirectTemporalNeRF()
    with torch.no_grad():   # larger weights than the default init so every layer's ReLU pattern matters
        for p in net.parameters():
            p.mul_(2.0)
    frags, bias = pack_fused_mlp(net)
    x = torch.rand(32, 3) * 2 - 1
    t = torch.full((32,), 0.4)
    got = torch.as_tensor(_emulate_fused_mlp(frags, bias, x.numpy(), t.numpy()))
    with torch.no_grad():
        ref = torch.cat(net(x, t[:, None], 5000), -1)
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 3e-2, err
    # and a wrong permutation is caught: natural k order in the hidden layers breaks it
    import gsd_amd.deform_mlp as dm
    saved = dm._PERM16
    try:
        dm._PERM16 = tuple(range(16))
        f2, b2 = pack_fused_mlp(net)
    finally:
        dm._PERM16 = saved
    bad = torch.as_tensor(_emulate_fused_mlp(f2, b2, x.numpy(), t.numpy()))
    assert float((bad - ref).abs().max() / ref.abs().max()) > 0.1


# ---- DirectTemporalNeRF_se3 (scene/gaussian_model.py:99-173) against the reference's own run (tests/golden/mlp_se3.npz)
def se3net_weights(named_params, seed=82):
    """The fixture's weights, regenerated as tests/golden/make_golden.py:se3net_weights draws them."""
    import math
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in named_params:
            fan_in = p.shape[1] if p.dim() == 2 else p.shape[0]
            if name.endswith("bias"):
                fan_in = 256
            p.copy_((torch.rand(p.shape, generator=g) * 2.0 - 1.0) / math.sqrt(fan_in))


def se3net_from_fixture(device="cpu"):
    from conftest import golden
    from gsd_amd.deform_mlp import DirectTemporalNeRF_se3
    g = golden("mlp_se3.npz")
    net = DirectTemporalNeRF_se3()
    se3net_weights(list(net.named_parameters()))
    return net.to(device), g


def _rel(a, b):
    a, b = torch.as_tensor(a).detach().double(), torch.as_tensor(b).detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def test_se3net_parameter_names_are_the_references():
    from gsd_amd.deform_mlp import DirectTemporalNeRF_se3
    sd = DirectTemporalNeRF_se3().state_dict()
    assert list(sd)[:2] == ["_time.0.weight", "_time.0.bias"] and list(sd)[-4:] == ["_w.weight", "_w.bias",
                                                                                    "_v.weight", "_v.bias"]
    assert sd["_time.0.weight"].shape == (256, 4) and sd["_time.5.weight"].shape == (256, 259)


def test_se3net_matches_reference_fixture_cpu():
    """The torch path (CPU): query_time's w / v, the transform, the zeros before 3000 and the autograd gradients of
    the moved points against the reference's DirectTemporalNeRF_se3 run."""
    net, g = se3net_from_fixture()
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    t = torch.from_numpy(g["t"])
    w, v = net.query_time(x, t)
    assert _rel(w, g["w"]) <= 1e-5 and _rel(v, g["v"]) <= 1e-5
    T = net(x, t, 5000)
    assert float((T.detach() - torch.from_numpy(g["T"])).abs().max()) <= 1e-6
    z = net(x.detach(), t, 2000)
    assert z.shape == g["zero2000"].shape and not z.any()
    moved = (T @ torch.cat([x, torch.ones_like(x[:, :1])], 1)[..., None])[:, :3, 0]
    assert float((moved.detach() - torch.from_numpy(g["moved"])).abs().max()) <= 1e-6
    params = dict(net.named_parameters())
    names = [str(n) for n in g["names"]]
    grads = torch.autograd.grad((moved * torch.from_numpy(g["upstream"])).sum(), [x] + [params[n] for n in names])
    assert _rel(grads[0], g["grad:x"]) <= 1e-4
    for n, gr in zip(names, grads[1:]):
        assert _rel(gr, g["grad:" + n]) <= 1e-4, n


def test_se3net_padded_weights_compute_the_same_network_cpu():
    """The structurally-zero embedding into DirectTemporalNeRF's layout (what the HIP kernels take), evaluated by
    the reference architecture's torch restatement on [enc(x), enc(t)]: the same w / v."""
    from gsd_amd.deform_mlp import positional_encoding
    net, g = se3net_from_fixture()
    ws, bs = net._padded()
    assert [tuple(w.shape) for w in ws] == [(256, 84)] + [(256, 256)] * 4 + [(256, 319)] + [(256, 256)] * 2 + \
        [(3, 256), (3, 256), (4, 256), (48, 256)]
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["t"])
    ex = positional_encoding(x, 10)
    h = torch.cat([ex, positional_encoding(t, 10)], -1)
    for i in range(8):
        h = torch.relu(h @ ws[i].t() + bs[i])
        if i == 4:
            h = torch.cat([ex, h], -1)
    w = h @ ws[8].t() + bs[8]
    v = h @ ws[9].t() + bs[9]
    assert _rel(w, g["w"]) <= 1e-5 and _rel(v, g["v"]) <= 1e-5
