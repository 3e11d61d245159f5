"""The deformation network (gsd_amd.deform_mlp) against an independent float64
restatement (oracle/deform_mlp_ref.py) and the reference's parameter layout (offset_model.pth keys and
shapes, scene/gaussian_model.py:242-276).  The reference module itself cannot be imported here (its file
needs plyfile / FrEIA / simple_knn), so parity is pinned by restatement; CPU."""
from __future__ import annotations

import numpy as np
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


# ---- k_mlp_fwd_fused16 / k_mlp_bwd_chain16 operand maps (gsd_mlp_train.hip, round 6), emulated on the CPU ----
# The lane maps of v_mfma_f32_16x16x32_bf16 (cdna_hip_programming.md §3): lane l holds A[l & 15][8 (l >> 4) + j],
# B[8 (l >> 4) + j][l & 15], and C[4 (l >> 4) + i][l & 15].  The emulation restates k_mlp_pack's m16 fragment index,
# the kernels' B operands (natural or the accumulator order), their epilogue / mask word layout, and multiplies in
# float64 (the BF16x6 split is the same as the 32-wide kernels' and is not what is checked here).
_LQ, _LC = np.arange(64) >> 4, np.arange(64) & 15


def _pack_m16(A, perm_from):
    """k_mlp_pack with m16: frag[ks, rb, lane, j] = A[16 rb + (lane & 15), kcol(ks, lane >> 4, j)]."""
    M, K = A.shape
    out = np.zeros((K // 32, M // 16, 64, 8))
    for ks in range(K // 32):
        for j in range(8):
            k = 32 * ks + (16 * (j >> 2) + 4 * _LQ + (j & 3) if ks >= perm_from else 8 * _LQ + j)
            for rb in range(M // 16):
                out[ks, rb, :, j] = A[16 * rb + _LC, k]
    return out


def _mfma16(frag, breg):
    """(64, 8) A fragment x (64, 8) B operand -> (64, 4) accumulator registers of one 16 x 16 x 32 product."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for j in range(8):
        A[_LC, 8 * _LQ + j] = frag[:, j]
        B[8 * _LQ + j, _LC] = breg[:, j]
    C = A @ B
    return np.stack([C[4 * _LQ + i, _LC] for i in range(4)], -1)


def _run16(frags, operands):
    """A layer's k-steps: acc[rb] (64, 4) = sum over k-steps of frag[ks, rb] x operands[ks]."""
    KS, RB = frags.shape[:2]
    acc = np.zeros((RB, 64, 4))
    for ks in range(KS):
        for rb in range(RB):
            acc[rb] += _mfma16(frags[ks, rb], operands[ks])
    return acc


def _epilogue16(acc, bias):
    """fused16_epilogue: act[k][lane][4 a + i] = relu(acc[2 k + a] + bias[16 (2 k + a) + 4 q + i]) and the ReLU words
    (word 2 k + (q & 1), lane halves combined as __shfl_xor(w, 32) does)."""
    act = np.zeros((8, 64, 8))
    bits = np.zeros((8, 64), dtype=np.int64)
    for k in range(8):
        w = np.zeros(64, dtype=np.int64)
        for a in range(2):
            for i in range(4):
                y = np.maximum(acc[2 * k + a][:, i] + bias[16 * (2 * k + a) + 4 * _LQ + i], 0.0)
                act[k][:, 4 * a + i] = y
                w |= (y > 0).astype(np.int64) << (8 * a + i)
        w <<= 4 * (_LQ >> 1)
        bits[k] = w | w[np.arange(64) ^ 32]
    return act, bits


def _padded_layers(net):
    """The kernels' A matrices in float64: layer 0 [enc(x) 63 | 0 | enc(t) 21 | 0 x 11], layer 5 [enc(x) 63 | 0 | h
    256], the heads' 58 rows padded to 64; and the biases (heads padded)."""
    Ws = [l.weight.detach().double().numpy() for l in net._time]
    bs = [l.bias.detach().double().numpy() for l in net._time]
    A = []
    for i, w in enumerate(Ws):
        if i == 0:
            a = np.zeros((256, 96))
            a[:, :63], a[:, 64:85] = w[:, :63], w[:, 63:]
        elif i == 5:
            a = np.zeros((256, 320))
            a[:, :63], a[:, 64:] = w[:, :63], w[:, 63:]
        else:
            a = w
        A.append(a)
    heads = (net._time_out, net._time_out_scale, net._time_out_rot, net._time_out_shs)
    wh = np.zeros((64, 256))
    wh[:58] = torch.cat([m.weight for m in heads]).detach().double().numpy()
    bh = np.zeros(64)
    bh[:58] = torch.cat([m.bias for m in heads]).detach().double().numpy()
    return A + [wh], bs + [bh]


def test_fused16_and_chain16_maps_emulated():
    """k_mlp_fwd_fused16's and k_mlp_bwd_chain16's operand maps, emulated lane by lane for one wave of 16 Gaussians:
    the m16 packing (natural and accumulator-order k, the transposed W^T with layer 5's row offset), the B operands
    chained from the accumulators with no lane movement, the ReLU words (checked against k_mlp_fwd_fused's layout:
    word 2 rb + h, bit 4 q4 + i = row 32 rb + 8 q4 + 4 h + i) and the chain's mask read back from the words' rows.
    The heads and the encoding's gradient equal float64 autograd of the network."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF, positional_encoding
    torch.manual_seed(12)
    net = DirectTemporalNeRF().double()
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(2.0)
    x = torch.rand(16, 3, dtype=torch.float64) * 2 - 1
    t = torch.full((16, 1), 0.45, dtype=torch.float64)
    ex = positional_encoding(x).detach().requires_grad_(True)
    et = positional_encoding(t)
    # float64 reference: heads and d(sum(heads . wg)) / d enc(x)
    h = torch.cat((ex, et), -1)
    hs = []
    for i, layer in enumerate(net._time):
        h = torch.relu(layer(h))
        hs.append(h)
        if i in net.skips:
            h = torch.cat((ex, h), -1)
    heads = (net._time_out, net._time_out_scale, net._time_out_rot, net._time_out_shs)
    ref = torch.cat([m(h) for m in heads], -1)
    wg = torch.randn(16, 58, dtype=torch.float64, generator=torch.Generator().manual_seed(3))
    (ref * wg).sum().backward()
    ref_dE = ex.grad.numpy()
    A, b = _padded_layers(net)
    E = np.zeros((64, 16))
    E[:63] = ex.detach().numpy().T
    ET = np.zeros((32, 16))
    ET[:21] = et.numpy().T
    # ---- forward (k_mlp_fwd_fused16) ----
    xe = [E[32 * s + 8 * _LQ[:, None] + np.arange(8)[None, :], _LC[:, None]] for s in range(2)]
    xt = ET[8 * _LQ[:, None] + np.arange(8)[None, :], _LC[:, None]]
    acc = _run16(_pack_m16(A[0], 1 << 30), [xe[0], xe[1], xt])
    words = {}
    for l in range(1, 8):
        act, bits = _epilogue16(acc, b[l - 1])
        words[l] = bits   # h_l's ReLU words
        ops = ([xe[0], xe[1]] if l == 5 else []) + [act[k] for k in range(8)]
        act7 = act   # layer 7's B operand (h_7), for the negative check below
        acc = _run16(_pack_m16(A[l], 2 if l == 5 else 0), ops)
    act, bits = _epilogue16(acc, b[7])
    words[8] = bits
    # a wrong k order is caught: layer 7 packed in the natural order (its B operand is in the accumulator order)
    bad, _ = _epilogue16(_run16(_pack_m16(A[7], 1 << 30), [act7[k] for k in range(8)]), b[7])
    assert np.abs(bad - act).max() > 0.1 * np.abs(act).max()
    ho = _run16(_pack_m16(A[8], 0), [act[k] for k in range(8)])
    got = np.zeros((16, 64))
    for r in range(4):
        for i in range(4):
            got[_LC, 16 * r + 4 * _LQ + i] = ho[r][:, i] + b[8][16 * r + 4 * _LQ + i]
    ref = ref.detach().numpy()
    np.testing.assert_allclose(got[:, :58], ref, rtol=0, atol=1e-9 * float(np.abs(ref).max()))
    # the words in k_mlp_fwd_fused's layout, from the float64 hidden outputs
    for l in range(1, 9):
        hl = hs[l - 1].detach().numpy()   # (16, 256): h_l
        for k in range(8):
            for hh in range(2):
                lanes = np.where((_LQ & 1) == hh)[0]
                for cc in range(16):
                    want = sum(int(hl[cc, 32 * k + 8 * (bit >> 2) + 4 * hh + (bit & 3)] > 0) << bit
                               for bit in range(16))
                    assert all(words[l][k][lanes[lanes & 15 == cc]] == want), (l, k, hh, cc)

    # ---- backward chain (k_mlp_bwd_chain16) ----
    def rows16(words_l):   # the [16][Gaussian] u16 rows chain16_words copies to LDS: row 2 k + h
        rows = np.zeros((16, 16), dtype=np.int64)
        for k in range(8):
            for ln in range(64):
                rows[2 * k + (_LQ[ln] & 1), _LC[ln]] = words_l[k][ln]
        return rows

    def mask(acc, rows):   # chain16_mask
        out = np.zeros((8, 64, 8))
        for k in range(8):
            wk = rows[2 * k + (_LQ & 1), _LC] >> (4 * (_LQ >> 1))
            for a in range(2):
                for i in range(4):
                    out[k][:, 4 * a + i] = np.where((wk >> (8 * a + i)) & 1, acc[2 * k + a][:, i], 0.0)
        return out

    g8 = np.zeros((64, 16))
    g8[:58] = wg.numpy().T
    gops = [g8[32 * s + 8 * _LQ[:, None] + np.arange(8)[None, :], _LC[:, None]] for s in range(2)]
    acc = _run16(_pack_m16(A[8].T, 1 << 30), gops)   # W8^T (256 x 64), natural k
    act = mask(acc, rows16(words[8]))                 # g7
    dE = None
    for L in range(7, 0, -1):
        if L == 5:   # W5^T's enc(x) rows (0-63) times g5
            he = _run16(_pack_m16(A[5].T[:64], 0), [act[k] for k in range(8)])
            dE = he
        AT = A[L].T[64:] if L == 5 else A[L].T   # layer 5: the h rows (m_off 64)
        acc = _run16(_pack_m16(AT, 0), [act[k] for k in range(8)])
        act = mask(acc, rows16(words[L]))        # g_{L-1}
    dE = dE + _run16(_pack_m16(A[0].T[:64], 0), [act[k] for k in range(8)])
    got_dE = np.zeros((16, 64))
    for r in range(4):
        for i in range(4):
            got_dE[_LC, 16 * r + 4 * _LQ + i] = dE[r][:, i]
    np.testing.assert_allclose(got_dE[:, :63], ref_dE, rtol=0, atol=1e-9 * float(np.abs(ref_dE).max()))
