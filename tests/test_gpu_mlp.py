"""The deformation network on the GPU.

- The fused bf16 forward (gsd_mlp.hip, gsd_deform_mlp_forward_bf16) against the module's torch bf16 path (the same
  rounding points, hipBLASLt's accumulation order: 2 % of the output scale), the float32 forward (4 %: bf16's own
  error) and the lane-level CPU emulation of the kernel (tests/test_deform_mlp.py).
- The float32 training path (gsd_mlp_train.hip, gsd_deform_mlp_train_forward / _backward: BF16x6 GEMMs) against the
  float64 restatement oracle/deform_mlp_ref.py and its autograd: outputs and every gradient within 2e-5 of each
  tensor's scale (f32-level), and against torch's own f32 GEMMs within 1e-5.
P off the 32-, 128- and 256-Gaussian grains."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from conftest import PKG  # noqa: F401

pytestmark = pytest.mark.gpu


def _net(seed, scale=1.0):
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    torch.manual_seed(seed)
    net = DirectTemporalNeRF(dtype=torch.bfloat16)
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(scale)
    return net.cuda()


@pytest.mark.parametrize("P", [1, 77, 5003])
def test_fused_mlp_matches_torch_bf16_and_f32(P):
    from gsd_amd import _native
    net = _net(11, 2.0)
    g = torch.Generator().manual_seed(P)
    x = (torch.rand(P, 3, generator=g) * 4 - 2).cuda()
    t = torch.full((P, 1), 0.35, device="cuda")
    lib = _native.load()
    lib.gsd_timing_enable(1)
    lib.gsd_timing_reset()
    with torch.no_grad():
        fused = torch.cat(net(x, t, 5000), -1)
    names = (torch.zeros(32 * 64, dtype=torch.uint8)).numpy()
    import ctypes
    buf = ctypes.create_string_buffer(32 * 64)
    n = lib.gsd_timing_collect(64, buf, None, None)
    lib.gsd_timing_enable(0)
    launched = [buf.raw[32 * i: 32 * i + 32].split(b"\0")[0].decode() for i in range(n)]
    assert "deform_mlp" in launched   # the HIP kernel ran, not the torch path
    os.environ["GSD_MLP_TORCH"] = "1"
    try:
        with torch.no_grad():
            ref_bf16 = torch.cat(net(x, t, 5000), -1)
    finally:
        del os.environ["GSD_MLP_TORCH"]
    net32 = _net(11, 2.0)
    net32.compute_dtype = torch.float32
    with torch.no_grad():
        ref32 = torch.cat(net32(x, t, 5000), -1)
    assert torch.isfinite(fused).all()
    scale = float(ref32.abs().max())
    assert float((fused - ref_bf16).abs().max()) <= 2e-2 * scale
    assert float((fused - ref32).abs().max()) <= 4e-2 * scale
    # most outputs are bit-identical to torch's bf16 path (same rounding points, different summation order)
    assert float((fused == ref_bf16).float().mean()) > 0.5


def test_fused_mlp_matches_lane_emulation():
    from test_deform_mlp import _emulate_fused_mlp

    from gsd_amd.deform_mlp import pack_fused_mlp
    net = _net(12, 2.0)
    x = (torch.rand(32, 3) * 2 - 1)
    t = torch.full((32,), 0.4)
    with torch.no_grad():
        got = torch.cat(net(x.cuda(), t[:, None].cuda(), 5000), -1).cpu()
    frags, bias = pack_fused_mlp(net)
    want = torch.as_tensor(_emulate_fused_mlp(frags.cpu(), bias.cpu(), x.numpy(), t.numpy()))
    assert float((got - want).abs().max()) <= 1e-2 * float(want.abs().max())


def test_fused_mlp_not_used_with_grad():
    net = _net(13)
    x = torch.rand(100, 3, device="cuda", requires_grad=True)
    t = torch.full((100, 1), 0.1, device="cuda")
    outs = net(x, t, 5000)
    sum(o.sum() for o in outs).backward()   # the torch path, differentiable
    assert x.grad is not None and torch.isfinite(x.grad).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("P,N,relu", [(1, 256, True), (1000, 256, True), (5003, 58, False), (70_001, 256, True)])
def test_relu_backward_bias_matches_torch(dtype, P, N, relu):
    """gsd_relu_backward_bias (the MLP backward's ReLU mask + bias-gradient sums in one pass) against
    threshold_backward and sum(0); the mask bit for bit, the sums within float32 reordering."""
    from gsd_amd.deform_mlp import _relu_bias_backward
    g0 = torch.Generator(device="cuda").manual_seed(P)
    gy = torch.randn(P, N, device="cuda", generator=g0).to(dtype)
    y = torch.randn(P, N, device="cuda", generator=g0).relu().to(dtype) if relu else None
    g, db = _relu_bias_backward(gy, y)
    want = torch.ops.aten.threshold_backward(gy, y, 0) if relu else gy
    assert torch.equal(g, want)
    ref = want.double().sum(0)
    assert float((db.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(want.double().abs().sum(0).max()))


def test_mlp_training_backward_matches_reference_torch_path():
    """The module's backward on the GPU (split-K weight gradients, fused mask + bias kernel) against plain
    F.linear autograd, float32."""
    import torch.nn.functional as F

    from gsd_amd.deform_mlp import positional_encoding
    net = _net(14)
    net.compute_dtype = torch.float32
    P = 20_000
    x = (torch.rand(P, 3, device="cuda") * 2 - 1)
    t = torch.full((P, 1), 0.2, device="cuda")
    w = [torch.randn(P, n, device="cuda") for n in (3, 3, 4, 48)]

    def plain(xx, pre=None):
        ex, et = positional_encoding(xx), positional_encoding(t)
        h = torch.cat((ex, et), -1)
        for i, layer in enumerate(net._time):
            a = F.linear(h, layer.weight, layer.bias)
            if pre is not None:
                pre.append(a)
            h = F.relu(a)
            if i in net.skips:
                h = torch.cat((ex, h), -1)
        return [F.linear(h, m.weight, m.bias) for m in (net._time_out, net._time_out_scale, net._time_out_rot,
                                                        net._time_out_shs)]

    # ReLU ties: a pre-activation within f32 rounding of 0 takes a different mask in two correct f32 evaluations
    # (different summation orders), and that Gaussian's gradients then differ by a whole unit's contribution
    # (amplified up to 2^9 by the encoding in dx) -- 0-3 of these 20k Gaussians per seed, with the layer-fused forward
    # or the GEMMs alike.  The Gaussians with a pre-activation within 1e-5 of its layer's scale (located in float64)
    # get no upstream gradient, so no tie can reach any gradient; every gradient is then compared within 1e-4.
    with torch.no_grad():
        pre = []
        net.double()
        plain(x.double(), pre)
        net.float()
        tie = torch.zeros(P, dtype=torch.bool, device="cuda")
        for a in pre:
            tie |= (a.abs() < 1e-5 * float(a.abs().max())).any(-1)
    assert int(tie.sum()) < P // 10
    w = [wi * (~tie)[:, None] for wi in w]

    grads = {}
    for name, fn in (("fused", lambda xx: net(xx, t, 5000)), ("plain", plain)):
        net.zero_grad()
        xx = x.clone().requires_grad_(True)
        sum((o * wi).sum() for o, wi in zip(fn(xx), w)).backward()
        grads[name] = [xx.grad] + [p.grad.clone() for p in net.parameters()]
    for a, b in zip(grads["fused"], grads["plain"]):
        assert float((a - b).abs().max()) <= 1e-4 * float(b.abs().max()) + 1e-7


def test_fused_mlp_repacks_after_fused_adam_step():
    """The fused forward caches its packed weights under the parameters' (data_ptr, _version); FusedAdam updates
    them in place through raw pointers, so its step must advance their versions: a fused forward after the step
    uses the new weights (equal to a fresh pack's), not the cached ones."""
    from gsd_amd.optim import FusedAdam
    net = _net(15, 2.0)
    opt = FusedAdam([{"params": list(net.parameters()), "lr": 1e-2, "name": "offset_model"}], lr=0.0, eps=1e-15)
    x = (torch.rand(300, 3) * 2 - 1).cuda()
    t = torch.full((300, 1), 0.3, device="cuda")
    with torch.no_grad():
        before = torch.cat(net(x, t, 5000), -1)
    for p in net.parameters():
        p.grad.copy_(torch.randn_like(p))
    opt.step(zero_grad=True)
    with torch.no_grad():
        after = torch.cat(net(x, t, 5000), -1)
    net._fused_key = None   # force a fresh pack of the current weights
    with torch.no_grad():
        fresh = torch.cat(net(x, t, 5000), -1)
    assert not torch.equal(after, before)
    assert torch.equal(after, fresh)


def _launched(fn):
    """Run fn with the library's kernel timing on; the names of the C-ABI kernels it launched."""
    import ctypes

    from gsd_amd import _native
    lib = _native.load()
    lib.gsd_timing_enable(1)
    lib.gsd_timing_reset()
    try:
        out = fn()
        torch.cuda.synchronize()
        buf = ctypes.create_string_buffer(32 * 64)
        n = lib.gsd_timing_collect(64, buf, None, None)
    finally:
        lib.gsd_timing_enable(0)
    return out, {buf.raw[32 * i: 32 * i + 32].split(b"\0")[0].decode() for i in range(n)}


@pytest.fixture(params=[("w32", "w32"), ("w16", "w16"), ("w32", "w16")], ids=["f32c32", "f16c16", "f32c16"])
def fwd_kernel(request, monkeypatch):
    """The layer-fused training forward and the backward's dX chain: k_mlp_fwd_fused / k_mlp_bwd_chain (32 Gaussians
    per wave) or k_mlp_fwd_fused16 / k_mlp_bwd_chain16 (16 per wave, two waves per SIMD, round 6), and the mixed pair
    (the ReLU words and hidden outputs are one layout); the library reads GSD_MLP_FWD / GSD_MLP_CHAIN per call."""
    if request.param != ("w32", "w32") and os.environ.get("GSD_TEST_MLP16") != "1":
        pytest.skip("the 16-wide kernels (opt-in: GSD_MLP_FWD / GSD_MLP_CHAIN = w16) have their operand maps pinned "
                    "on the CPU (test_deform_mlp.py::test_fused16_and_chain16_maps_emulated) and are not yet run on "
                    "the GPU by default; GSD_TEST_MLP16=1 runs them")
    monkeypatch.setenv("GSD_MLP_FWD", request.param[0])
    monkeypatch.setenv("GSD_MLP_CHAIN", request.param[1])
    return request.param


def _train_run(net, x, t, w, torch_path):
    """Outputs and (dL/dx, parameter gradients) of sum(out . w) through the HIP path or torch's f32 GEMMs."""
    if torch_path:
        os.environ["GSD_MLP_TORCH"] = "1"
    try:
        net.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        outs, n1 = _launched(lambda: net(xx, t, 5000))
        _, n2 = _launched(lambda: sum((o * wi).sum() for o, wi in zip(outs, w)).backward())
    finally:
        os.environ.pop("GSD_MLP_TORCH", None)
    assert torch_path or ("deform_mlp_train_fwd" in n1 and "deform_mlp_train_bwd" in n2)   # the HIP path ran
    return torch.cat(outs, -1).detach(), [xx.grad] + [p.grad for p in net.parameters()]


@pytest.mark.parametrize("P,scale", [(1, 2.0), (77, 2.0), (128, 1.0), (257, 2.0), (5003, 1.0), (5003, 2.0),
                                     (70_001, 1.0)])
def test_train_f32_matches_float64_oracle_like_torch_f32(P, scale, fwd_kernel):
    """The f32 training path (gsd_mlp_train.hip: BF16x6 GEMMs, forward and backward) against the float64
    restatement of DirectTemporalNeRF (oracle/deform_mlp_ref.py) and its float64 autograd, side by side with the
    reference's own f32 computation (torch's f32 GEMMs, GSD_MLP_TORCH=1).  f32 itself is not float64: a
    pre-activation within rounding of 0 flips a ReLU mask, and dL/dx carries the encoding's 2^9 factors, so torch f32
    lands up to ~3 % (dL/dx) / ~0.3 % (weights) off float64 on this network with doubled weights.  Bar, per output
    tensor and per gradient tensor (max |err| over the tensor's max |value|): the HIP path's error <= max(2e-5, 2x
    torch f32's error) -- as accurate as the reference's own training precision."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    from oracle import deform_mlp_ref
    torch.manual_seed(40 + P % 7)
    net = DirectTemporalNeRF()
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(scale)   # doubled: every layer's ReLU pattern matters
    g = torch.Generator().manual_seed(P)
    x = torch.rand(P, 3, generator=g) * 4 - 2
    t = torch.full((P, 1), 0.35)
    w = [torch.randn(P, n, generator=g) for n in (3, 3, 4, 48)]
    sd = {k: v.detach().double().requires_grad_(True) for k, v in net.state_dict().items()}
    x64 = x.double().requires_grad_(True)
    ref = deform_mlp_ref.forward(sd, x64, t.double(), 5000)
    sum((o * wi.double()).sum() for o, wi in zip(ref, w)).backward()
    ref_out = torch.cat([r.detach() for r in ref], -1)
    ref_grads = [x64.grad] + [sd[k].grad for k, _ in net.named_parameters()]
    netc = net.cuda()
    xc, tc, wc = x.cuda(), t.cuda(), [wi.cuda() for wi in w]
    hip = _train_run(netc, xc, tc, wc, False)
    tor = _train_run(netc, xc, tc, wc, True)

    def err(a, b):
        return float((a.cpu().double() - b).abs().max()) / max(float(b.abs().max()), 1e-30)
    names = ["out", "x"] + [k for k, _ in net.named_parameters()]
    for name, h, tt, r in zip(names, [hip[0]] + hip[1], [tor[0]] + tor[1], [ref_out] + ref_grads):
        e_hip, e_torch = err(h, r), err(tt, r)
        assert e_hip <= max(2e-5, 2.0 * e_torch), (name, e_hip, e_torch)


def test_train_f32_large_p_weight_gradients_match_torch_f32(fwd_kernel):
    """Above 524,288 Gaussians the 256 x 256 weight gradients run in one round of 256 chunks of > 2048 Gaussians
    (launch_mlp_wgrad, round 5) -- a size the float64-oracle test above cannot reach on the CPU.  Against torch's f32
    GEMMs at P = 600,001: the four heads and the 24 parameter gradients within 1e-4 of each tensor's scale.  ReLU ties
    (a pre-activation within f32 rounding of 0 takes different masks in two correct f32 evaluations, moving that
    Gaussian's whole contribution) are kept out as in test_mlp_training_backward_matches_reference_torch_path: the
    Gaussians with a pre-activation within 1e-5 of its layer's scale (found in float64) get no upstream gradient.
    dL/dx is per Gaussian and is covered by the float64-oracle test."""
    import torch.nn.functional as F

    from gsd_amd.deform_mlp import DirectTemporalNeRF, positional_encoding
    P = 600_001
    torch.manual_seed(3)
    net = DirectTemporalNeRF().cuda()
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.rand(P, 3, device="cuda", generator=g) * 4 - 2
    t = torch.full((P, 1), 0.6, device="cuda")
    w = [torch.randn(P, n, device="cuda", generator=g) for n in (3, 3, 4, 48)]
    with torch.no_grad():   # the ReLU ties, from a float64 evaluation of the hidden layers
        xd, td = x.double(), t.double()
        ex = positional_encoding(xd)
        h = torch.cat((ex, positional_encoding(td)), -1)
        tie = torch.zeros(P, dtype=torch.bool, device="cuda")
        for i, layer in enumerate(net._time):
            a = F.linear(h, layer.weight.double(), layer.bias.double())
            tie |= (a.abs() < 1e-5 * float(a.abs().max())).any(-1)
            h = F.relu(a)
            if i in net.skips:
                h = torch.cat((ex, h), -1)
        del h, a, ex
    assert int(tie.sum()) < P // 10
    w = [wi * (~tie)[:, None] for wi in w]
    hip = _train_run(net, x, t, w, False)
    tor = _train_run(net, x, t, w, True)
    names = ["out", "x"] + [k for k, _ in net.named_parameters()]
    for name, h_, r in zip(names, [hip[0]] + hip[1], [tor[0]] + tor[1]):
        if name == "x":
            continue
        e = float((h_ - r).abs().max()) / max(float(r.abs().max()), 1e-30)
        assert e <= 1e-4, (name, e)


def test_train_f32_matches_reference_network_fixture(fwd_kernel):
    """The HIP f32 training path against the reference's own DirectTemporalNeRF run (tests/golden/mlp.npz:
    gaussian_model.py:242-316 with a seeded init, float32 forward + autograd on the CPU): the four heads, dL/dx and
    every parameter gradient, each within 2e-5 of its tensor's scale (max |err| / max |value|); the iteration-2000
    call returns exact zeros."""
    from conftest import golden
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    g = golden("mlp.npz")
    names = [str(n) for n in g["names"]]
    net = DirectTemporalNeRF()
    net.load_state_dict({n: torch.from_numpy(g["w:" + n]) for n in names})
    net = net.cuda()
    heads = ("dx", "dscale", "drot", "dshs")
    x = torch.from_numpy(g["x"]).cuda()
    t = torch.from_numpy(g["t"]).cuda()
    w = [torch.from_numpy(g["upstream:" + k]).cuda() for k in heads]
    out, grads = _train_run(net, x, t, w, False)
    want_out = np.concatenate([g["out:" + k] for k in heads], -1)
    assert np.abs(out.cpu().numpy() - want_out).max() <= 2e-5 * np.abs(want_out).max()
    for n, gr in zip(["x"] + names, grads):
        want = g["grad:" + n]
        err = float(np.abs(gr.cpu().numpy() - want).max()) / max(float(np.abs(want).max()), 1e-30)
        assert err <= 2e-5, (n, err)
    zero = net(x, t, 2000)
    assert all(float(z.abs().max()) == 0.0 and z.shape == g["zero2000:" + k].shape for z, k in zip(zero, heads))


def test_train_f32_nan_and_autograd_contracts():
    """(1) a NaN pre-activation propagates through the HIP path as through torch's F.relu (the ReLU is
    NaN-preserving, the backward mask passes a NaN's gradient as threshold_backward does): NaN outputs and
    gradients in the same places as the torch f32 path; (2) an in-place parameter update between the forward and
    the backward raises autograd's version error; (3) a second backward raises a clear error; (4) without grad the
    forward takes the evaluation kernel (no ~17-KB-per-Gaussian training workspace)."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    torch.manual_seed(5)
    net = DirectTemporalNeRF().cuda()
    with torch.no_grad():
        net._time[3].weight[7, :] = float("nan")   # one hidden unit of layer 3 is NaN for every Gaussian
    P = 300
    x = (torch.rand(P, 3, device="cuda") * 2 - 1)
    t = torch.full((P, 1), 0.4, device="cuda")
    w = [torch.randn(P, n, device="cuda") for n in (3, 3, 4, 48)]
    hip = _train_run(net, x, t, w, False)
    from oracle import deform_mlp_ref   # float64, torch.relu: NaN-propagating forward, threshold_backward masks
    sd = {k: v.detach().cpu().double().requires_grad_(True) for k, v in net.state_dict().items()}
    x64 = x.cpu().double().requires_grad_(True)
    ref = deform_mlp_ref.forward(sd, x64, t.cpu().double(), 5000)
    sum((o * wi.cpu().double()).sum() for o, wi in zip(ref, w)).backward()
    ref_out = torch.cat([r.detach() for r in ref], -1)
    assert torch.equal(torch.isnan(hip[0]).cpu(), torch.isnan(ref_out)) and bool(torch.isnan(ref_out).any())
    names = ["x"] + [k for k, _ in net.named_parameters()]
    for n, a, b in zip(names, hip[1], [x64.grad] + [sd[k].grad for k, _ in net.named_parameters()]):
        assert torch.equal(torch.isnan(a).cpu(), torch.isnan(b)), n
    net2 = DirectTemporalNeRF().cuda()
    xg = x.clone().requires_grad_(True)
    outs = net2(xg, t, 5000)
    with torch.no_grad():
        net2._time[0].weight.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        sum(o.sum() for o in outs).backward()
    outs = net2(xg, t, 5000)
    loss = sum(o.sum() for o in outs)
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="second time"):
        loss.backward()
    with torch.no_grad():
        _, names = _launched(lambda: net2(x, t, 5000))
    assert "deform_mlp_train_fwd" not in names and "deform_mlp_eval_fwd" in names


def test_train_f32_inplace_gradients_and_unused_heads():
    """The ABI-15 boundary of the training call (gsd_deform_mlp_train_forward_heads / _backward_heads): (1) heads the
    loss does not use reach the backward as None (autograd's unmaterialised gradients) and are read as zero -- bit
    for bit the gradients of the same loss with those heads weighted by explicit zeros; (2) parameters (and x) in a
    FlatGrads get their gradients written into their views -- stored while the views are stale, bit for bit the
    plain-autograd gradients; added on a second backward without an invalidate: exactly twice them."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    from gsd_amd.parallel import FlatGrads
    torch.manual_seed(11)
    net = DirectTemporalNeRF().cuda()
    P = 5003
    x = torch.rand(P, 3, device="cuda") * 4 - 2
    t = torch.full((P, 1), 0.3, device="cuda")
    w0, w3 = torch.randn(P, 3, device="cuda"), torch.randn(P, 48, device="cuda")

    def run(explicit_zeros, flat=None):
        xx = x.clone().requires_grad_(True)
        if flat is None:
            net.zero_grad(set_to_none=True)
        outs, n1 = _launched(lambda: net(xx, t, 5000))
        loss = (outs[0] * w0).sum() + (outs[3] * w3).sum()
        if explicit_zeros:
            loss = loss + (outs[1] * 0.0).sum() + (outs[2] * 0.0).sum()
        _, n2 = _launched(lambda: loss.backward())
        assert "deform_mlp_train_fwd" in n1 and "deform_mlp_train_bwd" in n2
        return xx, [p.grad.clone() for p in net.parameters()]

    xa, ga = run(False)
    xb, gb = run(True)
    assert torch.equal(xa.grad, xb.grad) and all(torch.equal(a, b) for a, b in zip(ga, gb))
    # in place: x's gradient sink is a FlatGrads view as well
    net.zero_grad(set_to_none=True)
    xx = x.clone().requires_grad_(True)
    params = list(net.parameters())
    flat = FlatGrads(params + [xx])
    flat.invalidate()
    outs = net(xx, t, 5000)
    ((outs[0] * w0).sum() + (outs[3] * w3).sum()).backward()
    assert torch.equal(xx.grad, xa.grad) and all(torch.equal(p.grad, a) for p, a in zip(params, ga))
    assert not flat.stale   # every view was claimed by the fused backward
    outs = net(xx, t, 5000)
    ((outs[0] * w0).sum() + (outs[3] * w3).sum()).backward()
    assert torch.equal(xx.grad, 2 * xa.grad) and all(torch.equal(p.grad, 2 * a) for p, a in zip(params, ga))
    flat.remove_hooks()


@pytest.mark.parametrize("P,scale", [(1, 2.0), (77, 2.0), (257, 2.0), (5003, 1.0), (70_001, 1.0)])
def test_eval_f32_matches_float64_oracle_and_training_forward(P, scale, fwd_kernel):
    """The f32 network without autograd (gsd_deform_mlp_eval_forward_heads: the training forward's fused kernel
    without its hidden-output stores) -- what render.py's torch.no_grad() evaluation runs: the four heads within
    max(2e-5, 2x torch f32's error) of the float64 restatement, and bit-identical to the training forward's heads
    (the same kernel arithmetic; only the stores differ)."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    from oracle import deform_mlp_ref
    torch.manual_seed(60 + P % 5)
    net = DirectTemporalNeRF()
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(scale)
    g = torch.Generator().manual_seed(P + 1)
    x = torch.rand(P, 3, generator=g) * 4 - 2
    t = torch.full((P, 1), 0.6)
    sd = {k: v.detach().double() for k, v in net.state_dict().items()}
    ref = torch.cat(deform_mlp_ref.forward(sd, x.double(), t.double(), 5000), -1)
    netc = net.cuda()
    xc, tc = x.cuda(), t.cuda()
    with torch.no_grad():
        ev, names = _launched(lambda: netc(xc, tc, 5000))
        os.environ["GSD_MLP_TORCH"] = "1"
        try:
            tor = torch.cat(netc(xc, tc, 5000), -1)
        finally:
            os.environ.pop("GSD_MLP_TORCH", None)
    assert "deform_mlp_eval_fwd" in names and "deform_mlp_train_fwd" not in names
    ev = torch.cat(ev, -1)
    scale_ = float(ref.abs().max())
    e_hip = float((ev.cpu().double() - ref).abs().max()) / scale_
    e_torch = float((tor.cpu().double() - ref).abs().max()) / scale_
    assert e_hip <= max(2e-5, 2.0 * e_torch), (e_hip, e_torch)
    tr = torch.cat(netc(xc.clone().requires_grad_(True), tc, 5000), -1).detach()
    assert torch.equal(ev, tr)


def test_empty_point_set_gives_empty_heads():
    """P = 0 (an empty point set, which the torch path always handled): empty heads of the right widths, with and
    without autograd, and no native call that would reject P <= 0."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    net = DirectTemporalNeRF().cuda()
    x, t = torch.zeros(0, 3, device="cuda"), torch.zeros(0, 1, device="cuda")
    with torch.no_grad():
        outs = net(x, t, 5000)
    assert [tuple(o.shape) for o in outs] == [(0, 3), (0, 3), (0, 4), (0, 48)]
    outs = net(x.clone().requires_grad_(True), t, 5000)
    assert [tuple(o.shape) for o in outs] == [(0, 3), (0, 3), (0, 4), (0, 48)]


def test_eval_f32_matches_reference_network_fixture(fwd_kernel):
    """The evaluation kernel against the reference's own DirectTemporalNeRF run (tests/golden/mlp.npz): the four
    heads within 2e-5 of their scale."""
    from conftest import golden
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    g = golden("mlp.npz")
    names = [str(n) for n in g["names"]]
    net = DirectTemporalNeRF()
    net.load_state_dict({n: torch.from_numpy(g["w:" + n]) for n in names})
    net = net.cuda()
    heads = ("dx", "dscale", "drot", "dshs")
    with torch.no_grad():
        out, launched = _launched(lambda: net(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda(), 5000))
    assert "deform_mlp_eval_fwd" in launched
    want = np.concatenate([g["out:" + k] for k in heads], -1)
    got = torch.cat(out, -1).cpu().numpy()
    assert np.abs(got - want).max() <= 2e-5 * np.abs(want).max()


def test_train_f32_fallback_kernels():
    """The comparison paths kept beside the defaults -- the per-layer GEMM forward (GSD_MLP_FWD=gemm), the per-layer
    dX GEMMs instead of the chain (GSD_MLP_BWD=gemm, which also sizes the workspace without the chain's gradient
    buffers), the eight-wave weight gradient (GSD_WGRAD16=0) and the 2048-Gaussian chunks at every size
    (GSD_WGRAD_ROUND1=0) -- read their switches once per process, so they run here in a child pytest over the
    float64-oracle, fixture, in-place/unused-heads and large-P tests."""
    import subprocess
    import sys
    env = dict(os.environ, GSD_MLP_FWD="gemm", GSD_MLP_BWD="gemm", GSD_WGRAD16="0", GSD_WGRAD_ROUND1="0")
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        os.path.join(here, "test_gpu_mlp.py"), "-k",
                        "train_f32_matches_float64 or train_f32_matches_reference or inplace_gradients or large_p"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "failed" not in r.stdout


def test_se3net_hip_path_matches_reference_fixture():
    """DirectTemporalNeRF_se3 on the HIP training kernels (its weights embedded, structurally zero elsewhere, in
    DirectTemporalNeRF's layout) and the fused HIP exp-map (se3_deform): w / v, the moved means and the gradients
    of the reference's weighted sum of them (x and the parameters, through the kernels' backward) against the
    reference's own run (tests/golden/mlp_se3.npz)."""
    from test_deform_mlp import _rel, se3net_from_fixture
    from gsd_amd._native import kernel_times
    from gsd_amd.deform import se3_deform
    net, g = se3net_from_fixture("cuda")
    x = torch.from_numpy(g["x"]).cuda().requires_grad_(True)
    t = torch.from_numpy(g["t"]).cuda()
    kernel_times(enable=True, reset=True)
    tw = net.twist(x, t, 5000)
    moved, _ = se3_deform(tw, x)
    names = [str(n) for n in g["names"]]
    params = dict(net.named_parameters())
    grads = torch.autograd.grad((moved * torch.from_numpy(g["upstream"]).cuda()).sum(), [x] + [params[n] for n in names])
    torch.cuda.synchronize()
    kt = kernel_times(enable=False, reset=True)
    assert "deform_mlp_train_fwd" in kt and "deform_mlp_train_bwd" in kt and "se3_fwd" in kt, sorted(kt)
    assert _rel(tw[:, :3].cpu(), g["w"]) <= 2e-5 and _rel(tw[:, 3:].cpu(), g["v"]) <= 2e-5
    assert float((moved.detach().cpu() - torch.from_numpy(g["moved"])).abs().max()) <= 2e-6
    assert _rel(grads[0].cpu(), g["grad:x"]) <= 1e-4
    for n, gr in zip(names, grads[1:]):
        assert _rel(gr.cpu(), g["grad:" + n]) <= 1e-4, n
    assert not net(x.detach(), t, 2000).any()


def test_se3net_drives_render_se3_mode():
    """render() in the SE(3) mode with the network as its twist producer (twist_model=net.twist): the frame renders
    and a loss on it reaches every layer of the network through the rasterizer, the exp-map and the kernels."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.deform_mlp import DirectTemporalNeRF_se3
    from gsd_amd.scene import make_gaussians
    torch.manual_seed(5)
    net = DirectTemporalNeRF_se3().cuda()
    P, W, H = 4000, 160, 128
    pc = DeformableGaussians(make_gaussians(P, W, H, seed=3).to("cuda"), sh_degree=3, deform="se3",
                             twist_model=net.twist)
    cam = synthetic_camera(W, H).to("cuda")
    out = render(cam, pc, default_pipe(), torch.zeros(3, device="cuda"), iteration=5000)
    assert out["means3D_offset"].abs().max() > 0
    out["render"].square().sum().backward()
    assert all(p.grad is not None and p.grad.abs().sum() > 0 for p in net.parameters())
