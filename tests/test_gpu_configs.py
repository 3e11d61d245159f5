"""BASELINE.json configurations 1-5 at their full sizes.

- cfg 1 (10k Gaussians, SH0, 400x400, identity SE(3)): the zero twist through the fused SE(3) kernel (exactly
  the identity on the means) into the rasterizer, against the C oracle, and d_twist through the whole chain
  against the oracle chain (C rasterizer backward -> float64 autograd of se3_ref).
- cfg 4 (1M, SH3, 1920x1080: the bench workload) and cfg 5 (2M, SH3, 3840x2160): the whole view against the
  OpenMP C oracle -- num_rendered, radii, ranges, point_list and the per-Gaussian state bit-exact, image and
  final_T within 1e-5 and n_contrib exact at every pixel whose decisions are not borderline in the oracle
  (test_gpu_parity.image_bar; the borderline pixels' flips are counted and reported), all eight gradients within
  rel L2 1e-4.
- cfg 2 (100k Gaussians, SH2, 800x800, static): the whole view against the C oracle -- binning and
  per-Gaussian state bit-exact, image / gradients within the bars of test_gpu_parity.py.
- cfg 3 (500k, SH3, 1920x1080, per-Gaussian SE(3) + d_se3): the fused SE(3) kernel against the float64
  restatement of rigid_body.exp_se3 (oracle/se3_ref.py); the rasterizer on the moved Gaussians against the C
  oracle (bit-exact binning); d_twist through the whole chain (HIP rasterizer backward -> HIP SE(3) backward)
  against the oracle chain (C rasterizer backward -> float64 autograd of se3_ref).
- cfg 5 (2M, SH3, 3840x2160, densification active): besides the oracle check above, size-independent
  properties of the forward (ranges partition [0, K), (tile, depth, id) order, every visible
  Gaussian binned, n_contrib <= range length, final_T in [1e-4, 1]), then a full training view through render()
  + loss + backward + the fused densification statistics + densify_and_prune on the FusedAdam slabs, whose
  point count must be exactly P + clones + 2 splits - split parents, followed by another view.
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from conftest import scene_inputs
from test_gpu_parity import check_forward, check_forward_against, gpu_backward, gpu_forward, oracle_fwd_bwd, rel_l2

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GRAD_NAMES = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"]


def check_invariants(P, W, H, fwd):
    """Size-independent properties of one forward (the cfg-4 test's checks, any resolution)."""
    from gsd_amd.introspect import decode
    K, color, radii, geom, binning, img = fwd
    st = decode(P, W, H, K, geom, binning, img)
    ranges = st["ranges"].cpu().numpy().astype(np.int64)
    counts = st["tile_count"].cpu().numpy().astype(np.int64)
    nz = counts > 0
    assert counts.sum() == K > 0
    np.testing.assert_array_equal(ranges[nz, 1] - ranges[nz, 0], counts[nz])
    starts = ranges[nz, 0]
    assert starts[0] == 0 and np.all(starts[1:] == ranges[nz, 1][:-1])
    pl = st["point_list"].cpu().numpy().astype(np.int64)
    depth_bits = st["depths"].cpu().numpy().view(np.uint32).astype(np.int64)
    key = (depth_bits[pl] << 32) | pl
    tile_of = np.repeat(np.nonzero(nz)[0], counts[nz])
    assert ((tile_of[1:] > tile_of[:-1]) | (key[1:] > key[:-1])).all()
    r = radii.cpu().numpy()
    assert np.array_equal(np.unique(pl), np.nonzero(r > 0)[0])
    T = st["final_T"].cpu().numpy()
    assert T.min() >= 1e-4 and T.max() <= 1.0
    gx = (W + 15) // 16
    tiles = (np.arange(H)[:, None] // 16) * gx + (np.arange(W)[None] // 16)
    assert np.all(st["n_contrib"].cpu().numpy().astype(np.int64) <= counts[tiles])
    assert torch.isfinite(color).all()
    return K


def test_config2_full_view_matches_oracle(oracle_mod):
    P, W, H, deg = 100_000, 800, 800, 2
    d = scene_inputs(P, W, H, deg, seed=2, device=DEV)
    o, fwd = check_forward(oracle_mod, d)
    assert o["num_rendered"] > P
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(2)).mul_(1e-3).to(DEV)
    _, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    grads = gpu_backward(d, gpu_forward(d), dpix)
    for name, gt in zip(GRAD_NAMES, grads):
        got = gt.cpu().numpy().reshape(ob[name].shape)
        assert np.isfinite(got).all(), name
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))


def full_view_matches_oracle(oracle_mod, P, W, H, deg, seed):
    """One whole view at a BASELINE configuration's size: forward (check_forward: bit-exact binning and
    per-Gaussian state, image / final_T / n_contrib bars) and all eight gradients against the C oracle."""
    d = scene_inputs(P, W, H, deg, seed=seed, device=DEV)
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(seed)).mul_(1e-3).to(DEV)
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    fwd = gpu_forward(d)
    K = check_forward_against(o, d, fwd)
    assert K == o["num_rendered"] > P
    grads = gpu_backward(d, fwd, dpix)
    for name, gt in zip(GRAD_NAMES, grads):
        got = gt.cpu().numpy().reshape(ob[name].shape)
        assert np.isfinite(got).all(), name
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))
    return d, fwd


def test_config4_full_view_matches_oracle(oracle_mod):
    """BASELINE configuration 4, the bench workload: 1M Gaussians, SH3, 1920x1080, seed 4."""
    d, fwd = full_view_matches_oracle(oracle_mod, 1_000_000, 1920, 1080, 3, seed=4)
    check_invariants(1_000_000, 1920, 1080, fwd)


def test_config5_full_view_matches_oracle(oracle_mod):
    """BASELINE configuration 5's view: 2M Gaussians, SH3, 3840x2160 (K ~ 6.5M instances, 32400 tiles)."""
    d, fwd = full_view_matches_oracle(oracle_mod, 2_000_000, 3840, 2160, 3, seed=5)
    del d, fwd
    torch.cuda.empty_cache()


def test_config1_identity_se3_chain_matches_oracle(oracle_mod):
    """BASELINE configuration 1: 10k Gaussians, SH0, 400x400, identity SE(3).  The zero twist through the fused
    SE(3) kernel leaves the means bit-identical (the guarded series, not the reference's NaN at theta = 0,
    SURVEY.md 0.5); the rasterizer on its output matches the oracle; d_twist / d_means / d_rot through the HIP
    chain match float64 autograd of se3_ref fed with the oracle's rasterizer gradients."""
    from gsd_amd import _C
    from gsd_amd.scene import make_gaussians
    from oracle import se3_ref
    P, W, H, deg = 10_000, 400, 400, 0
    g = make_gaussians(P, W, H, seed=1, se3="identity")
    assert float(g.twist.abs().max()) == 0.0
    d = scene_inputs(P, W, H, deg, seed=1, device=DEV)
    twist = g.twist.to(DEV)
    means0, rots0 = d["means3D"], d["rotations"]
    m, q = _C.se3_deform_forward(twist, means0, rots0)
    assert torch.equal(m, means0)
    tw64, x64, q64 = (t.detach().cpu().double().requires_grad_(True) for t in (twist, means0, rots0))
    m_ref, q_ref = se3_ref.deform(tw64, x64, q64)
    assert torch.isfinite(m_ref).all() and torch.isfinite(q_ref).all()
    assert rel_l2(q.cpu(), q_ref.detach()) <= 1e-6
    d["means3D"], d["rotations"] = m.contiguous(), q.contiguous()
    o, fwd = check_forward(oracle_mod, d)
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)).mul_(1e-3).to(DEV)
    _, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    grads = dict(zip(GRAD_NAMES, gpu_backward(d, fwd, dpix)))
    for name in GRAD_NAMES:
        got = grads[name].cpu().numpy().reshape(ob[name].shape)
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))
    d_tw, d_m, d_q = _C.se3_deform_backward(twist, means0, rots0, grads["dL_dmeans3D"].reshape(P, 3).contiguous(),
                                            grads["dL_drotations"].reshape(P, 4).contiguous())
    up_m = torch.from_numpy(ob["dL_dmeans3D"].reshape(P, 3)).double()
    up_q = torch.from_numpy(ob["dL_drotations"].reshape(P, 4)).double()
    ((m_ref * up_m).sum() + (q_ref * up_q).sum()).backward()
    for got, want, name in ((d_tw, tw64.grad, "d_twist"), (d_m, x64.grad, "d_means"), (d_q, q64.grad, "d_rot")):
        assert torch.isfinite(got).all(), name
        assert rel_l2(got.cpu(), want) <= 1e-4, (name, rel_l2(got.cpu(), want))


def test_config3_se3_full_view_matches_oracle_chain(oracle_mod):
    from gsd_amd import _C
    from gsd_amd.scene import make_gaussians
    from oracle import se3_ref
    P, W, H, deg = 500_000, 1920, 1080, 3
    g = make_gaussians(P, W, H, seed=3, se3="random")
    d = scene_inputs(P, W, H, deg, seed=3, device=DEV)
    twist = g.twist.to(DEV)
    means0, rots0 = d["means3D"], d["rotations"]
    # forward: the fused SE(3) kernel vs float64 exp_se3 applied to means and rotations
    m, q = _C.se3_deform_forward(twist, means0, rots0)
    tw64, x64, q64 = (t.detach().cpu().double().requires_grad_(True) for t in (twist, means0, rots0))
    m_ref, q_ref = se3_ref.deform(tw64, x64, q64)
    assert rel_l2(m.cpu(), m_ref.detach()) <= 1e-6
    assert rel_l2(q.cpu(), q_ref.detach()) <= 1e-6
    # the rasterizer on the moved Gaussians: bit-exact binning / state against the oracle on the same inputs
    d["means3D"], d["rotations"] = m.contiguous(), q.contiguous()
    o, fwd = check_forward(oracle_mod, d)
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(3)).mul_(1e-3).to(DEV)
    _, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    grads = dict(zip(GRAD_NAMES, gpu_backward(d, fwd, dpix)))
    for name in ("dL_dmeans3D", "dL_drotations", "dL_dscales", "dL_dsh"):
        got = grads[name].cpu().numpy().reshape(ob[name].shape)
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))
    # d_se3: HIP SE(3) backward of the HIP rasterizer gradients vs float64 autograd of the oracle's
    d_tw, d_m, d_q = _C.se3_deform_backward(twist, means0, rots0, grads["dL_dmeans3D"].reshape(P, 3).contiguous(),
                                            grads["dL_drotations"].reshape(P, 4).contiguous())
    up_m = torch.from_numpy(ob["dL_dmeans3D"].reshape(P, 3)).double()
    up_q = torch.from_numpy(ob["dL_drotations"].reshape(P, 4)).double()
    ((m_ref * up_m).sum() + (q_ref * up_q).sum()).backward()
    for got, want, name in ((d_tw, tw64.grad, "d_twist"), (d_m, x64.grad, "d_means"), (d_q, q64.grad, "d_rot")):
        assert torch.isfinite(got).all(), name
        assert rel_l2(got.cpu(), want) <= 1e-4, (name, rel_l2(got.cpu(), want))


def test_config5_invariants_and_densify_step():
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.loss import l1_ssim_loss
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    P, W, H = 2_000_000, 3840, 2160
    d = scene_inputs(P, W, H, 3, seed=5, device=DEV)
    K = check_invariants(P, W, H, gpu_forward(d))
    assert K > P
    del d
    torch.cuda.empty_cache()
    # one training view with densification: render -> loss -> backward -> stats -> densify_and_prune -> view
    prm = make_gaussians(P, W, H, seed=5, device=DEV)
    pc = DeformableGaussians(prm, sh_degree=3)
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    lrs = [0.00016, 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]
    opt = FusedAdam([{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(pc.parameters(), lrs, names)],
                    lr=0.0, eps=1e-15)
    dens = GaussianDensifier(pc, opt)
    cam = synthetic_camera(W, H).to(DEV)
    bg = torch.zeros(3, device=DEV)
    gt = torch.rand(3, H, W, generator=torch.Generator().manual_seed(5)).to(DEV)
    for yaw in (0.0, 2.0):
        out = render(synthetic_camera(W, H, yaw_deg=yaw).to(DEV), pc, default_pipe(), bg)
        l1_ssim_loss(out["render"], gt).backward()
        dens.add_densification_stats(out["viewspace_points"], out["radii"])
        opt.step(zero_grad=True)
    assert float(dens.denom.max()) == 2.0
    assert torch.isfinite(dens.xyz_gradient_accum).all()
    grads = dens.xyz_gradient_accum / dens.denom
    grads[grads.isnan()] = 0.0
    max_grad = float(grads[grads > 0].quantile(0.9))
    extent = float(torch.exp(pc._scaling.detach()).max(dim=1).values.median()) / 0.01
    with torch.no_grad():
        big = torch.exp(pc._scaling).max(dim=1).values > 0.01 * extent
        hot = grads.squeeze(1) >= max_grad
        n_clone, n_split = int((hot & ~big).sum()), int((hot & big).sum())
    assert n_clone > 0 and n_split > 0
    dens.densify_and_prune(max_grad, 0.0, extent, None)
    P2 = pc._xyz.shape[0]
    assert P2 == P + n_clone + n_split, (P2, P, n_clone, n_split)
    assert all(p.shape[0] == P2 for p in pc.parameters())
    out = render(cam, pc, default_pipe(), bg)
    l1_ssim_loss(out["render"], gt).backward()
    opt.step()
    assert out["radii"].shape[0] == P2 and torch.isfinite(out["render"]).all()
    assert all(torch.isfinite(p).all() for p in pc.parameters())
    assert math.isfinite(float(out["render"].sum()))


@pytest.mark.parametrize("P,W,H,deg,seed", [(100_000, 800, 800, 2, 2), (500_000, 1920, 1080, 3, 3),
                                            (1_000_000, 1920, 1080, 3, 4), (2_000_000, 3840, 2160, 3, 5)])
def test_reference_alpha_mode_meets_survey_bar(oracle_mod, P, W, H, deg, seed):
    """gsd_raster_args.alpha_mode = reference (ABI 17: alpha as forward.cu:343-345 writes it, o * expf(power),
    skipped when min(0.99, alpha) < 1/255) at the BASELINE configurations' view sizes, against SURVEY.md 8(c)'s
    image bar: |diff| <= 1e-4 at EVERY pixel (flips included), mean |diff| <= 1e-6, n_contrib exact except at
    pixels with an alpha within 3 ulp of 1/255 (the device's and the host's expf may round such an alpha to either
    side) or a termination test within 1e-5 of its threshold (at most 4), final_T within 5e-6 relative where
    n_contrib agrees; bit-exact binning; all eight gradients within rel
    L2 1e-4.  (The default mode's bar, image_bar in tests/test_gpu_parity.py, is looser: DESIGN.md 4.)"""
    from gsd_amd import _C
    from gsd_amd.introspect import decode
    from test_gpu_parity import ALPHA_MARGIN
    _C.set_alpha_mode("reference")
    try:
        d = scene_inputs(P, W, H, deg, seed=seed, device=DEV)
        dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(seed)).mul_(1e-3).to(DEV)
        o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
        fwd = gpu_forward(d)
        K, color, radii, geom, binning, img = fwd
        assert K == o["num_rendered"]
        st = {k: v.cpu().numpy() for k, v in decode(P, W, H, K, geom, binning, img).items()}
        np.testing.assert_array_equal(st["point_list"].astype(np.uint32), o["point_list"])
        c = color.cpu().numpy()
        diff = np.abs(c - o["color"])
        assert diff.max() <= 1e-4 and diff.mean() <= 1e-6, (diff.max(), diff.mean())
        nc_bad = st["n_contrib"].astype(np.uint32) != o["n_contrib"]
        # a decision may differ only where the oracle's own margin is within the two implementations' rounding:
        # an alpha within 3 ulp of 1/255, or T (1 - alpha) within 1e-5 (relative) of 1e-4 (the termination test,
        # which sees T's ~1e-6 deviation); measured: one such pixel at cfg5 (profiles/round6/parity/)
        border = (o["margin_alpha"] < ALPHA_MARGIN) | (o["margin_T"] < 1e-5)
        assert not (nc_bad & ~border).any() and nc_bad.sum() <= 4, int(nc_bad.sum())
        T, Tr = st["final_T"].astype(np.float64), np.maximum(o["final_T"].astype(np.float64), 1e-30)
        assert (np.abs(T - Tr) / Tr)[~nc_bad].max() <= 5e-6
        grads = gpu_backward(d, fwd, dpix)
        for name, gt in zip(GRAD_NAMES, grads):
            got = gt.cpu().numpy().reshape(ob[name].shape)
            assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))
    finally:
        _C.set_alpha_mode("fast")
