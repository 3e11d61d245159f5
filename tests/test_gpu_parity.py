"""HIP path (through the C-ABI) vs the CPU oracle -- the parity tests proper.

Bars (DESIGN.md "Parity"):
  bit-exact   radii, depths, means2D, conic/opacity, rgb, clamp flags, num_rendered,
              ranges, point_list (== the reference's stable sort of |tile|depth| keys)
  tolerance   image and final_T |diff| <= 1e-5 and n_contrib exact at every pixel whose compositing decisions are
              not borderline in the oracle; at a borderline pixel (some alpha within 3 ulp of 1/255, or some
              T (1 - alpha) within T_MARGIN of 1e-4, relative) a decision may flip -- the flips are counted and
              reported, and there |diff| <= FLIP_ABS_CAP (image_bar).  Mean |diff| <= 1e-7.  Gradients: per-tensor
              relative L2 <= 1e-4 (float atomics reorder sums), SE(3) deform vs float64 autograd: rel L2 <= 1e-5.
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from conftest import oracle_kwargs, scene_inputs

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def gpu_forward(d, *, colors=None, cov3D=None, scale_modifier=1.0, prefiltered=False, debug=False):
    from gsd_amd import _C
    empty = torch.empty(0)
    shs = d["shs"] if colors is None else empty
    scales, rots = (d["scales"], d["rotations"]) if cov3D is None else (empty, empty)
    return _C.rasterize_gaussians(d["bg"], d["means3D"], empty if colors is None else colors, d["opacities"], scales,
                                  rots, scale_modifier, empty if cov3D is None else cov3D, d["viewmatrix"],
                                  d["projmatrix"], d["tanfovx"], d["tanfovy"], d["H"], d["W"], shs, d["sh_degree"],
                                  d["campos"], prefiltered, debug)


def poison_allocator(nbytes=256 << 20):
    """Leave NaN-filled blocks in the caching allocator, so an output the kernels fail to write shows up."""
    t = torch.full((nbytes // 4,), float("nan"), device=DEV)
    del t


def gpu_backward(d, fwd, dpix, *, colors=None, cov3D=None, scale_modifier=1.0, scratch=None):
    from gsd_amd import _C
    poison_allocator()
    num_rendered, color, radii, geom, binning, img = fwd
    empty = torch.empty(0)
    shs = d["shs"] if colors is None else empty
    scales, rots = (d["scales"], d["rotations"]) if cov3D is None else (empty, empty)
    return _C.rasterize_gaussians_backward(d["bg"], d["means3D"], radii, empty if colors is None else colors, scales,
                                           rots, scale_modifier, empty if cov3D is None else cov3D, d["viewmatrix"],
                                           d["projmatrix"], d["tanfovx"], d["tanfovy"], dpix, shs, d["sh_degree"],
                                           d["campos"], geom, num_rendered, binning, img, False, scratch=scratch)


def oracle_fwd_bwd(oracle_mod, d, dpix=None, *, colors=None, cov3D=None, scale_modifier=1.0):
    kw = oracle_kwargs(d)
    means = d["means3D"].cpu().numpy()
    common = dict(viewmatrix=kw["viewmatrix"], projmatrix=kw["projmatrix"], campos=kw["campos"], W=d["W"], H=d["H"],
                  tanfovx=kw["tanfovx"], tanfovy=kw["tanfovy"], sh_degree=d["sh_degree"], bg=kw["bg"],
                  scale_modifier=scale_modifier)
    mode = dict(shs=None if colors is not None else kw["shs"],
                colors_precomp=None if colors is None else colors.cpu().numpy(),
                scales=None if cov3D is not None else kw["scales"],
                rotations=None if cov3D is not None else kw["rotations"],
                cov3D_precomp=None if cov3D is None else cov3D.cpu().numpy())
    fwd = oracle_mod.forward(means, kw["opacities"], **mode, **common)
    bwd = None
    if dpix is not None:
        bwd = oracle_mod.backward(fwd, dpix.cpu().numpy(), means, **mode, **common)
    return fwd, bwd


def check_forward(oracle_mod, d, **mode):
    o, _ = oracle_fwd_bwd(oracle_mod, d, **mode)
    fwd = gpu_forward(d, **mode)
    check_forward_against(o, d, fwd, colors=mode.get("colors"))
    return o, fwd


def check_forward_against(o, d, fwd, colors=None):
    """The forward's bars against an oracle forward `o` of the same inputs; returns num_rendered."""
    from gsd_amd.introspect import decode
    K, color, radii, geom, binning, img = fwd
    torch.cuda.synchronize()
    st = {k: v.cpu().numpy() for k, v in decode(d["means3D"].shape[0], d["W"], d["H"], K, geom, binning, img).items()}
    radii = radii.cpu().numpy()
    vis = o["radii"] > 0
    np.testing.assert_array_equal(radii, o["radii"])
    assert K == o["num_rendered"]
    np.testing.assert_array_equal(st["depths"][vis].view(np.uint32), o["depths"][vis].view(np.uint32))
    np.testing.assert_array_equal(st["means2D"][vis].view(np.uint32), o["means2D"][vis].view(np.uint32))
    np.testing.assert_array_equal(st["conic_opacity"][vis].view(np.uint32), o["conic_opacity"][vis].view(np.uint32))
    if colors is None:
        np.testing.assert_array_equal(st["rgb"][vis].view(np.uint32), o["rgb"][vis].view(np.uint32))
        cl = np.stack([(st["clamped"] >> c) & 1 for c in range(3)], 1).astype(bool)
        np.testing.assert_array_equal(cl[vis], o["clamped"][vis].astype(bool))
    np.testing.assert_array_equal(st["ranges"].astype(np.uint32), o["ranges"])
    np.testing.assert_array_equal(st["point_list"].astype(np.uint32), o["point_list"])
    # the reference's sort keys, rebuilt from (tile of the range, depth bits of the id): identical
    c = color.cpu().numpy()
    image_bar(c, st["final_T"], st["n_contrib"], o, tag=f"P={d['means3D'].shape[0]} {d['W']}x{d['H']}")
    return K


# Borderline decisions (the oracle's per-pixel margins, oracle.forward).  The HIP kernels decide alpha >= 1/255 as
# power >= t_o (record_og, gsd_render.hip): the real comparison against t_o = -ln(255 o) rounded to the nearest float,
# where the oracle rounds o * expf(power).  The two can part only where the oracle's alpha lies within its own rounding
# of 1/255 (expf's ulp + the product's half ulp) plus t_o's half ulp (up to ~1 relative ulp of alpha): 2.5 ulp, and the
# flips measured in round 5 sit at 0.5, 1.5 and 2.5 ulp (profiles/round5/parity/).  ALPHA_MARGIN is 3 ulp of 1/255
# (the relative ulp there is 255 * 2^-31 = 1.19e-7).  T (1 - alpha) within T_MARGIN (relative) of 1e-4: T carries the
# few-ulp alpha VALUE differences of the hardware exp over every record before it; T_MARGIN is twice the largest
# relative final_T deviation measured at the configurations' pixels with no borderline alpha.
ALPHA_MARGIN = 3 * 255 * 2.0 ** -31
# measured at the alpha-clear pixels of configurations 1-5 (round 5): 6.5e-6, 8.4e-6, 9.2e-6, 1.04e-5, 1.05e-5
T_MARGIN = 2.1e-5
# a flip changes one record's share: bounded at twice the largest measured (8.4e-4 at cfg5, round 5)
FLIP_ABS_CAP = 1.7e-3


def image_bar(c, T, nc, o, tag=""):
    """Image / final_T / n_contrib bars against the oracle forward `o`.  Outside the borderline
    pixels: |diff| <= 1e-5 and n_contrib exact.  A pixel whose result differs beyond that must be borderline (a
    flip); flips are counted and reported (GSD_PARITY_REPORT: a JSONL file to append the counts to), bounded by
    FLIP_ABS_CAP and at most a third of the borderline pixels (or 4).  Mean |diff| <= 1e-7."""
    import json
    import os
    c_ref, T_ref, nc_ref = o["color"], o["final_T"], o["n_contrib"]
    border = (o["margin_alpha"] < ALPHA_MARGIN) | (o["margin_T"] < T_MARGIN)
    dc = np.abs(c - c_ref).max(axis=0)          # per pixel, over the channels
    dT = np.abs(T - T_ref)
    nc_bad = nc.astype(np.uint32) != nc_ref
    flips = (dc > 1e-5) | (dT > 1e-5) | nc_bad
    T_ref64 = np.maximum(np.asarray(T_ref, np.float64), 1e-30)
    rel_T = np.abs(np.asarray(T, np.float64) - T_ref64) / T_ref64
    stats = dict(tag=tag, pixels=int(dc.size), borderline=int(border.sum()), flips=int(flips.sum()),
                 n_contrib_mismatch=int(nc_bad.sum()),
                 alpha_borderline=int((o["margin_alpha"] < ALPHA_MARGIN).sum()),
                 max_abs_outside=float(dc[~border].max(initial=0.0)), max_abs_flips=float(dc[flips].max(initial=0.0)),
                 max_rel_T_outside_flips=float(rel_T[~flips].max(initial=0.0)),
                 max_rel_T_alpha_clear=float(rel_T[~flips & (o["margin_alpha"] >= ALPHA_MARGIN)].max(initial=0.0)),
                 flip_margins=[[float(a), float(b)] for a, b in zip(o["margin_alpha"][flips], o["margin_T"][flips])])
    if os.environ.get("GSD_PARITY_REPORT"):
        with open(os.environ["GSD_PARITY_REPORT"], "a") as f:
            f.write(json.dumps(stats) + "\n")
    assert not (flips & ~border).any(), ("a decision flipped at a non-borderline pixel", stats)
    assert dc.max() <= FLIP_ABS_CAP and dT.max() <= FLIP_ABS_CAP, stats
    # and they stay rare among the borderline pixels (measured: 11 of 54 at cfg5, 3 of 10 at cfg3, 1 of 302 at cfg4)
    assert stats["flips"] <= max(4, stats["borderline"] // 3), stats
    assert np.abs(c - c_ref).mean() <= 1e-7 and dT.mean() <= 1e-7, (np.abs(c - c_ref).mean(), dT.mean())
    return stats


CASES = [  # (P, W, H, deg, seed): config-1 shape, odd sizes, every SH degree
    (10_000, 400, 400, 0, 1),
    (3_000, 333, 217, 1, 2),
    (4_000, 256, 256, 2, 3),
    (6_000, 640, 360, 3, 4),
]


@pytest.mark.parametrize("P,W,H,deg,seed", CASES)
def test_forward_bit_exact(oracle_mod, P, W, H, deg, seed):
    d = scene_inputs(P, W, H, deg, seed=seed, device=DEV)
    check_forward(oracle_mod, d)


@pytest.mark.parametrize("P,W,H,deg,seed", CASES)
def test_backward_matches_oracle(oracle_mod, P, W, H, deg, seed):
    d = scene_inputs(P, W, H, deg, seed=seed, device=DEV)
    g = torch.Generator().manual_seed(seed)
    dpix = torch.randn(3, H, W, generator=g).mul_(1e-3).to(DEV)
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    fwd = gpu_forward(d)
    grads = gpu_backward(d, fwd, dpix)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    for name, gt in zip(names, grads):
        got = gt.cpu().numpy().reshape(ob[name].shape)
        assert np.isfinite(got).all(), name
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))


# the per-Gaussian gradient record (gsd_kernels.h GradRecField): dL/dmean2D x, y; dL/dconic a, b, c; dL/dopacity;
# dL/dcolor r, g, b -- 16 floats per Gaussian in the backward's scratch
_REC_FLOATS = 16


@pytest.mark.parametrize("lo,hi,ceiling", [(5.0, 20.0, 2e-2), (40.0, 200.0, 0.2)])
def test_anisotropic_gaussians_forward_and_backward(oracle_mod, lo, hi, ceiling):
    """Needle-like Gaussians (one axis lo-hi times the others, random rotations, opacities up to 0.999): their alpha
    boxes are loose and the linear ellipse bound over each 4x4 block does most of the list culling in both render
    kernels (bwd_compact_groups).  The forward stays bit-exact; the render kernel's gradients (dL/dmean2D, dL/dconic
    read from the backward's gradient records, dL/dcolor, dL/dopacity) and dL/dsh match the oracle at this file's
    1e-4.  The 2D covariances are near-singular in float32 (a c / det up to 2.7e3 at 5-20x, 2.5e5 at 40-200x), so the
    reference's own conic -> cov3D -> scale / rotation chain (backward.cu:144-274, 278-341) amplifies the last-bit
    differences of dL/dconic (float-atomic order) into the 1e-3..1e-2 range for dL/dmeans3D, dL/dcov3D, dL/dscales
    and dL/drotations.  That chain is pinned on its own instead: the oracle's preprocess backward
    (oracle.preprocess_backward, backward.cu:144-396) fed with the HIP run's own render-level gradients must give
    the HIP's four chain gradients within rel L2 1e-5.  Against the full oracle (the amplified order noise) they stay
    under a fixed ceiling per range: 2e-2 at 5-20x, 0.2 at 40-200x (measured round 6: dL/drotations 7.3e-2 there)."""
    from gsd_amd import _C
    P, W, H, deg, seed = 5_000, 320, 240, 1, 11
    d = scene_inputs(P, W, H, deg, seed=seed, device=DEV)
    g = torch.Generator().manual_seed(seed)
    s = d["scales"].cpu().clone()  # activated scales
    s[:, 0] *= torch.empty(P).uniform_(lo, hi, generator=g)
    s[:, 1:] *= 0.4
    d["scales"] = s.to(DEV)
    d["opacities"] = torch.empty(d["opacities"].shape).uniform_(0.02, 0.999, generator=g).to(DEV)
    check_forward(oracle_mod, d)
    dpix = torch.randn(3, H, W, generator=g).mul_(1e-3).to(DEV)
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    fwd = gpu_forward(d)
    scratch = torch.zeros(_C.backward_scratch_bytes(P), dtype=torch.uint8, device=DEV)
    assert scratch.data_ptr() % 128 == 0   # the library aligns the records to 128 B: offset 0 here
    grads = [t.cpu().numpy() for t in gpu_backward(d, fwd, dpix, scratch=scratch)]
    torch.cuda.synchronize()
    rec = scratch[: 4 * _REC_FLOATS * P].view(torch.float32).view(P, _REC_FLOATS).cpu().numpy()
    vis = (fwd[2].cpu().numpy() > 0)[:, None]
    dmean2D = np.where(vis, np.concatenate([rec[:, 0:2], np.zeros((P, 1), np.float32)], 1), 0).astype(np.float32)
    dconic = np.where(vis, np.stack([rec[:, 2], rec[:, 3], np.zeros(P, np.float32), rec[:, 4]], 1), 0)
    dconic = dconic.astype(np.float32)
    dcolor = np.where(vis, rec[:, 6:9], 0).astype(np.float32)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    got = {n: gt.reshape(ob[n].shape) for n, gt in zip(names, grads)}
    # the records are what the API returned, and the render-level gradients match the oracle's
    np.testing.assert_array_equal(got["dL_dmeans2D"], dmean2D)
    np.testing.assert_array_equal(got["dL_dcolors"], dcolor)
    assert rel_l2(dconic, ob["dL_dconic"]) <= 1e-4, ("dL_dconic", rel_l2(dconic, ob["dL_dconic"]))
    for n in ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dsh"]:
        assert np.isfinite(got[n]).all(), n
        assert rel_l2(got[n], ob[n]) <= 1e-4, (n, rel_l2(got[n], ob[n]))
    kw = oracle_kwargs(d)
    pre = oracle_mod.preprocess_backward(o, dmean2D, dconic, dcolor, d["means3D"].cpu().numpy(), shs=kw["shs"],
                                         scales=kw["scales"], rotations=kw["rotations"],
                                         viewmatrix=kw["viewmatrix"], projmatrix=kw["projmatrix"],
                                         campos=kw["campos"], W=W, H=H, tanfovx=kw["tanfovx"],
                                         tanfovy=kw["tanfovy"], sh_degree=deg)
    for n in ["dL_dmeans3D", "dL_dcov3D", "dL_dscales", "dL_drotations"]:
        assert np.isfinite(got[n]).all(), n
        e_chain = rel_l2(got[n], pre[n])
        assert e_chain <= 1e-5, (n, "vs the oracle chain on the HIP's records", e_chain)
        assert rel_l2(got[n], ob[n]) <= ceiling, (n, "vs the full oracle", rel_l2(got[n], ob[n]))


@pytest.mark.parametrize("short_binning", [False, True])
def test_backward_with_forward_zeroed_scratch(oracle_mod, short_binning):
    """ABI 14 grad_scratch: the forward's compositing kernel zeroes the backward's gradient records (here a
    NaN-filled buffer) and the backward given that scratch skips its memset -- gradients still match the oracle.
    short_binning: the first phase-2 launch is cut short by a small binning buffer, the relaunch zeroes again."""
    from gsd_amd import _C
    P, W, H, deg, seed = 6_000, 640, 360, 3, 4
    d = scene_inputs(P, W, H, deg, seed=seed, device=DEV)
    g = torch.Generator().manual_seed(seed)
    dpix = torch.randn(3, H, W, generator=g).mul_(1e-3).to(DEV)
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    scratch = torch.full((_C.backward_scratch_bytes(P),), 0xFF, dtype=torch.uint8, device=DEV)   # NaN floats
    if short_binning:
        _C._K_GUESS[torch.device(DEV)] = 8
    empty = torch.empty(0)
    fwd = _C.rasterize_gaussians(d["bg"], d["means3D"], empty, d["opacities"], d["scales"], d["rotations"], 1.0,
                                 empty, d["viewmatrix"], d["projmatrix"], d["tanfovx"], d["tanfovy"], d["H"], d["W"],
                                 d["shs"], d["sh_degree"], d["campos"], False, False, grad_scratch=scratch)
    check_forward_against(o, d, fwd)
    K, color, radii, geom, binning, img = fwd
    grads = _C.rasterize_gaussians_backward(d["bg"], d["means3D"], radii, empty, d["scales"], d["rotations"], 1.0,
                                            empty, d["viewmatrix"], d["projmatrix"], d["tanfovx"], d["tanfovy"], dpix,
                                            d["shs"], d["sh_degree"], d["campos"], geom, K, binning, img, False,
                                            scratch=scratch)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    for name, gt in zip(names, grads):
        got = gt.cpu().numpy().reshape(ob[name].shape)
        assert np.isfinite(got).all(), name
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))


def test_backward_low_opacity(oracle_mod):
    """Opacity logits down to -9 (o ~ 1.2e-4, far below the 1/255 alpha floor) and up to +4: every gradient,
    dL/dopacity included, within rel L2 1e-4 of the oracle's sum of G * dL/dalpha (backward.cu:552), and
    per Gaussian within 1e-3 relative (+ 1e-3 of the largest) where the oracle's dL/dopacity is non-zero --
    the kernel recovers dL/dopacity from its sum of o * G * dL/dalpha, which must not lose the small
    opacities.  Gaussians that never reach alpha >= 1/255 get exactly zero."""
    P, W, H, deg = 8_000, 320, 240, 3
    d = scene_inputs(P, W, H, deg, seed=21, device=DEV)
    logit = torch.empty(P).uniform_(-9.0, 4.0, generator=torch.Generator().manual_seed(21))
    d["opacities"] = torch.sigmoid(logit)[:, None].contiguous().to(DEV)
    d["scales"] = d["scales"] * 2.0     # larger footprints: more low-opacity Gaussians cross the alpha floor
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(22)).mul_(1e-3).to(DEV)
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    fwd = gpu_forward(d)
    check_forward_against(o, d, fwd)
    grads = gpu_backward(d, fwd, dpix)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    for name, gt in zip(names, grads):
        got = gt.cpu().numpy().reshape(ob[name].shape)
        assert np.isfinite(got).all(), name
        assert rel_l2(got, ob[name]) <= 1e-4, (name, rel_l2(got, ob[name]))
    got = grads[2].cpu().numpy().reshape(-1).astype(np.float64)
    want = ob["dL_dopacity"].reshape(-1).astype(np.float64)
    op = d["opacities"].cpu().numpy().reshape(-1)
    low = (op < 0.02) & (want != 0)
    assert low.sum() > 20, low.sum()          # the case is exercised
    assert np.all(np.abs(got - want) <= 1e-3 * np.abs(want) + 1e-3 * np.abs(want).max())
    assert np.all(got[op < 1.0 / 255.0] == 0.0)


@pytest.mark.parametrize("kind", ["negative_zero", "nan"])
def test_opacities_outside_the_unit_interval(oracle_mod, kind):
    """The activated API takes opacities as given.  Negative ones give alpha = min(0.99, o G) < 1/255 at
    every pixel, so they are never composited (forward.cu:343-345; the kernels' threshold t_o = +inf); zero ones
    likewise; a NaN one composites at alpha = fminf(0.99, NaN) = 0.99 wherever power <= 0 (CUDA's min is IEEE
    minNum).  Forward bars and backward gradients against the oracle.  With NaN opacities the gradients of the other
    Gaussians are compared (the NaN Gaussians' own are NaN through dL/dG = o dL/dalpha, backward.cu:538, except
    dL/dopacity, which the kernel recovers from its sum of o G dL/dalpha and so cannot give for a NaN o)."""
    P, W, H, deg = 6_000, 320, 240, 3
    d = scene_inputs(P, W, H, deg, seed=31, device=DEV)
    op = d["opacities"].clone()
    if kind == "negative_zero":
        op[0:600:3] = -op[0:600:3]
        op[1:600:3] = 0.0
    else:
        op[0:600:50] = float("nan")
    d["opacities"] = op.contiguous()
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(32)).mul_(1e-3).to(DEV)
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix)
    fwd = gpu_forward(d)
    check_forward_against(o, d, fwd)
    grads = gpu_backward(d, fwd, dpix)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    rows = np.isfinite(op.cpu().numpy().reshape(-1))     # the Gaussians compared
    for name, gt in zip(names, grads):
        got = gt.cpu().numpy().reshape(ob[name].shape)[rows]
        want = ob[name][rows]
        assert np.isfinite(got).all() and np.isfinite(want).all(), name
        assert rel_l2(got, want) <= 1e-4, (name, rel_l2(got, want))
    if kind == "negative_zero":
        g_op = grads[2].cpu().numpy().reshape(-1)
        assert np.all(g_op[(op.cpu().numpy().reshape(-1) <= 0)] == 0.0)


def test_backward_run_to_run_noise():
    """The backward's gradient sums are float atomics in scheduling order, so two runs on the same inputs differ
    in the last bits; the per-record reductions must not amplify that (a formulation whose centring cancels
    turned it into ~1e-4 relative).  Two backward passes of one forward: per-tensor relative L2 <= 2e-6."""
    d = scene_inputs(60_000, 640, 480, 3, seed=5, device=DEV)
    dpix = torch.randn(3, 480, 640, generator=torch.Generator().manual_seed(5)).mul_(1e-3).to(DEV)
    fwd = gpu_forward(d)
    a = [t.cpu().numpy() for t in gpu_backward(d, fwd, dpix)]
    b = [t.cpu().numpy() for t in gpu_backward(d, fwd, dpix)]
    for i, (x, y) in enumerate(zip(a, b)):
        if y.size:
            assert rel_l2(x, y) <= 2e-6, (i, rel_l2(x, y))


def test_precomputed_colors_and_cov3d(oracle_mod):
    from gsd_amd.renderer import build_covariance_from_scaling_rotation
    d = scene_inputs(5_000, 320, 240, 3, seed=7, device=DEV)
    cov = build_covariance_from_scaling_rotation(d["scales"], 1.0, d["rotations"]).contiguous()
    colors = torch.rand(5_000, 3, generator=torch.Generator().manual_seed(3)).to(DEV)
    check_forward(oracle_mod, d, colors=colors, cov3D=cov)
    dpix = torch.randn(3, 240, 320, generator=torch.Generator().manual_seed(5)).mul_(1e-3).to(DEV)
    _, ob = oracle_fwd_bwd(oracle_mod, d, dpix, colors=colors, cov3D=cov)
    grads = gpu_backward(d, gpu_forward(d, colors=colors, cov3D=cov), dpix, colors=colors, cov3D=cov)
    for name, gt in zip(["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D"], grads[:5]):
        assert rel_l2(gt.cpu().numpy().reshape(ob[name].shape), ob[name]) <= 1e-4, name


def test_background_and_scale_modifier(oracle_mod):
    d = scene_inputs(4_000, 200, 150, 2, seed=11, device=DEV)
    d["bg"] = torch.tensor([0.2, 0.5, 0.9], device=DEV)
    check_forward(oracle_mod, d, scale_modifier=0.7)
    dpix = torch.randn(3, 150, 200, generator=torch.Generator().manual_seed(2)).mul_(1e-3).to(DEV)
    _, ob = oracle_fwd_bwd(oracle_mod, d, dpix, scale_modifier=0.7)
    grads = gpu_backward(d, gpu_forward(d, scale_modifier=0.7), dpix, scale_modifier=0.7)
    for name, gt in zip(["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D"], grads[:4]):
        assert rel_l2(gt.cpu().numpy().reshape(ob[name].shape), ob[name]) <= 1e-4, name


def test_dense_tile_merge_path(oracle_mod):
    """A tile holding > 4096 instances takes the chunk-sort + merge-path branch."""
    d = scene_inputs(12_000, 128, 128, 0, seed=5, device=DEV)
    g = torch.Generator().manual_seed(9)
    z = torch.rand(12_000, generator=g) * 4 + 3
    xy = (torch.rand(12_000, 2, generator=g) - 0.5) * 0.02 * z[:, None]
    d["means3D"] = torch.cat([xy, z[:, None]], 1).to(DEV)
    d["scales"] = torch.full((12_000, 3), 0.002).to(DEV)
    o, _ = check_forward(oracle_mod, d)
    counts = o["ranges"][:, 1].astype(np.int64) - o["ranges"][:, 0]
    assert counts.max() > 4096


@pytest.mark.parametrize("P,lo,hi", [(700, 512, 1024), (1500, 1024, 2048), (3000, 2048, 4096)])
def test_dense_tile_sort_classes(oracle_mod, P, lo, hi):
    """The tile sort's size classes above the 512-key register network: 1024 and 2048 keys in registers, and
    2049-4096 keys, which take the LDS-chunk + merge path since the LDS cap is 2048 (gsd_kernels.h kSortCap)."""
    d = scene_inputs(P, 128, 128, 0, seed=6, device=DEV)
    g = torch.Generator().manual_seed(10)
    z = torch.rand(P, generator=g) * 4 + 3
    xy = (torch.rand(P, 2, generator=g) - 0.5) * 0.02 * z[:, None]
    d["means3D"] = torch.cat([xy, z[:, None]], 1).to(DEV)
    d["scales"] = torch.full((P, 3), 0.002).to(DEV)
    o, _ = check_forward(oracle_mod, d)
    counts = o["ranges"][:, 1].astype(np.int64) - o["ranges"][:, 0]
    assert lo < counts.max() <= hi


def test_binning_buffer_too_small_retries(oracle_mod):
    """The binning buffer is sized from the previous count before the forward knows num_rendered; a short one
    (GSD_NEED_BINNING) is re-allocated and phase 2 re-run -- same results as a well-sized one."""
    from gsd_amd import _C
    d = scene_inputs(6_000, 640, 360, 3, seed=4, device=DEV)
    _C._K_GUESS[torch.device(DEV)] = 1
    check_forward(oracle_mod, d)
    assert _C._K_GUESS[torch.device(DEV)] > 1000


def test_binning_capacity_boundary():
    """Phase 2 is queued before num_rendered reaches the host, guarded by the binning buffer's capacity: buffers
    holding a little less than, exactly, and a little more than num_rendered all give the same image, radii
    and final count (short ones through GSD_NEED_BINNING and a second phase-2 call)."""
    from gsd_amd import _C
    d = scene_inputs(6_000, 640, 360, 3, seed=6, device=DEV)
    K, color, radii, *_ = gpu_forward(d)
    assert K > 1000
    for want in (K - 300, K - 1, K, K + 1):
        guess = next(g for g in range(max(1, want * 4 // 5 - 8), want * 4 // 5 + 8) if g + g // 4 >= want)
        _C._K_GUESS[torch.device(DEV)] = guess     # the buffer holds gsd_binning_buffer_bytes(guess + guess // 4)
        K2, color2, radii2, *_ = gpu_forward(d)
        assert K2 == K
        assert torch.equal(radii2, radii)
        assert torch.equal(color2, color), want


def test_empty_and_culled():
    d = scene_inputs(100, 64, 64, 0, seed=1, device=DEV)
    d["means3D"] = d["means3D"] * torch.tensor([1.0, 1.0, -1.0], device=DEV)   # all behind the camera
    K, color, radii, *_ = gpu_forward(d)
    assert K == 0 and int(radii.abs().sum()) == 0
    assert torch.equal(color, torch.zeros_like(color))
    d0 = scene_inputs(1, 64, 64, 0, seed=1, device=DEV)
    d0 = {k: (v[:0] if k in ("means3D", "scales", "rotations", "opacities", "shs") else v) for k, v in d0.items()}
    K0, c0, r0, *_ = gpu_forward(d0)
    assert K0 == 0 and r0.numel() == 0 and c0.shape == (3, 64, 64)


def test_prefiltered_raises():
    from gsd_amd._native import NativeError
    d = scene_inputs(100, 64, 64, 0, seed=1, device=DEV)
    d["means3D"][0, 2] = -1.0
    with pytest.raises(NativeError, match="prefiltered"):
        gpu_forward(d, prefiltered=True)


def test_mark_visible(oracle_mod):
    from gsd_amd import _C
    d = scene_inputs(5_000, 64, 64, 0, seed=2, device=DEV)
    d["means3D"][::3, 2] *= -1
    got = _C.mark_visible(d["means3D"], d["viewmatrix"], d["projmatrix"]).cpu().numpy()
    want = oracle_mod.mark_visible(d["means3D"].cpu().numpy(), d["viewmatrix"].cpu().numpy(),
                                   d["projmatrix"].cpu().numpy())
    np.testing.assert_array_equal(got, want)


def test_se3_deform_matches_float64_autograd():
    from gsd_amd.deform import se3_deform
    from oracle import se3_ref
    g = torch.Generator().manual_seed(0)
    P = 4096
    tw = torch.cat([torch.randn(P, 3, generator=g) * 0.5, torch.randn(P, 3, generator=g) * 0.2], 1)
    tw[:8, :3] *= torch.tensor([0.0, 1e-9, 1e-7, 1e-5, 1e-3, 1e-2, 0.1, 3.0])[:, None]   # across the series switch
    x = torch.randn(P, 3, generator=g) * 3
    q = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=1)
    gm, gq = torch.randn(P, 3, generator=g), torch.randn(P, 4, generator=g)
    tw64, x64, q64 = (t.double().requires_grad_(True) for t in (tw, x, q))
    m_ref, q_ref = se3_ref.deform(tw64, x64, q64)
    ((m_ref * gm.double()).sum() + (q_ref * gq.double()).sum()).backward()
    twd, xd, qd = (t.to(DEV).requires_grad_(True) for t in (tw, x, q))
    m, qo = se3_deform(twd, xd, qd)
    ((m * gm.to(DEV)).sum() + (qo * gq.to(DEV)).sum()).backward()
    assert rel_l2(m.detach().cpu(), m_ref.detach()) <= 1e-6
    assert rel_l2(qo.detach().cpu(), q_ref.detach()) <= 1e-6
    for got, want in [(twd.grad, tw64.grad), (xd.grad, x64.grad), (qd.grad, q64.grad)]:
        assert rel_l2(got.cpu(), want) <= 1e-5
    # zero twist is exactly the identity on the means
    z, _ = se3_deform(torch.zeros(4, 6, device=DEV), xd[:4].detach())
    assert torch.equal(z, xd[:4].detach())


def test_render_end_to_end_autograd():
    """render() drop-in: additive and SE(3) modes, gradients reach every parameter."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.scene import make_gaussians
    for mode, se3 in (("additive", None), ("se3", "random")):
        params = make_gaussians(20_000, 320, 240, seed=3, se3=se3, device=DEV)
        pc = DeformableGaussians(params, sh_degree=3, deform=mode)
        cam = synthetic_camera(320, 240).to(DEV)
        out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV))
        assert out["render"].shape == (3, 240, 320)
        loss = (out["render"] - 0.5).abs().mean()
        loss.backward()
        for p in pc.parameters():
            assert p.grad is not None and torch.isfinite(p.grad).all()
        assert out["viewspace_points"].grad is not None
        assert int(out["visibility_filter"].sum()) > 0


@pytest.mark.parametrize("with_offsets", [False, True])
def test_fused_activation_matches_torch(with_offsets):
    """gsd_activate_forward/backward == the reference's torch preamble (gaussian_renderer/__init__.py:79-140)."""
    from gsd_amd.activate import activate
    g = torch.Generator().manual_seed(3)
    P = 5000
    mk = lambda *s: torch.randn(*s, generator=g).to(DEV).requires_grad_(True)  # noqa: E731
    xyz, sc, rot, op, fdc, frest = mk(P, 3), mk(P, 3), mk(P, 4), mk(P, 1), mk(P, 1, 3), mk(P, 15, 3)
    offs = [mk(P, 3), mk(P, 3), mk(P, 4), mk(P, 16, 3)] if with_offsets else [None] * 4
    outs = activate(xyz, sc, rot, op, fdc, frest, *offs)
    z = lambda t, s: torch.zeros(s, device=DEV) if t is None else t  # noqa: E731
    ref = (xyz + z(offs[0], (P, 3)), torch.exp(sc + z(offs[1], (P, 3))),
           torch.nn.functional.normalize(rot + z(offs[2], (P, 4))), torch.sigmoid(op),
           torch.cat([fdc, frest], 1) + z(offs[3], (P, 16, 3)))
    for a, b in zip(outs, ref):
        assert rel_l2(a.detach().cpu(), b.detach().cpu()) <= 1e-6
    ws = [torch.randn(o.shape, generator=g).to(DEV) for o in outs]
    leaves = [xyz, sc, rot, op, fdc, frest] + [o for o in offs if o is not None]
    got = torch.autograd.grad(sum((o * w).sum() for o, w in zip(outs, ws)), leaves)
    want = torch.autograd.grad(sum((o * w).sum() for o, w in zip(ref, ws)), leaves)
    for a, b in zip(got, want):
        assert rel_l2(a.cpu(), b.cpu()) <= 1e-5
    # in-place accumulation into existing .grad buffers
    for t in (xyz, sc, rot, op, fdc, frest):
        t.grad = torch.ones_like(t)
        t._gsd_inplace_grad = True
    outs = activate(xyz, sc, rot, op, fdc, frest, *offs)
    sum((o * w).sum() for o, w in zip(outs, ws)).backward()
    for t, w in zip((xyz, sc, rot, op, fdc, frest), want):
        assert rel_l2((t.grad - 1).cpu(), w.cpu()) <= 1e-5


class _FixedOffsets:
    """A deformation producer with fixed non-zero offsets (dx, dscale, drot, dSH), all differentiable."""

    def __init__(self, P, seed):
        g = torch.Generator(device="cpu").manual_seed(seed)
        mk = lambda *shape: (torch.randn(*shape, generator=g) * 0.02).to(DEV).requires_grad_(True)  # noqa: E731
        self.t = [mk(P, 3), mk(P, 3), mk(P, 4), mk(P, 48)]

    def __call__(self, pts, time, iteration):
        return tuple(self.t)


@pytest.mark.parametrize("offsets", [False, True])
@pytest.mark.parametrize("inplace", [False, "zero", "stale"])
def test_fused_preamble_render_matches_reference_path(offsets, inplace):
    """render(): fused HIP preamble + split-SH rasterizer vs the reference-literal torch preamble: same image,
    parameter grads and offset grads, with plain autograd .grad or in-place FlatGrads accumulation -- into a
    zeroed slab, or into a stale one (after FlatGrads.invalidate, as the fused Adam step leaves it: the first
    backward stores, the second adds)."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.parallel import FlatGrads
    from gsd_amd.scene import make_gaussians
    P = 20_000
    params = make_gaussians(P, 320, 240, seed=9, device=DEV)
    cam = synthetic_camera(320, 240).to(DEV)
    res = []
    for fused in (True, False):
        offs = _FixedOffsets(P, seed=3) if offsets else None
        pc = DeformableGaussians(params, sh_degree=3, offset_model=offs)
        pc.fused_preamble = fused
        flat = FlatGrads(pc.parameters()) if inplace else None
        if inplace == "stale":
            flat.slab.fill_(123.0)
            flat.invalidate()
        for _ in range(2 if inplace else 1):  # twice: the in-place path must accumulate, not overwrite
            out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV))
            (out["render"] * torch.linspace(0, 1, 320, device=DEV)).sum().backward()
        if flat is not None:
            flat.collect()
        grads = [p.grad.clone() for p in pc.parameters()] + ([t.grad.clone() for t in offs.t] if offsets else [])
        res.append((out["render"].detach(), grads))
    assert (res[0][0] - res[1][0]).abs().max() <= 1e-5
    assert len(res[0][1]) == len(res[1][1])
    for a, b in zip(res[0][1], res[1][1]):
        assert rel_l2(a.cpu(), b.cpu()) <= 1e-4


def test_config4_invariants():
    """Full-size (1M Gaussians, 1080p, SH3) size-independent properties."""
    from gsd_amd.introspect import decode
    d = scene_inputs(1_000_000, 1920, 1080, 3, seed=4, device=DEV)
    K, color, radii, geom, binning, img = gpu_forward(d)
    st = decode(1_000_000, 1920, 1080, K, geom, binning, img)
    ranges = st["ranges"].cpu().numpy().astype(np.int64)
    counts = st["tile_count"].cpu().numpy().astype(np.int64)
    nz = counts > 0
    assert counts.sum() == K
    np.testing.assert_array_equal(ranges[nz, 1] - ranges[nz, 0], counts[nz])
    starts = ranges[nz, 0]
    assert starts[0] == 0 and np.all(starts[1:] == (ranges[nz, 1])[:-1])   # ranges partition [0, K)
    pl = st["point_list"].cpu().numpy().astype(np.int64)
    depth_bits = st["depths"].cpu().numpy().view(np.uint32).astype(np.int64)
    key = (depth_bits[pl] << 32) | pl
    tile_of = np.repeat(np.nonzero(nz)[0], counts[nz])
    order_ok = (tile_of[1:] > tile_of[:-1]) | (key[1:] > key[:-1])
    assert order_ok.all()                                  # (tile, depth, id) strictly increasing
    r = radii.cpu().numpy()
    assert set(np.unique(pl)) == set(np.nonzero(r > 0)[0])  # every visible Gaussian is binned
    T = st["final_T"].cpu().numpy()
    assert T.min() >= 1e-4 and T.max() <= 1.0
    nc = st["n_contrib"].cpu().numpy().astype(np.int64)
    W = 1920
    tiles = (np.arange(1080)[:, None] // 16) * ((W + 15) // 16) + (np.arange(W)[None] // 16)
    assert np.all(nc <= counts[tiles])
    assert torch.isfinite(color).all()


def test_sh_grad_views_sums_per_view_sh_gradients():
    """gsd_sh_grad_views over two views' masked dL/dRGB rows (gsd_sh_split.d_rgb) equals the sum of the two
    views' SH gradients from the ordinary split-SH backward; the d_rgb mode leaves every other gradient as it
    was (up to the float-atomic summation order, which varies from run to run)."""
    from gsd_amd import _C
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.scene import make_gaussians
    P, W, H = 20_000, 320, 240
    g = make_gaussians(P, W, H, seed=12, device=DEV)
    means = g.xyz.contiguous()
    scales, rots = torch.exp(g.scaling), torch.nn.functional.normalize(g.rotation, dim=1)
    opac = torch.sigmoid(g.opacity)
    f_dc, f_rest = g.features_dc.contiguous(), g.features_rest.contiguous()
    bg = torch.zeros(3, device=DEV)
    rows, sums, others = [], [torch.zeros_like(f_dc), torch.zeros_like(f_rest)], []
    for k, yaw in enumerate((0.0, 7.0)):
        cam = synthetic_camera(W, H, yaw_deg=yaw).to(DEV)
        tx, ty = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
        split = _C.ShSplit(f_dc, f_rest)
        fwd = _C.rasterize_gaussians(bg, means, None, opac, scales, rots, 1.0, None, cam.world_view_transform,
                                     cam.full_proj_transform, tx, ty, H, W, None, 3, cam.camera_center, False, False,
                                     sh_split=split)
        K, color, radii, geom, binning, img = fwd
        dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(k)).mul_(1e-3).to(DEV)
        d_dc, d_rest = torch.empty_like(f_dc), torch.empty_like(f_rest)
        res = []
        for mode in ("sinks", "rgb"):
            row = torch.full((3 * P + 4,), float("nan"), device=DEV)
            row[3 * P:3 * P + 3] = cam.camera_center
            sp = (_C.ShSplit(f_dc, f_rest, None, d_dc, d_rest, None, accumulate=False) if mode == "sinks" else
                  _C.ShSplit(f_dc, f_rest, None, None, None, None, d_rgb=row[:3 * P]))
            res.append(_C.rasterize_gaussians_backward(bg, means, radii, None, scales, rots, 1.0, None,
                                                       cam.world_view_transform, cam.full_proj_transform, tx, ty,
                                                       dpix, None, 3, cam.camera_center, geom, K, binning, img,
                                                       False, sh_split=sp))
        for a, b in zip(res[0], res[1]):   # the same up to the float-atomic summation order
            if a is not None:
                assert rel_l2(a.cpu(), b.cpu()) <= 1e-5
        sums[0] += d_dc
        sums[1] += d_rest
        rows.append(row)
    views = torch.stack(rows)
    out_dc, out_rest = torch.full_like(f_dc, float("nan")), torch.full_like(f_rest, float("nan"))
    _C.sh_grad_views(3, means, views, P, 16, d_dc=out_dc, d_rest=out_rest, accumulate=False)
    assert rel_l2(out_dc.cpu(), sums[0].cpu()) <= 1e-5 and rel_l2(out_rest.cpu(), sums[1].cpu()) <= 1e-5
    _C.sh_grad_views(3, means, views, P, 16, d_dc=out_dc, d_rest=out_rest, accumulate=True)
    assert rel_l2(out_rest.cpu(), 2 * sums[1].cpu()) <= 1e-5


@pytest.mark.parametrize("P,deg", [(20_000, 3), (20_003, 1)])
def test_sh_grad_views_deferred_view_direction_term(P, deg):
    """gsd_sh_split.defer_view_dir: the backward reads no SH coefficient -- it writes the view's d_rgb row and
    leaves the view-direction term of the SH colour out of dL/dmeans3D -- and gsd_sh_grad_views_ex supplies that
    term summed over the views (d_means).  Summed over two views: deferred dL/dmeans3D + d_means == the ordinary
    backward's dL/dmeans3D; the rows and the SH gradient are those of the non-deferred exchange."""
    from gsd_amd import _C
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.scene import make_gaussians
    W, H = 320, 240
    g = make_gaussians(P, W, H, seed=13, device=DEV)
    means = g.xyz.contiguous()
    scales, rots = torch.exp(g.scaling), torch.nn.functional.normalize(g.rotation, dim=1)
    opac = torch.sigmoid(g.opacity)
    f_dc, f_rest = g.features_dc.contiguous(), g.features_rest.contiguous()
    bg = torch.zeros(3, device=DEV)
    rows, rows_ref = [], []
    m3d_full, m3d_defer = torch.zeros(P, 3, device=DEV), torch.zeros(P, 3, device=DEV)
    for k, yaw in enumerate((0.0, 9.0)):
        cam = synthetic_camera(W, H, yaw_deg=yaw).to(DEV)
        tx, ty = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
        K, color, radii, geom, binning, img = _C.rasterize_gaussians(
            bg, means, None, opac, scales, rots, 1.0, None, cam.world_view_transform, cam.full_proj_transform, tx,
            ty, H, W, None, deg, cam.camera_center, False, False, sh_split=_C.ShSplit(f_dc, f_rest))
        dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(20 + k)).mul_(1e-3).to(DEV)
        for defer, acc, out in ((False, m3d_full, rows_ref), (True, m3d_defer, rows)):
            row = torch.full((3 * P + 4,), float("nan"), device=DEV)
            row[3 * P:3 * P + 3] = cam.camera_center
            row[3 * P + 3] = 0.0
            sp = _C.ShSplit(f_dc, f_rest, None, None, None, None, d_rgb=row[:3 * P], defer_view_dir=defer)
            grads = _C.rasterize_gaussians_backward(bg, means, radii, None, scales, rots, 1.0, None,
                                                    cam.world_view_transform, cam.full_proj_transform, tx, ty, dpix,
                                                    None, deg, cam.camera_center, geom, K, binning, img, False,
                                                    sh_split=sp)
            acc += grads[3]
            out.append(row)
    for r, q in zip(rows, rows_ref):
        assert torch.isfinite(r).all() and rel_l2(r.cpu(), q.cpu()) <= 1e-5
    views = torch.stack(rows)
    d_means = torch.full((P, 3), float("nan"), device=DEV)
    out_dc, out_rest = torch.empty_like(f_dc), torch.empty_like(f_rest)
    ref_dc, ref_rest = torch.empty_like(f_dc), torch.empty_like(f_rest)
    _C.sh_grad_views(deg, means, views, P, 16, d_dc=out_dc, d_rest=out_rest, sh=(f_dc, f_rest), d_means=d_means)
    _C.sh_grad_views(deg, means, views, P, 16, d_dc=ref_dc, d_rest=ref_rest)
    assert torch.equal(out_dc, ref_dc) and torch.equal(out_rest, ref_rest)
    assert torch.isfinite(d_means).all()
    assert float(d_means.abs().max()) > 0.0
    assert rel_l2((m3d_defer + d_means).cpu(), m3d_full.cpu()) <= 1e-5
    assert rel_l2(m3d_defer.cpu(), m3d_full.cpu()) > 1e-3   # the term is not negligible here


def test_sh_grad_views_mean_at_camera_centre():
    """A Gaussian whose mean sits exactly at one view's camera centre is culled in that view (zero dL/dRGB
    row); its SH gradient must be the other views' sum, finite -- not NaN from that view's zero-length
    direction times the zero row."""
    from gsd_amd import _C
    P = 300
    gen = torch.Generator().manual_seed(4)
    means = torch.randn(P, 3, generator=gen).to(DEV)
    cams = [torch.zeros(3), torch.tensor([0.5, -0.25, 1.0])]
    means[7] = cams[0].to(DEV)
    rows = []
    for v, c in enumerate(cams):
        g = torch.randn(P, 3, generator=gen)
        if v == 0:
            g[7] = 0.0   # culled in the view it sits in
        rows.append(torch.cat([g.reshape(-1), c, torch.zeros(1)]).to(DEV))
    f_dc = torch.full((P, 1, 3), float("nan"), device=DEV)
    f_rest = torch.full((P, 15, 3), float("nan"), device=DEV)
    _C.sh_grad_views(3, means, torch.stack(rows), P, 16, d_dc=f_dc, d_rest=f_rest, accumulate=False)
    assert bool(torch.isfinite(f_dc).all()) and bool(torch.isfinite(f_rest).all())
    one = torch.full((P, 1, 3), float("nan"), device=DEV)
    one_rest = torch.full((P, 15, 3), float("nan"), device=DEV)
    _C.sh_grad_views(3, means, rows[1][None].contiguous(), P, 16, d_dc=one, d_rest=one_rest, accumulate=False)
    assert torch.equal(f_dc[7], one[7]) and torch.equal(f_rest[7], one_rest[7])
