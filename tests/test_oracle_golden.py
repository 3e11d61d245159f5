"""Pin the oracle (and the product's host-side camera code) against vectors the
reference's own Python modules produced (tests/golden/make_golden.py)."""
from __future__ import annotations

import numpy as np
import torch

from conftest import golden


def test_camera_matrices_match_reference():
    """gsd_amd.camera restates graphics_utils + cameras.py:55-58 exactly."""
    from gsd_amd.camera import Camera
    g = golden("camera.npz")
    for k in range(3):
        cam = Camera(g[f"R{k}"], g[f"T{k}"], float(g[f"fovx{k}"]), float(g[f"fovy{k}"]), int(g[f"W{k}"]),
                     int(g[f"H{k}"]))
        np.testing.assert_array_equal(cam.world_view_transform.numpy(), g[f"view{k}"])
        np.testing.assert_array_equal(cam.projection_matrix.numpy(), g[f"proj{k}"])
        np.testing.assert_array_equal(cam.full_proj_transform.numpy(), g[f"full{k}"])
        np.testing.assert_array_equal(cam.camera_center.numpy(), g[f"campos{k}"])


def test_oracle_sh_matches_reference_eval_sh(oracle_mod):
    """forward.cu:20-71 restated in C == utils/sh_utils.eval_sh (+0.5, clamp >= 0)."""
    g = golden("sh.npz")
    for deg in range(4):
        sh = g[f"sh{deg}"]                      # (N,3,16): eval_sh layout [..., C, coeff]
        dirs = g[f"dirs{deg}"].astype(np.float32)
        ref = g[f"out{deg}"] + 0.5
        sh_pmc = np.ascontiguousarray(np.transpose(sh, (0, 2, 1)))  # rasterizer layout (P, M, 3)
        campos = np.zeros(3, np.float32)
        rgb, cl = oracle_mod.sh_to_rgb(deg, dirs * 3.0, campos, sh_pmc)   # |pos - campos| = 3 -> dir
        np.testing.assert_allclose(rgb, np.maximum(ref, 0.0), rtol=0, atol=2e-6)
        np.testing.assert_array_equal(cl, ref < 0)


def test_oracle_cov3d_matches_reference_python_covariance(oracle_mod):
    """computeCov3D (forward.cu:118-152) == build_scaling_rotation/strip_symmetric for unit quaternions."""
    g = golden("cov3d.npz")
    cov = oracle_mod.cov3d(g["scales"], g["rotations"])
    scale = np.abs(g["cov"]).max(axis=1, keepdims=True)
    np.testing.assert_allclose(cov / scale, g["cov"] / scale, rtol=0, atol=2e-6)


def test_higher_msb_table(oracle_mod):
    """rasterizer_impl.cu:35-50 getHigherMsb: the sort end bits of SURVEY.md 0.6."""
    for tiles, msb in [(625, 10), (2500, 12), (8160, 13), (32400, 15), (1, 1), (2, 2), (3, 2), (4, 3)]:
        assert oracle_mod.higher_msb(tiles) == msb, tiles


def test_se3_oracle_matches_reference_exp_se3():
    """oracle/se3_ref.py == scene/rigid_body.exp_se3 on normalised twists (float64)."""
    from oracle import se3_ref
    g = golden("se3.npz")
    tw = torch.tensor(g["twist"])
    x = torch.tensor(g["means"])
    out, _ = se3_ref.deform(tw, x)
    theta = np.linalg.norm(g["twist"][:, :3], axis=1)
    ok = theta >= 1e-6       # below that the reference's normalisation is itself 0/0-fragile
    np.testing.assert_allclose(out.numpy()[ok], g["moved"][ok], rtol=1e-9, atol=1e-9)
    # the tiny-theta rows: the reference is finite there and our limit agrees to first order
    np.testing.assert_allclose(out.numpy()[~ok], g["moved"][~ok], rtol=0, atol=1e-6)
    # zero twist: the reference NaNs; the build's guarded map is the identity
    assert np.isnan(g["zero_twist_T"][0, :3]).all()
    z, _ = se3_ref.deform(torch.zeros(2, 6, dtype=torch.float64), x[:2])
    np.testing.assert_array_equal(z.numpy(), x[:2].numpy())


def test_product_sh_restatement_matches_reference():
    from gsd_amd.sh import eval_sh
    g = golden("sh.npz")
    for deg in range(4):
        out = eval_sh(deg, torch.tensor(g[f"sh{deg}"]), torch.tensor(g[f"dirs{deg}"]))
        np.testing.assert_allclose(out.numpy(), g[f"out{deg}"], rtol=0, atol=1e-6)


def test_loss_oracle_matches_reference_fixture():
    """oracle/loss_ref.py (the fp32 restatement gsd_amd.loss is tested against) vs the values the
    reference's utils/loss_utils.py produced for the same images (tests/golden/loss.npz)."""
    import torch
    from oracle import loss_ref
    g = golden("loss.npz")
    x, y = torch.from_numpy(g["img1"]), torch.from_numpy(g["img2"])
    assert abs(float(loss_ref.l1_loss(x, y)) - float(g["l1"])) <= 1e-7
    assert abs(float(loss_ref.ssim(x, y)) - float(g["ssim"])) <= 1e-6


def test_knn_oracle_against_scipy():
    """oracle/knn_ref.py (distCUDA2 restatement) vs scipy's KD-tree 3-NN on a small cloud (float64 within
    float32 rounding), plus the FLT_MAX padding below four points."""
    import numpy as np
    from scipy.spatial import cKDTree
    from oracle.knn_ref import mean_dist2
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(400, 3)).astype(np.float32)
    d, _ = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k=4)
    np.testing.assert_allclose(mean_dist2(pts), (d[:, 1:] ** 2).mean(1), rtol=1e-5)
    assert np.isinf(mean_dist2(pts[:2])).all()
    np.testing.assert_allclose(mean_dist2(pts[:3]), np.finfo(np.float32).max / 3, rtol=1e-6)
