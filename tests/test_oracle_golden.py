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


def _mlp_fixture():
    g = golden("mlp.npz")
    names = [str(n) for n in g["names"]]
    sd = {n: torch.from_numpy(g["w:" + n]) for n in names}
    return g, names, sd


def test_deform_mlp_oracle_matches_reference_network():
    """oracle/deform_mlp_ref.py (float64) vs the reference's own DirectTemporalNeRF (gaussian_model.py:242-316,
    float32, seeded init; tests/golden/mlp.npz): the four heads at iteration 5000 within float32 rounding of the
    reference, dL/dx and every parameter gradient of its autograd within rel L2 1e-5, and exact zeros below
    iteration 3000 (:308-313)."""
    from oracle import deform_mlp_ref
    g, names, sd = _mlp_fixture()
    x = torch.from_numpy(g["x"]).double().requires_grad_(True)
    t = torch.from_numpy(g["t"]).double()
    sd64 = {n: v.double().requires_grad_(True) for n, v in sd.items()}
    outs = deform_mlp_ref.forward(sd64, x, t, int(g["iteration"]))
    heads = ("dx", "dscale", "drot", "dshs")
    for k, o in zip(heads, outs):
        want = g["out:" + k].astype(np.float64)
        assert np.abs(o.detach().numpy() - want).max() <= 2e-6 * max(1.0, np.abs(want).max()), k
    loss = sum((o * torch.from_numpy(g["upstream:" + k]).double()).sum() for k, o in zip(heads, outs))
    grads = torch.autograd.grad(loss, [x] + [sd64[n] for n in names])
    for n, gr in zip(["x"] + names, grads):
        want = g["grad:" + n].astype(np.float64)
        rel = np.linalg.norm(gr.numpy() - want) / max(np.linalg.norm(want), 1e-30)
        assert rel <= 1e-5, (n, rel)
    zero = deform_mlp_ref.forward(sd, torch.from_numpy(g["x"]), torch.from_numpy(g["t"]), 2000)
    for k, z in zip(heads, zero):
        assert not g["zero2000:" + k].any() and not z.any() and z.shape == g["zero2000:" + k].shape


def test_product_mlp_module_matches_reference_network_on_cpu():
    """gsd_amd.deform_mlp.DirectTemporalNeRF (its torch path, float32 on the CPU) loads the reference network's
    state dict by the same names and reproduces its float32 outputs and autograd gradients."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    g, names, sd = _mlp_fixture()
    net = DirectTemporalNeRF()
    net.load_state_dict(sd)
    assert [n for n, _ in net.named_parameters()] == names
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    outs = net(x, torch.from_numpy(g["t"]), int(g["iteration"]))
    heads = ("dx", "dscale", "drot", "dshs")
    for k, o in zip(heads, outs):
        want = g["out:" + k]
        assert np.abs(o.detach().numpy() - want).max() <= 1e-5 * max(1.0, np.abs(want).max()), k
    loss = sum((o * torch.from_numpy(g["upstream:" + k])).sum() for k, o in zip(heads, outs))
    grads = torch.autograd.grad(loss, [x] + [p for _, p in net.named_parameters()])
    for n, gr in zip(["x"] + names, grads):
        want = g["grad:" + n]
        rel = np.linalg.norm(gr.numpy() - want) / max(np.linalg.norm(want), 1e-30)
        assert rel <= 1e-5, (n, rel)


def _densify_fixture_run(g, make_model, step, stats, densify, reset, snapshot, tol):
    """Replays tests/golden/densify.npz's sequence on a model and compares every snapshot with the reference's."""
    groups = [str(n) for n in g["group_names"]]
    P = int(g["P"])
    m = make_model([g["init:" + n] for n in groups], [float(v) for v in g["lrs"]], float(g["percent_dense"]))
    for k in range(2):
        step(m, [g[f"step{k}:" + n] for n in groups])
    for k in range(3):
        stats(m, g[f"view{k}:grad"], g[f"view{k}:radii"])
    got = snapshot(m)
    for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
        np.testing.assert_allclose(got["stat:" + n], g["stats:" + n], rtol=0, atol=tol["stat"], err_msg=n)
    assert got["xyz"].shape[0] == P

    def compare(tag):
        got = snapshot(m)
        for n in groups:
            assert got[n].shape == g[f"{tag}:{n}"].shape, (tag, n)
            np.testing.assert_allclose(got[n], g[f"{tag}:{n}"], rtol=0, atol=tol["param"], err_msg=f"{tag} {n}")
            np.testing.assert_allclose(got[n + ":exp_avg"], g[f"{tag}:{n}:exp_avg"], rtol=0, atol=tol["m"],
                                       err_msg=f"{tag} {n} m")
            np.testing.assert_allclose(got[n + ":exp_avg_sq"], g[f"{tag}:{n}:exp_avg_sq"], rtol=0, atol=tol["v"],
                                       err_msg=f"{tag} {n} v")
        for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
            np.testing.assert_allclose(got["stat:" + n], g[f"{tag}:stat:{n}"], rtol=0, atol=tol["stat"])

    densify(m, float(g["max_grad"]), float(g["min_opacity"]), float(g["extent"]), float(g["max_screen_size"]),
            g["split_samples"])
    compare("densified")
    reset(m)
    compare("reset")
    step(m, [g["after:grad:" + n] for n in groups])
    compare("after")


def test_densify_oracle_matches_reference_gaussian_model(monkeypatch):
    """oracle/densify_ref.py vs the reference's own GaussianModel + torch.optim.Adam (tests/golden/densify.npz):
    two Adam steps, three views of statistics, densify_and_prune with the reference's split samples,
    reset_opacity and one more step -- identical point count, parameters, moments and statistics."""
    from oracle import densify_ref

    def make(init, lrs, pd):
        return densify_ref.RefGaussians(*(torch.from_numpy(v) for v in init), lrs=lrs, percent_dense=pd)

    def step(m, gs):
        for p, gr in zip(m.params(), gs):
            p.grad = torch.from_numpy(gr).clone()
        m.optimizer.step()
        m.optimizer.zero_grad()

    def stats(m, vg, radii):
        m.add_stats(torch.from_numpy(vg), torch.from_numpy(radii))

    def densify(m, max_grad, min_op, extent, mss, samples):
        monkeypatch.setattr(torch, "normal", lambda mean, std: torch.from_numpy(samples).to(mean.dtype))
        m.densify_and_prune(max_grad, min_op, extent, mss)
        monkeypatch.undo()

    def snapshot(m):
        out = {}
        for n, p in zip(["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"], m.params()):
            out[n] = p.detach().numpy()
            st = m.optimizer.state[p]
            out[n + ":exp_avg"], out[n + ":exp_avg_sq"] = st["exp_avg"].numpy(), st["exp_avg_sq"].numpy()
        for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
            out["stat:" + n] = getattr(m, n).numpy()
        return out

    _densify_fixture_run(golden("densify.npz"), make, step, stats, densify, lambda m: m.reset_opacity(), snapshot,
                         dict(param=1e-7, m=1e-9, v=1e-12, stat=1e-9))


def test_loss_oracle_gradient_matches_reference_autograd():
    """oracle/loss_ref.py's autograd vs the reference's utils/loss_utils.py autograd (tests/golden/loss_grad.npz):
    d SSIM / d image and d(0.8 L1 + 0.2 (1 - SSIM)) / d image (train.py:529)."""
    from oracle import loss_ref
    g = golden("loss_grad.npz")
    x = torch.from_numpy(g["img1"]).requires_grad_(True)
    y = torch.from_numpy(g["img2"])
    (ds,) = torch.autograd.grad(loss_ref.ssim(x, y), [x])
    np.testing.assert_allclose(ds.numpy(), g["dssim_dimg1"], rtol=0, atol=1e-6 * np.abs(g["dssim_dimg1"]).max())
    loss = loss_ref.l1_ssim_loss(x, y)
    (dl,) = torch.autograd.grad(loss, [x])
    assert abs(float(loss) - float(g["loss"])) <= 1e-6
    np.testing.assert_allclose(dl.numpy(), g["dloss_dimg1"], rtol=0, atol=1e-6 * np.abs(g["dloss_dimg1"]).max())
