"""render()'s reference-literal input modes and the current-stream contract, on the GPU.

- `pipe.compute_cov3D_python`, `pipe.convert_SHs_python` and `override_color`
  (gaussian_renderer/__init__.py:111-143): what render() hands the rasterizer is checked against a float64
  restatement of those reference lines -- including the quirks SURVEY.md Appendix A.15 names:
  `get_covariance` (gaussian_model.py:800-801) ignores the deform scale / rotation offsets and takes the raw
  `_rotation`, and the Python SH colour uses the undeformed means for the view direction and the features
  without the SH offset.  The image and the rasterizer gradients are checked against the C oracle fed the same
  precomputed inputs, and every parameter / offset / override-colour gradient against float64 autograd of the
  restatement with the oracle's gradients as the upstream.
- A forward + backward issued on a non-default `torch.cuda.Stream` whose inputs are written on that stream behind
  a long device-side sleep: the library must run on the caller's current stream (rasterize_points.cu has no stream
  argument; here every entry point takes the current stream), so it sees the written inputs.  Forward outputs are
  bit-identical to the default-stream run; gradients are float-atomic sums, equal within the run-to-run noise bound
  of test_gpu_parity.test_backward_run_to_run_noise (rel L2 2e-6).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from test_gpu_parity import _FixedOffsets, check_forward_against, gpu_backward, gpu_forward, oracle_fwd_bwd, rel_l2

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _cov_f64(scales, q):
    """utils/general_utils.py:78-110 + gaussian_model.py:634-638 in float64: build_rotation normalises q."""
    from oracle.torch_ref import quat_R
    R = quat_R(q / q.norm(dim=1, keepdim=True))
    L = R * scales[:, None, :]
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1)


MODES = [  # (name, PipelineParams flags, override_color)
    ("cov3D_python", dict(compute_cov3D_python=True), False),
    ("SHs_python", dict(convert_SHs_python=True), False),
    ("override_color", {}, True),
    ("cov3D_and_SHs_python", dict(compute_cov3D_python=True, convert_SHs_python=True), False),
]


@pytest.mark.parametrize("name,pipe_kw,override", MODES, ids=[m[0] for m in MODES])
def test_render_input_modes_match_reference_lines_and_oracle(oracle_mod, monkeypatch, name, pipe_kw, override):
    import gsd_amd.renderer as R
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.scene import make_gaussians
    from oracle.torch_ref import sh_rgb
    P, W, H, deg = 6_000, 320, 240, 3
    params = make_gaussians(P, W, H, seed=13, device=DEV)
    offs = _FixedOffsets(P, seed=4)
    pc = DeformableGaussians(params, sh_degree=deg, offset_model=offs)
    cam = synthetic_camera(W, H).to(DEV)
    bg = torch.zeros(3, device=DEV)
    ov = None
    if override:
        ov = torch.rand(P, 3, generator=torch.Generator().manual_seed(6)).to(DEV).requires_grad_(True)

    seen = {}

    class Recording(R.GaussianRasterizer):
        def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                    cov3D_precomp=None):
            seen.update(means3D=means3D, opacities=opacities, shs=shs, colors=colors_precomp, scales=scales,
                        rotations=rotations, cov3D=cov3D_precomp)
            return super().forward(means3D, means2D, opacities, shs=shs, colors_precomp=colors_precomp,
                                   scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp)

    monkeypatch.setattr(R, "GaussianRasterizer", Recording)
    out = render(cam, pc, default_pipe(**pipe_kw), bg, override_color=ov)
    assert seen, "render() did not take the reference-literal path"
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(8)).mul_(1e-3).to(DEV)
    (out["render"] * dpix).sum().backward()

    # 1. what render() hands the rasterizer == the reference lines, restated in float64
    leaves = [t.detach().cpu().double().requires_grad_(True) for t in pc.parameters()]
    xyz, fdc, frest, op, sc, rot = leaves
    off64 = [t.detach().cpu().double().requires_grad_(True) for t in offs.t]
    dx, ds, dq, dsh = off64
    campos = cam.camera_center.detach().cpu().double()
    ref = {"means3D": xyz + dx, "opacities": torch.sigmoid(op)}
    if pipe_kw.get("compute_cov3D_python"):
        ref["cov3D"] = _cov_f64(torch.exp(sc), rot)          # no ds / dq: gaussian_model.py:800-801
    else:
        ref["scales"] = torch.exp(sc + ds)
        ref["rotations"] = torch.nn.functional.normalize(rot + dq)
    ov64 = None
    if override:
        ov64 = ov.detach().cpu().double().requires_grad_(True)
        ref["colors"] = ov64
    elif pipe_kw.get("convert_SHs_python"):
        feats = torch.cat([fdc, frest], 1)                   # no dsh; undeformed means for the direction
        d = xyz - campos
        ref["colors"] = torch.clamp_min(sh_rgb(deg, feats, d / d.norm(dim=1, keepdim=True)), 0.0)
    else:
        ref["shs"] = torch.cat([fdc, frest], 1) + dsh.reshape(-1, 16, 3)
    for k, want in ref.items():
        got = seen[k]
        assert got is not None, k
        assert rel_l2(got.detach().cpu().double().reshape(want.shape), want.detach()) <= 1e-6, k
    for k in set(seen) - set(ref):
        assert seen[k] is None, k

    # 2. the rasterizer on those inputs == the C oracle fed the same (GPU-computed) precomputed inputs
    d = dict(means3D=seen["means3D"].detach(), opacities=seen["opacities"].detach(),
             shs=None if seen["shs"] is None else seen["shs"].detach(),
             scales=None if seen["scales"] is None else seen["scales"].detach(),
             rotations=None if seen["rotations"] is None else seen["rotations"].detach(),
             viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, campos=cam.camera_center,
             W=W, H=H, tanfovx=float(np.tan(cam.FoVx * 0.5)), tanfovy=float(np.tan(cam.FoVy * 0.5)),
             sh_degree=deg, bg=bg)
    colors = None if seen["colors"] is None else seen["colors"].detach().contiguous()
    cov = None if seen["cov3D"] is None else seen["cov3D"].detach().contiguous()
    o, ob = oracle_fwd_bwd(oracle_mod, d, dpix, colors=colors, cov3D=cov)
    K = check_forward_against(o, d, gpu_forward(d, colors=colors, cov3D=cov), colors=colors)
    assert K > P
    assert np.array_equal(out["radii"].cpu().numpy(), o["radii"])
    assert float(np.abs(out["render"].detach().cpu().numpy() - o["color"]).max()) <= 1e-2
    vs = out["viewspace_points"].grad.cpu().numpy()
    assert rel_l2(vs, ob["dL_dmeans2D"].reshape(vs.shape)) <= 1e-4

    # 3. every gradient == float64 autograd of the restatement, fed the oracle's rasterizer gradients
    up = {"means3D": ob["dL_dmeans3D"], "opacities": ob["dL_dopacity"], "cov3D": ob["dL_dcov3D"],
          "scales": ob["dL_dscales"], "rotations": ob["dL_drotations"], "colors": ob["dL_dcolors"],
          "shs": ob["dL_dsh"]}
    outs = [ref[k] for k in ref]
    grads = [torch.from_numpy(np.ascontiguousarray(up[k])).double().reshape(ref[k].shape) for k in ref]
    torch.autograd.backward(outs, grads)
    pairs = list(zip(pc.parameters(), leaves)) + list(zip(offs.t, off64))
    if override:
        pairs.append((ov, ov64))
    checked = 0
    for gpu_t, cpu_t in pairs:
        want = cpu_t.grad
        got = gpu_t.grad
        if want is None or float(want.abs().max()) == 0.0:
            assert got is None or float(got.abs().max()) == 0.0   # unused inputs (e.g. ds, dq under cov3D)
            continue
        assert got is not None
        assert rel_l2(got.detach().cpu().double(), want) <= 1e-4, (name, tuple(gpu_t.shape), rel_l2(got.cpu(), want))
        checked += 1
    assert checked >= 5


def test_forward_backward_on_a_side_stream_follows_the_current_stream():
    from conftest import scene_inputs
    P, W, H, deg = 60_000, 640, 480, 3
    d = scene_inputs(P, W, H, deg, seed=5, device=DEV)
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(5)).mul_(1e-3).to(DEV)
    ref_fwd = gpu_forward(d)
    ref_bwd = [t.cpu() for t in gpu_backward(d, ref_fwd, dpix)]
    torch.cuda.synchronize()

    side = torch.cuda.Stream(device=DEV)
    true_means = d["means3D"].clone()
    d2 = dict(d)
    d2["means3D"] = torch.full_like(true_means, float("nan"))   # poisoned until the side stream writes it
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)                            # the write lands well after the launches
        d2["means3D"].copy_(true_means)
        fwd = gpu_forward(d2)
        bwd = gpu_backward(d2, fwd, dpix)
    side.synchronize()
    from gsd_amd.introspect import decode
    K, color, radii, geom, binning, img = fwd
    assert K == ref_fwd[0]
    assert torch.equal(radii, ref_fwd[2]) and torch.equal(color, ref_fwd[1])
    a, b = decode(P, W, H, K, geom, binning, img), decode(P, W, H, K, *ref_fwd[3:])
    for k in ("ranges", "point_list", "final_T", "n_contrib"):
        assert torch.equal(a[k], b[k]), k      # the state the backward reads: bit-identical
    vis = radii > 0                            # per-Gaussian state is written for the visible Gaussians only
    for k in ("means2D", "conic_opacity", "depths"):
        assert torch.equal(a[k][vis], b[k][vis]), k
    for i, (x, y) in enumerate(zip(bwd, ref_bwd)):
        if y.numel():
            assert torch.isfinite(x).all(), i
            assert rel_l2(x.cpu().numpy(), y.numpy()) <= 2e-6, (i, rel_l2(x.cpu().numpy(), y.numpy()))


@pytest.mark.parametrize("offsets", [False, True])
def test_render_save_ply_writes_the_frame(tmp_path, monkeypatch, offsets):
    """render(..., save_ply=True) (gaussian_renderer/__init__.py:165-167): test_ply/point_cloud_{int(time*1000)}.ply
    under the working directory holds exactly the means, opacities and rotations render() returned (deformed and
    activated; the raw-parameter path builds them lazily), the raw scaling and the raw SH pieces."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.io import read_ply
    from gsd_amd.scene import make_gaussians
    monkeypatch.chdir(tmp_path)
    P = 5_000
    params = make_gaussians(P, 160, 120, seed=8, device=DEV)
    pc = DeformableGaussians(params, sh_degree=3, offset_model=_FixedOffsets(P, seed=5) if offsets else None)
    cam = synthetic_camera(160, 120).to(DEV)
    cam.time = 0.25
    with torch.no_grad():
        out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV), save_ply=True)
    v = read_ply(str(tmp_path / "test_ply" / "point_cloud_250.ply"))
    col = lambda *ks: np.stack([v[k] for k in ks], 1)  # noqa: E731
    assert np.array_equal(col("x", "y", "z"), out["means3D"].detach().cpu().numpy())
    assert np.array_equal(col("opacity"), out["opacities"].detach().cpu().numpy())
    assert np.array_equal(col("rot_0", "rot_1", "rot_2", "rot_3"), out["rotations"].detach().cpu().numpy())
    assert np.array_equal(col("scale_0", "scale_1", "scale_2"), pc._scaling.detach().cpu().numpy())
    assert np.array_equal(col(*[f"f_rest_{3 * 15 - 15 + i}" for i in range(15)]),
                          pc._features_rest.detach()[:, :, 2].cpu().numpy())
    if offsets:   # deformed: the file is not the raw parameters
        assert not np.array_equal(col("x", "y", "z"), pc._xyz.detach().cpu().numpy())
