"""Host-side behaviour of the drop-in API that needs no GPU: argument
validation (diff_gaussian_rasterization/__init__.py:187-220), the loud
refusal of CPU tensors (no CPU fallback), settings layout, and the Python-path
helpers render() uses."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import golden


def settings():
    from gsd_amd import GaussianRasterizationSettings
    return GaussianRasterizationSettings(image_height=32, image_width=32, tanfovx=0.5, tanfovy=0.5, bg=torch.zeros(3),
                                         scale_modifier=1.0, viewmatrix=torch.eye(4), projmatrix=torch.eye(4),
                                         sh_degree=0, campos=torch.zeros(3), prefiltered=False, debug=False)


def test_settings_field_order_matches_reference():
    from gsd_amd import GaussianRasterizationSettings
    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug")


def test_drop_in_module_names():
    import diff_gaussian_rasterization as dgr
    import gaussian_renderer
    assert hasattr(dgr, "GaussianRasterizer") and hasattr(dgr, "GaussianRasterizationSettings")
    assert hasattr(dgr, "rasterize_gaussians") and hasattr(dgr._C, "rasterize_gaussians_backward")
    assert hasattr(dgr._C, "mark_visible") and callable(gaussian_renderer.render)


def test_rasterizer_argument_validation():
    from gsd_amd import GaussianRasterizer
    r = GaussianRasterizer(settings())
    m = torch.zeros(4, 3)
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(m, m, torch.ones(4, 1))
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3), colors_precomp=torch.zeros(4, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3), scales=m, rotations=torch.zeros(4, 4),
          cov3D_precomp=torch.zeros(4, 6))


def test_cpu_tensors_fail_loudly():
    """No CPU fallback: host tensors are refused before any compute."""
    from gsd_amd import GaussianRasterizer
    r = GaussianRasterizer(settings())
    m = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="HIP device tensor"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3), scales=m, rotations=torch.zeros(4, 4))
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        r(torch.zeros(4, 2), m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3), scales=m, rotations=torch.zeros(4, 4))


def test_python_covariance_matches_reference():
    """compute_cov3D_python helpers (general_utils restated device-agnostic) vs golden."""
    from gsd_amd.renderer import build_covariance_from_scaling_rotation
    g = golden("cov3d.npz")
    cov = build_covariance_from_scaling_rotation(torch.tensor(g["scales"]), 1.0, torch.tensor(g["rotations"]))
    np.testing.assert_allclose(cov.numpy(), g["cov"], rtol=1e-6, atol=1e-12)


def test_scene_generator_is_seeded_and_in_front():
    from gsd_amd.scene import make_gaussians
    a = make_gaussians(1000, 400, 300, seed=3)
    b = make_gaussians(1000, 400, 300, seed=3)
    assert torch.equal(a.xyz, b.xyz) and torch.equal(a.features_rest, b.features_rest)
    assert float(a.xyz[:, 2].min()) >= 2.0 and float(a.xyz[:, 2].max()) <= 10.0
    assert a.features_dc.shape == (1000, 1, 3) and a.features_rest.shape == (1000, 15, 3)
