"""Shared test setup: import paths, the `gpu` marker, scene builders.

`-m "not gpu"` tests run in the build container (no GPU): oracle vs golden
vectors, host logic, the C-ABI library surface, multi-process gloo.  `-m gpu`
tests are the parity tests proper: HIP path (through the C-ABI) vs the oracle.
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gaussian-splatting_deformable_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def scene_inputs(P, W, H, sh_degree, seed=0, yaw=0.0, opacity_max=None, device="cpu"):
    """Activated rasterizer inputs for a seeded synthetic scene."""
    import torch
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.scene import make_gaussians

    g = make_gaussians(P, W, H, seed=seed)
    cam = synthetic_camera(W, H, yaw_deg=yaw)
    opac = torch.sigmoid(g.opacity)
    if opacity_max is not None:
        opac = opac.clamp_max(opacity_max)
    d = dict(
        means3D=g.xyz, scales=torch.exp(g.scaling), rotations=torch.nn.functional.normalize(g.rotation, dim=1),
        opacities=opac, shs=torch.cat([g.features_dc, g.features_rest], 1),
        viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, campos=cam.camera_center,
        W=W, H=H, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), sh_degree=sh_degree,
        bg=torch.zeros(3))
    if device != "cpu":
        d = {k: (v.to(device) if hasattr(v, "to") else v) for k, v in d.items()}
    return d


def oracle_kwargs(d):
    """Convert scene_inputs() to numpy keyword arguments of oracle.forward/backward."""
    out = {}
    for k, v in d.items():
        if k == "means3D":
            continue
        out[k] = v.detach().cpu().numpy() if hasattr(v, "detach") else v
    return out


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle
