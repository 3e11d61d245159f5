"""Initialisation from a point cloud: ``distCUDA2`` of simple-knn as a HIP kernel
(gsd_knn.hip, C-ABI gsd_knn_mean_dist2) and ``GaussianModel.create_from_pcd`` (scene/gaussian_model.py:807-832)."""
from __future__ import annotations

import torch

from . import _native
from ._C import _dev_f32, _ptr, _stream
from .renderer import inverse_sigmoid
from .scene import GaussianParams

C0 = 0.28209479177387814  # utils/sh_utils.py SH DC constant


def dist_cuda2(points: torch.Tensor) -> torch.Tensor:
    """distCUDA2 (simple_knn ext): mean squared distance of each point to its 3 nearest neighbours, (P,)."""
    if points.dim() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    dev = points.device
    if dev.type != "cuda":
        raise RuntimeError("points must be a HIP device tensor (there is no CPU implementation)")
    lib = _native.load()
    P = int(points.size(0))
    pts = _dev_f32(points, "points", dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    ws = torch.empty(lib.gsd_knn_workspace_bytes(P) + 256, dtype=torch.uint8, device=dev)
    base = (ws.data_ptr() + 255) // 256 * 256
    with torch.cuda.device(dev):
        _native.check(lib.gsd_knn_mean_dist2(P, _ptr(pts), _ptr(out), base, _stream(dev)))
    return out


distCUDA2 = dist_cuda2


def create_from_pcd(points: torch.Tensor, colors: torch.Tensor, sh_degree: int = 3) -> GaussianParams:
    """scene/gaussian_model.py:807-832: DC colour from RGB, zero higher SH, isotropic scales from the 3-NN
    distance (clamped at 1e-7), identity rotations, opacity 0.1 (as logits)."""
    dev = points.device
    pts = points.float().to(dev)
    fused_color = (colors.float().to(dev) - 0.5) / C0
    P = pts.shape[0]
    features = torch.zeros((P, 3, (sh_degree + 1) ** 2), device=dev)
    features[:, :3, 0] = fused_color
    dist2 = torch.clamp_min(dist_cuda2(pts), 0.0000001)
    scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
    rots = torch.zeros((P, 4), device=dev)
    rots[:, 0] = 1
    opac = inverse_sigmoid(0.1 * torch.ones((P, 1), dtype=torch.float, device=dev))
    return GaussianParams(xyz=pts, scaling=scales, rotation=rots, opacity=opac,
                          features_dc=features[:, :, 0:1].transpose(1, 2).contiguous(),
                          features_rest=features[:, :, 1:].transpose(1, 2).contiguous())
