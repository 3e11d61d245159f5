"""Per-Gaussian SE(3) deform as a torch autograd op over the fused HIP kernels.

Forward/backward of ``scene/rigid_body.py`` exp_se3 (:86-93) applied to the
means (``gaussian_renderer/__init__.py:90-95``) and, as the build's extension,
to the rotations (include/gsd_raster.h ``gsd_se3_deform_forward``).  The
reference's backward is torch autograd through ~30 small kernels with
(P,3,3)/(P,4,4) temporaries; here one kernel each way, 52 B in / 28 B out per
Gaussian forward.
"""
from __future__ import annotations

import torch

from . import _C


class _SE3Deform(torch.autograd.Function):
    @staticmethod
    def forward(ctx, twist, means, rotations):
        has_rot = rotations is not None and rotations.numel() > 0
        m_out, q_out = _C.se3_deform_forward(twist, means, rotations if has_rot else None)
        ctx.has_rot = has_rot
        ctx.save_for_backward(twist, means, rotations if has_rot else torch.empty(0, device=means.device))
        if not has_rot:
            q_out = torch.empty(0, device=means.device)
        return m_out, q_out

    @staticmethod
    def backward(ctx, g_means, g_rot):
        twist, means, rotations = ctx.saved_tensors
        q = rotations if ctx.has_rot else None
        if g_means is None:
            g_means = torch.zeros_like(means)
        if q is not None and g_rot is None:
            g_rot = torch.zeros_like(q)
        d_tw, d_m, d_q = _C.se3_deform_backward(twist, means, q, g_means, g_rot if q is not None else None)
        return d_tw, d_m, d_q


def se3_deform(twist: torch.Tensor, means: torch.Tensor, rotations: torch.Tensor | None = None):
    """(P,6) twist [w, v], (P,3) means, optional (P,4) rotations -> (means', rotations' or None)."""
    m, q = _SE3Deform.apply(twist, means, rotations)
    return m, (q if rotations is not None else None)
