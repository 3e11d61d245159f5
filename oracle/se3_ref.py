"""SE(3) deform oracle (float64 torch) -- TEST INFRASTRUCTURE ONLY.

Restates ``scene/rigid_body.py`` skew (:16-24), exp_so3 (:61-65), exp_se3
(:86-93), to/from_homogenous (:96-100) and the twist normalisation of
``scene/gaussian_model.py:161-165``; the reference's backward is torch
autograd, so ``torch.autograd`` of this function is the gradient oracle.
Below theta = 1e-3 the normalised form loses precision (and 0/0s at w = 0, where the reference NaNs,
SURVEY.md 0.5); there the same map is evaluated un-normalised by series in theta^2.
The rotation update is the build's extension:
q' = normalize(q_R (x) q), q_R = (cos t/2, sin t/2 * w/t), helpers.py:63-70.
"""
from __future__ import annotations

import torch


def skew(w):
    z = torch.zeros(w.shape[0], dtype=w.dtype)
    return torch.stack([torch.stack([z, -w[:, 2], w[:, 1]], 1), torch.stack([w[:, 2], z, -w[:, 0]], 1),
                        torch.stack([-w[:, 1], w[:, 0], z], 1)], 1)


def exp_se3_normalised(S, theta):
    """rigid_body.exp_se3(S, theta) with S = [w/theta, v/theta]: (P,4,4)."""
    w, v = S[:, :3], S[:, 3:]
    W = skew(w)
    I = torch.eye(3, dtype=S.dtype).expand(S.shape[0], 3, 3)
    st, ct = torch.sin(theta)[:, None, None], torch.cos(theta)[:, None, None]
    R = I + st * W + (1 - ct) * (W @ W)
    p = ((theta[:, None, None] * I + (1 - ct) * W + (theta[:, None, None] - st) * (W @ W)) @ v[..., None])[..., 0]
    T = torch.zeros(S.shape[0], 4, 4, dtype=S.dtype)
    T[:, :3, :3] = R
    T[:, :3, 3] = p
    T[:, 3, 3] = 1
    return T


def quat_mult(q1, q2):
    w1, x1, y1, z1 = q1.T
    w2, x2, y2, z2 = q2.T
    return torch.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2]).T


def deform(twist, means, rots=None):
    """(P,6) [w,v], (P,3), optional (P,4) -> (means', rots')."""
    w, v = twist[:, :3], twist[:, 3:]
    theta = torch.linalg.norm(w, dim=1)
    small = theta < 1e-3
    th_safe = torch.where(small, torch.ones_like(theta), theta)
    S = torch.cat([w / th_safe[:, None], v / th_safe[:, None]], 1)
    T = exp_se3_normalised(S, th_safe)
    hom = torch.cat([means, torch.ones_like(means[:, :1])], 1)
    moved = (T @ hom[..., None])[..., 0]
    moved = moved[:, :3] / moved[:, 3:]
    # same map, un-normalised: x + A w x x + B w x (w x x) + v + B w x v + C w x (w x v), series in theta^2
    t2 = (w * w).sum(1, keepdim=True)
    A = 1 - t2 / 6 + t2 * t2 / 120
    B = 0.5 - t2 / 24 + t2 * t2 / 720
    C = 1.0 / 6 - t2 / 120 + t2 * t2 / 5040
    cr = lambda a, b: torch.cross(a, b, dim=1)  # noqa: E731
    series = means + A * cr(w, means) + B * cr(w, cr(w, means)) + v + B * cr(w, v) + C * cr(w, cr(w, v))
    out = torch.where(small[:, None], series, moved)
    qo = None
    if rots is not None:
        half = 0.5 * th_safe
        tt = t2[:, 0]
        sh_over = torch.where(small, 0.5 - tt / 48 + tt * tt / 3840, torch.sin(half) / th_safe)
        ch = torch.where(small, 1 - tt / 8 + tt * tt / 384, torch.cos(half))
        qR = torch.cat([ch[:, None], sh_over[:, None] * w], 1)
        qo = torch.nn.functional.normalize(quat_mult(qR, rots), dim=1)
    return out, qo
