"""Float64 differentiable restatement of the reference forward -- TEST INFRASTRUCTURE ONLY.

Used to pin the oracle's analytic backward (raster_oracle.c, restating
backward.cu) to torch.autograd of the forward (restating forward.cu): with
the discrete decisions (visibility, tile lists, skip/termination masks) held
fixed, d(image)/d(inputs) from autograd must equal the reference's hand-written
gradients, except for the documented quirks,
which the test scenes avoid (opacity < 0.99, no Jacobian clamping).

Conventions follow the glm column-major code: Sigma = R S^2 R^T with R the
textbook rotation of quaternion (r,x,y,z); cov2D = J V Sigma V^T J^T + 0.3 I
(forward.cu:74-113, 118-152).
"""
from __future__ import annotations

import math

import torch

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435]


def sh_rgb(deg, sh, d):
    """forward.cu:20-71 without the clamp; sh (P,M,3), d unit (P,3) -> (P,3)."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = C0 * sh[:, 0]
    if deg > 0:
        r = r - C1 * y * sh[:, 1] + C1 * z * sh[:, 2] - C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            r = (r + C2[0] * xy * sh[:, 4] + C2[1] * yz * sh[:, 5] + C2[2] * (2 * zz - xx - yy) * sh[:, 6] +
                 C2[3] * xz * sh[:, 7] + C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                r = (r + C3[0] * y * (3 * xx - yy) * sh[:, 9] + C3[1] * xy * z * sh[:, 10] +
                     C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12] +
                     C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + C3[5] * z * (xx - yy) * sh[:, 14] +
                     C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r + 0.5


def quat_R(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def forward_image(means3D, means2D, shs, opac, scales, rots, view, proj, campos, W, H, tanx, tany, deg, bg,
                  ranges, point_list, visible, scale_mod=1.0):
    """Differentiable float64 image (3,H,W) given the oracle's binning (ranges, point_list, visible)."""
    fx = W / (2.0 * tanx)
    fy = H / (2.0 * tany)
    Vm = view.reshape(4, 4).t()   # math matrix: stored column-major (auxiliary.h:58-77)
    Pm = proj.reshape(4, 4).t()
    hom = torch.cat([means3D, torch.ones_like(means3D[:, :1])], 1)
    t = hom @ Vm[:3].t()                     # view space (P,3)
    ph = hom @ Pm.t()
    pw = 1.0 / (ph[:, 3] + 1e-7)
    ndc = ph[:, :2] * pw[:, None] + means2D[:, :2]   # means2D: the screen-space dummy (its grad = dL/dndc)
    pix_x = ((ndc[:, 0] + 1.0) * W - 1.0) * 0.5
    pix_y = ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5
    R = quat_R(rots)
    S = torch.diag_embed(scale_mod * scales)
    RS = R @ S
    Sigma = RS @ RS.transpose(1, 2)
    tz = t[:, 2]
    J = torch.zeros(means3D.shape[0], 2, 3, dtype=means3D.dtype)
    J[:, 0, 0] = fx / tz
    J[:, 0, 2] = -fx * t[:, 0] / (tz * tz)
    J[:, 1, 1] = fy / tz
    J[:, 1, 2] = -fy * t[:, 1] / (tz * tz)
    JV = J @ Vm[:3, :3]
    cov2 = JV @ Sigma @ JV.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    con_a, con_b, con_c = c / det, -b / det, a / det
    d = means3D - campos[None]
    d = d / torch.linalg.norm(d, dim=1, keepdim=True)
    rgb = torch.clamp_min(sh_rgb(deg, shs, d), 0.0)
    img = torch.zeros(3, H, W, dtype=means3D.dtype)
    gx = (W + 15) // 16
    gy = (H + 15) // 16
    rows = []
    for ty in range(gy):
        for tx in range(gx):
            r0, r1 = int(ranges[ty * gx + tx, 0]), int(ranges[ty * gx + tx, 1])
            ys = torch.arange(ty * 16, min(ty * 16 + 16, H))
            xs = torch.arange(tx * 16, min(tx * 16 + 16, W))
            PY, PX = torch.meshgrid(ys, xs, indexing="ij")
            PXf, PYf = PX.reshape(-1).double(), PY.reshape(-1).double()
            if r1 <= r0:
                tile = bg[:, None].expand(3, PXf.numel())
            else:
                ids = torch.as_tensor(point_list[r0:r1].astype("int64"))
                dx = pix_x[ids][None] - PXf[:, None]
                dy = pix_y[ids][None] - PYf[:, None]
                power = -0.5 * (con_a[ids][None] * dx * dx + con_c[ids][None] * dy * dy) - con_b[ids][None] * dx * dy
                G = torch.exp(power)
                alpha = opac[ids, 0][None] * G
                keep = (power <= 0) & (alpha.detach() >= 1.0 / 255.0)
                alpha = torch.where(keep, alpha, torch.zeros_like(alpha))
                one_m = 1 - alpha
                Tb = torch.cumprod(torch.cat([torch.ones_like(one_m[:, :1]), one_m[:, :-1]], 1), 1)
                Ta = Tb * one_m
                # termination: the first kept k with T_before*(1-alpha) < 1e-4 is dropped and ends the pixel
                stop = keep & (Ta.detach() < 1e-4)
                first = torch.where(stop.any(1), stop.float().argmax(1), torch.full_like(stop[:, 0], stop.shape[1],
                                                                                          dtype=torch.long))
                alive = torch.arange(stop.shape[1])[None] < first[:, None]
                w = torch.where(alive, alpha * Tb, torch.zeros_like(alpha))
                Tfin = torch.where(alive, one_m, torch.ones_like(one_m)).prod(1)
                tile = (w @ rgb[ids]).t() + bg[:, None] * Tfin[None]
            rows.append((ys, xs, tile))
    for ys, xs, tile in rows:
        img[:, ys[0]:ys[-1] + 1, xs[0]:xs[-1] + 1] = tile.reshape(3, len(ys), len(xs))
    return img
