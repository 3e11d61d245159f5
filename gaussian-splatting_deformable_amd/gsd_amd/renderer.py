"""Drop-in ``render()`` (L2) and the minimal Gaussian container it reads.

``render`` mirrors ``gaussian_renderer/__init__.py:20-195``: same signature,
same camera/model attributes read, same returned dict.  The deform preamble
(``:79-140``) supports the reference's live additive mode
(``xyz + dx``, ``exp(s + ds)``, ``normalize(q + dq)``, ``features + dSH``) and
the SE(3) mode the north star asks for (twist -> fused HIP exp-map on means
and rotations, ``gsd_amd.deform``).  The deformation network that produces
offsets/twists is outside the hot path: any callable
``offset_model(pts, time, iteration)`` can be plugged in.
"""
from __future__ import annotations

import math
import os
from types import SimpleNamespace

import torch
import torch.nn.functional as F

from .activate import activate_split_sh
from .deform import se3_deform
from .rasterizer import (GaussianRasterizationSettings, GaussianRasterizer, rasterize_gaussians_raw,
                         rasterize_gaussians_split_sh)
from .sh import eval_sh


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


def build_rotation(r):
    """utils/general_utils.py:78-99 (device taken from the input)."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device, dtype=r.dtype)
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - r * z)
    R[:, 0, 2] = 2 * (x * z + r * y)
    R[:, 1, 0] = 2 * (x * y + r * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - r * x)
    R[:, 2, 0] = 2 * (x * z - r * y)
    R[:, 2, 1] = 2 * (y * z + r * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def build_scaling_rotation(s, r):
    """utils/general_utils.py:101-110."""
    L = torch.zeros((s.shape[0], 3, 3), dtype=s.dtype, device=s.device)
    R = build_rotation(r)
    L[:, 0, 0], L[:, 1, 1], L[:, 2, 2] = s[:, 0], s[:, 1], s[:, 2]
    return R @ L


def strip_symmetric(L):
    """utils/general_utils.py:64-76 (upper triangle of the symmetric matrix)."""
    return torch.stack([L[:, 0, 0], L[:, 0, 1], L[:, 0, 2], L[:, 1, 1], L[:, 1, 2], L[:, 2, 2]], dim=1)


def build_covariance_from_scaling_rotation(scaling, scaling_modifier, rotation):
    """scene/gaussian_model.py:634-638."""
    L = build_scaling_rotation(scaling_modifier * scaling, rotation)
    return strip_symmetric(L @ L.transpose(1, 2))


class ZeroOffsets:
    """Deformation producer equivalent to the reference's pre-3000-iteration zeros
    (scene/gaussian_model.py:305-313) -- (dx, dscale, drot, dSH).  Returns None for
    each offset ("zero"), which the fused preamble skips instead of adding zeros."""

    def __call__(self, pts, time, iteration):
        return None, None, None, None


def _zeros_if_none(t, P, w, like):
    return like.new_zeros(P, w) if t is None else t


class DeformableGaussians:
    """The subset of scene/gaussian_model.py:GaussianModel that render() reads
    (:632-801): raw parameters, activations, get_xyz_all, get_features,
    get_covariance.  ``deform`` = "additive" (live reference path) or "se3"."""

    def __init__(self, params, sh_degree=3, deform="additive", offset_model=None, twist_model=None,
                 requires_grad=True):
        p = params
        mk = (lambda t: torch.nn.Parameter(t.contiguous(), requires_grad=requires_grad))
        self._xyz = mk(p.xyz)
        self._scaling = mk(p.scaling)
        self._rotation = mk(p.rotation)
        self._opacity = mk(p.opacity)
        self._features_dc = mk(p.features_dc)
        self._features_rest = mk(p.features_rest)
        self._twist = None if p.twist is None else mk(p.twist)
        self.max_sh_degree = sh_degree
        self.active_sh_degree = sh_degree
        self.deform = deform
        self.offset_model = offset_model or ZeroOffsets()
        self.twist_model = twist_model
        self.scaling_activation = torch.exp
        self.scaling_inverse_activation = torch.log
        self.opacity_activation = torch.sigmoid
        self.inverse_opacity_activation = inverse_sigmoid
        self.rotation_activation = F.normalize
        self.covariance_activation = build_covariance_from_scaling_rotation

    def parameters(self):
        ps = [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]
        if self._twist is not None:
            ps.append(self._twist)
        return ps

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation_ori(self):
        return self.rotation_activation(self._rotation)

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_opacity(self):
        return self.opacity_activation(self._opacity)

    def get_covariance(self, scaling_modifier=1):
        return self.covariance_activation(self.get_scaling, scaling_modifier, self._rotation)

    def get_twist(self, pts, time, iteration):
        if self.twist_model is not None:
            return self.twist_model(pts, time, iteration)
        return self._twist

    def get_xyz_all(self, pts, time, iteration):
        """scene/gaussian_model.py:761-763 -> (means3D, means3D_ori, offset, scale_off, rot_off, mlp_shs)."""
        dx, ds, dq, dsh = self.offset_model(pts, time, iteration)
        P = self._xyz.shape[0]
        dx, ds = _zeros_if_none(dx, P, 3, self._xyz), _zeros_if_none(ds, P, 3, self._xyz)
        dq, dsh = _zeros_if_none(dq, P, 4, self._xyz), _zeros_if_none(dsh, P, 48, self._xyz)
        if self.deform == "se3":
            twist = self.get_twist(pts, time, iteration)
            means, _ = se3_deform(twist, self._xyz + dx)
            return means, self._xyz, means - self._xyz, ds, dq, dsh
        return self._xyz + dx, self._xyz, dx, ds, dq, dsh


def se3_rot_or(pc, rot_offset, se3_rotations):
    """Rotations fed to the rasterizer: normalize(q + dq) (additive, :122) or its SE(3)-moved version."""
    if se3_rotations is not None:
        return se3_rotations
    return pc.rotation_activation(pc._rotation + rot_offset)


_ZEROS = {}


def _zeros(P, w, like):
    """A cached all-zero (P, w) float32 buffer on like's device, never written by this package."""
    key = (like.device, P, w)
    z = _ZEROS.get(key)
    if z is None:
        if len(_ZEROS) > 16:
            _ZEROS.clear()
        z = _ZEROS[key] = torch.zeros(P, w, dtype=torch.float32, device=like.device)
    return z


class RenderPackage(dict):
    """render()'s returned dict; "visibility_filter" (radii > 0) -- and, on the raw-parameter path, the
    activated "rotations" / "opacities" (torch ops, differentiable) -- are computed the first time they are
    read."""

    lazy = {}

    def __missing__(self, key):
        if key == "visibility_filter":
            v = self["radii"] > 0
        elif key in self.lazy:
            v = self.lazy[key]()
        else:
            raise KeyError(key)
        self[key] = v
        return v

    def __contains__(self, key):
        return key == "visibility_filter" or key in self.lazy or dict.__contains__(self, key)


class _Time:
    """The (P, 1) time tensor of gaussian_renderer/__init__.py:87, built only if a deformation model reads it."""

    def __init__(self, P, t, dev):
        self.P, self.t, self.dev, self.v = P, t, dev, None

    def get(self):
        if self.v is None:
            self.v = torch.full((self.P, 1), self.t, device=self.dev)
        return self.v


def _time_for(model, tm):
    return None if model is None or isinstance(model, ZeroOffsets) else tm.get()


def render(viewpoint_camera, pc, pipe, bg_color, iteration=0, scaling_modifier=1.0, override_color=None,
           save_ply=False, control_time=None):
    """gaussian_renderer/__init__.py:20-195.  save_ply=True also writes the frame's point cloud the way the reference
    does (:165-167): test_ply/point_cloud_{int(time * 1000)}.ply under the working directory, with the deformed
    means and rotations and the activated opacities the rasterizer was given (io.save_ply_t)."""
    out = _render(viewpoint_camera, pc, pipe, bg_color, iteration, scaling_modifier, override_color, control_time)
    if save_ply:
        from .io import save_ply_t
        t_id = str(int(viewpoint_camera.time * 1000))
        save_ply_t(os.path.join("test_ply", f"point_cloud_{t_id}.ply"), pc, xyz=out["means3D"],
                   opacities=out["opacities"], rotation=out["rotations"])
    return out


def _render(viewpoint_camera, pc, pipe, bg_color, iteration, scaling_modifier, override_color, control_time):
    dev = pc.get_xyz.device
    # the reference's zeros_like(xyz, requires_grad=True) + 0 with retain_grad(): a zero tensor whose .grad
    # receives dL/d means2D.  The rasterizer never reads its values, so it is a fresh leaf on a cached zero
    # buffer (no fill, no add, and autograd stores the gradient without the retain_grad copy).
    screenspace_points = _zeros(pc.get_xyz.shape[0], 3, pc.get_xyz).detach().requires_grad_(True)
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False,
        debug=getattr(pipe, "debug", False))
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    means3D = pc.get_xyz
    t = control_time if control_time is not None else viewpoint_camera.time
    tm = _Time(means3D.size(0), t, means3D.device)
    means2D = screenspace_points
    python_modes = (getattr(pipe, "compute_cov3D_python", False) or getattr(pipe, "convert_SHs_python", False)
                    or override_color is not None)
    if not python_modes and hasattr(pc, "_features_rest") and getattr(pc, "fused_preamble", True):
        # fused preamble: offsets + activations in one HIP pass (gsd_amd.activate); the SH are not
        # concatenated -- the rasterizer reads features_dc / features_rest / the SH offset in place
        P = means3D.size(0)
        dx, scale_offset, rot_offset, mlp_shs = pc.offset_model(means3D, _time_for(pc.offset_model, tm), iteration)
        if (dx is None and scale_offset is None and rot_offset is None and mlp_shs is None
                and getattr(pc, "deform", "additive") != "se3"):
            # no offsets: the raw parameters go straight to the rasterizer, which activates them itself
            # (gsd_activation) -- no preamble kernels.  The activated tensors of the returned dict are built
            # by torch only if read (RenderPackage), so they still carry gradients.
            rendered_image, radii = rasterize_gaussians_raw(pc._xyz, means2D, pc._features_dc, pc._features_rest,
                                                            pc._scaling, pc._rotation, pc._opacity, raster_settings,
                                                            sh_views=True)
            pkg = RenderPackage(render=rendered_image, viewspace_points=screenspace_points, radii=radii,
                                means3D=pc._xyz, means3D_ori=pc._xyz,
                                means3D_offset=_zeros(1, 3, pc._xyz).expand(P, 3),
                                rot_offset=_zeros(1, 4, pc._xyz).expand(P, 4))
            pkg.lazy = {"rotations": lambda: pc.rotation_activation(pc._rotation),
                        "opacities": lambda: pc.opacity_activation(pc._opacity)}
            return pkg
        dsh = None if mlp_shs is None else mlp_shs.reshape(P, -1, 3)
        means3D, scales, rotations, opacity = activate_split_sh(pc._xyz, pc._scaling, pc._rotation, pc._opacity, dx,
                                                                scale_offset, rot_offset)
        if getattr(pc, "deform", "additive") == "se3":
            # one fused kernel moves means AND rotations by the same rigid motion
            means3D, rotations = se3_deform(pc.get_twist(pc.get_xyz, _time_for(pc.twist_model, tm), iteration),
                                            means3D, rotations)
        means3D_ori = pc._xyz
        moved = dx is not None or getattr(pc, "deform", "additive") == "se3"
        # zero offsets are read-only expanded views of a cached zero row (in-place writes raise)
        means3D_offset = means3D - means3D_ori if moved else _zeros(1, 3, means3D).expand(P, 3)
        rot_offset = rot_offset if rot_offset is not None else _zeros(1, 4, means3D).expand(P, 4)
        # undeformed means are the same on every data-parallel rank: the SH gradient can then be exchanged as
        # per-view dL/dRGB rows (gsd_amd.rasterizer.rasterize_gaussians_split_sh)
        rendered_image, radii = rasterize_gaussians_split_sh(means3D, means2D, pc._features_dc, pc._features_rest,
                                                             dsh, opacity, scales, rotations, raster_settings,
                                                             sh_views=not moved)
        return RenderPackage(render=rendered_image, viewspace_points=screenspace_points, radii=radii,
                             means3D=means3D, means3D_ori=means3D_ori, rotations=rotations,
                             means3D_offset=means3D_offset, opacities=opacity, rot_offset=rot_offset)
    # reference-literal path (Python covariance / SH modes, override colours)
    se3_rot = getattr(pc, "deform", "additive") == "se3" and not getattr(pipe, "compute_cov3D_python", False)
    if se3_rot:
        dx, scale_offset, rot_offset, mlp_shs = pc.offset_model(means3D, tm.get(), iteration)
        P = means3D.size(0)
        dx, scale_offset = _zeros_if_none(dx, P, 3, pc._xyz), _zeros_if_none(scale_offset, P, 3, pc._xyz)
        rot_offset, mlp_shs = _zeros_if_none(rot_offset, P, 4, pc._xyz), _zeros_if_none(mlp_shs, P, 48, pc._xyz)
        twist = pc.get_twist(means3D, tm.get(), iteration)
        means3D_ori = pc._xyz
        means3D, se3_rotations = se3_deform(twist, pc._xyz + dx, pc.rotation_activation(pc._rotation + rot_offset))
        means3D_offset = means3D - means3D_ori
    else:
        means3D, means3D_ori, means3D_offset, scale_offset, rot_offset, mlp_shs = pc.get_xyz_all(means3D, tm.get(),
                                                                                                 iteration)
    opacity = pc.get_opacity
    scales = rotations = cov3D_precomp = None
    if getattr(pipe, "compute_cov3D_python", False):
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.scaling_activation(pc._scaling + scale_offset)
        rotations = se3_rot_or(pc, rot_offset, se3_rotations if se3_rot else None)
    shs = colors_precomp = None
    if override_color is None:
        if getattr(pipe, "convert_SHs_python", False):
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = pc.get_xyz - viewpoint_camera.camera_center.repeat(pc.get_features.shape[0], 1)
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            sh2rgb = eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized)
            colors_precomp = torch.clamp_min(sh2rgb + 0.5, 0.0)
        else:
            shs = pc.get_features + mlp_shs.reshape(-1, 16, 3)
    else:
        colors_precomp = override_color
    rendered_image, radii = rasterizer(means3D=means3D, means2D=means2D, shs=shs, colors_precomp=colors_precomp,
                                       opacities=opacity, scales=scales, rotations=rotations,
                                       cov3D_precomp=cov3D_precomp)
    return {"render": rendered_image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii, "means3D": means3D, "means3D_ori": means3D_ori, "rotations": rotations,
            "means3D_offset": means3D_offset, "opacities": opacity, "rot_offset": rot_offset}


def default_pipe(**kw):
    """PipelineParams (arguments/__init__.py:64-69)."""
    d = dict(convert_SHs_python=False, compute_cov3D_python=False, debug=False)
    d.update(kw)
    return SimpleNamespace(**d)
