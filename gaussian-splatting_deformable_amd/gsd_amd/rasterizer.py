"""Drop-in rasterizer API (L1): mirrors
``submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py``.

``GaussianRasterizationSettings`` (12 fields, same order, :157-169),
``GaussianRasterizer`` (:171-220, same validation messages), the functional
``rasterize_gaussians`` (:21-42) and the autograd Function
``_RasterizeGaussians`` (:44-155, same gradient-tuple order) -- backed by the
HIP kernels through ``gsd_amd._C``.
"""
from __future__ import annotations

import os
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C, _native, parallel
from .optim import FusedAdam


def cpu_deep_copy_tuple(input_tuple):
    copied = [item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple]
    return tuple(copied)


def _post_layout_checks(*tensors):
    """Post the data-parallel layout check (parallel.FlatGrads.post_layout_check) of every gradient slab among a
    forward's inputs: the check then describes the layout this step's collectives will use and its host-side
    exchange overlaps the forward.  No-op without a data-parallel group."""
    seen = set()
    for t in tensors:
        f = getattr(t, "_gsd_flat", None)
        if f is not None and id(f) not in seen:
            seen.add(id(f))
            f.post_layout_check()


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    _post_layout_checks(means3D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp)
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        args = (raster_settings.bg, means3D, colors_precomp, opacities, scales, rotations,
                raster_settings.scale_modifier, cov3Ds_precomp, raster_settings.viewmatrix,
                raster_settings.projmatrix, raster_settings.tanfovx, raster_settings.tanfovy,
                raster_settings.image_height, raster_settings.image_width, sh, raster_settings.sh_degree,
                raster_settings.campos, raster_settings.prefiltered, raster_settings.debug)
        if raster_settings.debug:
            cpu_args = cpu_deep_copy_tuple(args)  # copy before they can be corrupted (:83-90)
            try:
                num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _C.rasterize_gaussians(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _C.rasterize_gaussians(*args)
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _):
        num_rendered = ctx.num_rendered
        rs = ctx.raster_settings
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer, imgBuffer = \
            ctx.saved_tensors
        args = (rs.bg, means3D, radii, colors_precomp, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, sh, rs.sh_degree, rs.campos,
                geomBuffer, num_rendered, binningBuffer, imgBuffer, rs.debug)
        if rs.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                grads_raw = _C.rasterize_gaussians_backward(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            grads_raw = _C.rasterize_gaussians_backward(*args)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations) = grads_raw
        # (:143-153) order; gradients for absent (empty placeholder) inputs are dropped
        grads = (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                 grad_rotations, grad_cov3Ds_precomp, None)
        inputs = (means3D, None, sh, colors_precomp, None, scales, rotations, cov3Ds_precomp)
        return tuple(None if (i < len(inputs) and inputs[i] is not None and inputs[i].numel() == 0) else g
                     for i, g in enumerate(grads))


def rasterize_gaussians_split_sh(means3D, means2D, f_dc, f_rest, sh_offset, opacities, scales, rotations,
                                 raster_settings, sh_views=False):
    """The fused render() path's rasterizer call (no reference counterpart: the reference builds
    shs = cat(f_dc, f_rest) + sh_offset in torch first, gaussian_renderer/__init__.py:129-134).  The SH
    pieces are read in place, and their gradients are written by the rasterizer backward -- added
    straight into ``.grad`` for parameters registered with FlatGrads.  -> (color, radii).

    ``sh_views``: the caller guarantees means3D is the same on every data-parallel rank (no per-view
    deformation).  Then, with more than one rank, the backward exchanges each view's masked dL/dRGB (12 B per
    Gaussian, one all_gather) and every rank sums the SH gradient of all views itself (gsd_sh_grad_views)
    instead of all-reducing the 192-B SH gradient (parallel.FlatGrads leaves it out of its all-reduce)."""
    _post_layout_checks(means3D, f_dc, f_rest, sh_offset, opacities, scales, rotations)
    return _RasterizeSplitSH.apply(means3D, means2D, f_dc, f_rest, sh_offset, opacities, scales, rotations,
                                   raster_settings, sh_views)


class _RasterizeSplitSH(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, f_dc, f_rest, sh_offset, opacities, scales, rotations, raster_settings,
                sh_views=False):
        rs = raster_settings
        ctx.sh_views = bool(sh_views)
        split = _C.ShSplit(f_dc, f_rest, sh_offset)
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _C.rasterize_gaussians(
            rs.bg, means3D, None, opacities, scales, rotations, rs.scale_modifier, None, rs.viewmatrix, rs.projmatrix,
            rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, None, rs.sh_degree, rs.campos, rs.prefiltered,
            rs.debug, sh_split=split, grad_scratch=_grad_scratch(ctx, means3D))
        _save(ctx, rs, num_rendered, radii, means3D, scales, rotations, f_dc, f_rest, sh_offset, geomBuffer,
              binningBuffer, imgBuffer)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _):
        if grad_out_color is None:
            return (None,) * 10
        g_m2d, d_dc, d_rest, d_off, rest = _split_sh_backward(ctx, grad_out_color)
        g_op, g_m3d, g_sc, g_rot = rest
        return g_m3d, g_m2d, d_dc, d_rest, d_off, g_op, g_sc, g_rot, None, None


def rasterize_gaussians_raw(xyz, means2D, f_dc, f_rest, scaling, rotation, opacity, raster_settings,
                            sh_views=False):
    """The fused render() path without offsets: the raw parameters (_xyz, _features_dc, _features_rest,
    _scaling, _rotation, _opacity) go straight to the rasterizer, which applies exp / normalize / sigmoid itself
    (gsd_activation) and whose backward writes their gradients -- into ``.grad`` for FlatGrads parameters.
    Replaces the preamble kernels of gsd_amd.activate (gaussian_renderer/__init__.py:79-140). -> (color, radii)"""
    _post_layout_checks(xyz, f_dc, f_rest, scaling, rotation, opacity)
    return _RasterizeRaw.apply(xyz, means2D, f_dc, f_rest, scaling, rotation, opacity, raster_settings, sh_views)


class _RasterizeRaw(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xyz, means2D, f_dc, f_rest, scaling, rotation, opacity, raster_settings, sh_views=False):
        rs = raster_settings
        ctx.sh_views = bool(sh_views)
        split = _C.ShSplit(f_dc, f_rest, None)
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _C.rasterize_gaussians(
            rs.bg, xyz, None, opacity, scaling, rotation, rs.scale_modifier, None, rs.viewmatrix, rs.projmatrix,
            rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, None, rs.sh_degree, rs.campos, rs.prefiltered,
            rs.debug, sh_split=split, activation=_native.Activation(), grad_scratch=_grad_scratch(ctx, xyz))
        _save(ctx, rs, num_rendered, radii, xyz, scaling, rotation, f_dc, f_rest, None, geomBuffer, binningBuffer,
              imgBuffer, opacity=opacity)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _):
        from .activate import _sinks
        if grad_out_color is None:
            return (None,) * 9
        saved = ctx.saved_tensors
        xyz, scaling, rotation, opacity = saved[0], saved[1], saved[2], saved[10]
        raw = (xyz, scaling, rotation, opacity)
        sinks, acc = _sinks(raw)
        epi = None
        if sinks is None:
            sinks, acc = [torch.empty_like(t) for t in raw], False
            ret = sinks
        else:
            ret = [None] * 4
            owner = FusedAdam.fused_owner(raw) if not acc else None
            if owner is not None:   # the raw parameters' Adam step runs inside this backward
                epi = owner.fuse(dict(zip(("xyz", "scaling", "rotation", "opacity"), raw)))
        act = _native.Activation(d_xyz=sinks[0].data_ptr(), d_scaling=sinks[1].data_ptr(),
                                 d_rotation=sinks[2].data_ptr(), d_opacity=sinks[3].data_ptr(),
                                 accumulate=int(bool(acc)))
        g_m2d, d_dc, d_rest, _, _ = _split_sh_backward(ctx, grad_out_color, activation=act, raw_opacity=opacity,
                                                       epi=epi, raw=raw)
        return ret[0], g_m2d, d_dc, d_rest, ret[1], ret[2], ret[3], None, None


FWD_ZERO_SCRATCH = os.environ.get("GSD_FWD_ZERO_SCRATCH", "1") != "0"   # 0: the backward zeroes its own scratch


def _grad_scratch(ctx, means3D):
    """The backward's gradient-record scratch, allocated by the forward when a gradient will be asked for: the
    forward's compositing kernel zeroes it (ABI 14 grad_scratch), so the backward needs no memset launch."""
    ctx.grad_scratch = None
    if FWD_ZERO_SCRATCH and any(ctx.needs_input_grad) and means3D.is_cuda and means3D.size(0) > 0:
        ctx.grad_scratch = torch.empty(_C.backward_scratch_bytes(means3D.size(0)), dtype=torch.uint8,
                                       device=means3D.device)
    return ctx.grad_scratch


def _take_scratch(ctx):
    """The zeroed scratch for the first backward of this forward; None afterwards (a second backward through the
    same graph zeroes a fresh one itself)."""
    s = getattr(ctx, "grad_scratch", None)
    ctx.grad_scratch = None
    return s


def _save(ctx, rs, num_rendered, radii, means3D, scales, rotations, f_dc, f_rest, sh_offset, geomBuffer,
          binningBuffer, imgBuffer, opacity=None):
    ctx.raster_settings = rs
    ctx.num_rendered = num_rendered
    ctx.has_offset = sh_offset is not None
    ctx.mark_non_differentiable(radii)
    ctx.set_materialize_grads(False)   # no zero-filled int32 gradient for radii
    ctx.params = (f_dc, f_rest)
    ctx.save_for_backward(means3D, scales, rotations, radii, f_dc, f_rest,
                          sh_offset if sh_offset is not None else torch.empty(0), geomBuffer, binningBuffer,
                          imgBuffer, opacity if opacity is not None else torch.empty(0))


def _split_sh_backward(ctx, grad_out_color, activation=None, raw_opacity=None, epi=None, raw=()):
    """Shared backward of the split-SH rasterizer paths -> (dL/dmeans2D, d_dc, d_rest, d_offset,
    (dL/dopacity, dL/dmeans3D, dL/dscales, dL/drotations)); the SH gradients are None when they went into
    the parameters' .grad in place, the last four when ``activation`` took them.  ``epi``: the Adam epilogue
    the caller set up for ``raw`` (FusedAdam.step_in_backward); the SH pieces join it when they can."""
    from .activate import _sinks
    rs = ctx.raster_settings
    means3D, scales, rotations, radii, f_dc, f_rest, sh_offset, geomBuffer, binningBuffer, imgBuffer, opac = \
        ctx.saved_tensors
    sinks, acc = _sinks(ctx.params)
    offset = sh_offset if ctx.has_offset else None
    world = parallel.data_parallel_world()
    if ctx.sh_views and parallel.dp_active() and sinks is not None and offset is None and parallel.SH_VIEWS:
        g_m2d, g_op, g_m3d, g_sc, g_rot = _backward_sh_views(ctx, rs, grad_out_color, means3D, scales, rotations,
                                                             radii, f_dc, f_rest, geomBuffer, binningBuffer,
                                                             imgBuffer, sinks, acc, world, activation, raw_opacity,
                                                             raw=raw)
        return g_m2d, None, None, None, (g_op, g_m3d, g_sc, g_rot)
    if sinks is not None:
        d_dc, d_rest = sinks
        owner = FusedAdam.fused_owner(ctx.params) if not acc else None
        if owner is not None and f_dc.is_contiguous() and f_rest.is_contiguous():
            epi = owner.fuse({"dc": f_dc, "rest": f_rest}, epi)
    else:
        d_dc, d_rest = torch.zeros_like(f_dc), torch.zeros_like(f_rest)
    d_off = None
    if ctx.has_offset:
        d_off = torch.zeros(f_dc.size(0), 1 + f_rest.size(1), 3, device=f_dc.device)
    split = _C.ShSplit(f_dc, f_rest, offset, d_dc, d_rest, d_off, accumulate=sinks is not None and acc)
    g_m2d, _, g_op, g_m3d, _, _, g_sc, g_rot = _C.rasterize_gaussians_backward(
        rs.bg, means3D, radii, None, scales, rotations, rs.scale_modifier, None, rs.viewmatrix, rs.projmatrix,
        rs.tanfovx, rs.tanfovy, grad_out_color, None, rs.sh_degree, rs.campos, geomBuffer, ctx.num_rendered,
        binningBuffer, imgBuffer, rs.debug, sh_split=split, activation=activation, raw_opacity=raw_opacity,
        adam=epi, scratch=_take_scratch(ctx))
    if epi is not None:   # parameters the kernel updated in place: autograd's saved-tensor checks must see it
        for p in (*raw, f_dc, f_rest):
            if id(p) in p._gsd_flat.fused:
                torch.autograd.graph.increment_version(p)
    if sinks is not None:
        d_dc = d_rest = None
    return g_m2d, d_dc, d_rest, d_off, (g_op, g_m3d, g_sc, g_rot)


_VIEWS_ROW = {}


def _views_row(P, dev):
    """This rank's exchange row [d_rgb (P*3) | campos (3) | 0] (rasterizer._backward_sh_views), kept per (P, device):
    the compute stream waits for each step's all-gather before it writes the row again."""
    key = (P, str(dev))
    row = _VIEWS_ROW.get(key)
    if row is None:
        _VIEWS_ROW.clear()
        row = _VIEWS_ROW[key] = torch.zeros(3 * P + 4, dtype=torch.float32, device=dev)
    return row


_VIEWS_MEANS = {}


def _views_means(P, dev):
    """The views' summed view-direction term of the means (gsd_sh_grad_views_ex d_means), kept per (P, device):
    the step's Adam pass (or FlatGrads.allreduce) consumes it before the next backward writes it."""
    key = (P, str(dev))
    t = _VIEWS_MEANS.get(key)
    if t is None:
        _VIEWS_MEANS.clear()
        t = _VIEWS_MEANS[key] = torch.empty(P, 3, dtype=torch.float32, device=dev)
    return t


def _backward_sh_views(ctx, rs, grad_out_color, means3D, scales, rotations, radii, f_dc, f_rest, geomBuffer,
                       binningBuffer, imgBuffer, sinks, acc, world, activation=None, raw_opacity=None, raw=()):
    """Data-parallel backward of the split-SH rasterizer with the SH gradient exchanged per view: this rank's
    row [masked dL/dRGB (P*3) | campos (3) | pad] is all-gathered and every rank runs gsd_sh_grad_views over
    all rows into its SH sinks, which FlatGrads then leaves out of the gradient all-reduce.  Inside
    FusedAdam.step_in_backward the raw parameters' gradients (``raw``, stored by this backward) are final per
    rank here: their all-reduce goes out right behind the all-gather (FusedAdam.reduce_early) and runs on the
    links while the device assembles and steps the SH gradient."""
    import torch.distributed as dist
    P, dev = int(f_dc.size(0)), f_dc.device
    stride = 3 * P + 4
    row = _views_row(P, dev)   # its pad float was zeroed once; the previous step's all-gather is done with it
    row[3 * P:3 * P + 3].copy_(rs.campos.reshape(-1))
    # defer_view_dir: the raw path, whose xyz gradient is a FlatGrads view -- the backward then reads no SH
    # coefficient (no SH half at all) and gsd_sh_grad_views_ex adds every view's view-direction term of the means
    # after the all-reduce (FlatGrads.add_after_reduce); elsewhere (an autograd consumer of dL/dmeans3D) this
    # rank's own term stays in its backward
    xyz = raw[0] if raw else None
    flat = getattr(xyz, "_gsd_flat", None)
    defer = (activation is not None and flat is not None and not acc and xyz.grad is not None
             and activation.d_xyz == xyz.grad.data_ptr() and f_dc.is_contiguous() and f_rest.is_contiguous()
             and int(f_rest.size(1)) == 15)
    split = _C.ShSplit(f_dc, f_rest, None, None, None, None, accumulate=False, d_rgb=row[:3 * P],
                       defer_view_dir=defer)
    g_m2d, _, g_op, g_m3d, _, _, g_sc, g_rot = _C.rasterize_gaussians_backward(
        rs.bg, means3D, radii, None, scales, rotations, rs.scale_modifier, None, rs.viewmatrix, rs.projmatrix,
        rs.tanfovx, rs.tanfovy, grad_out_color, None, rs.sh_degree, rs.campos, geomBuffer, ctx.num_rendered,
        binningBuffer, imgBuffer, rs.debug, sh_split=split, activation=activation, raw_opacity=raw_opacity,
        scratch=_take_scratch(ctx))
    f_flat = getattr(f_dc, "_gsd_flat", None)
    if f_flat is not None:
        f_flat.verify_layout()   # every rank's P and settings agree before the P-sized all-gather
    views = torch.empty(world, stride, dtype=torch.float32, device=dev)
    gathered = None
    if dist.get_backend() == "nccl":   # RCCL: one all_gather into the (world, stride) buffer
        gathered = dist.all_gather_into_tensor(views, row, async_op=True)
    else:                              # gloo (tests): through host memory
        parts = [torch.empty(stride, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, row.cpu())
        views.copy_(torch.stack(parts))
    if raw and activation is not None and not activation.accumulate:
        owner = FusedAdam.fused_owner(raw)
        if owner is not None:
            owner.reduce_early(raw)    # queued behind the all-gather on RCCL's stream
    if gathered is not None:
        gathered.wait()                # the compute stream waits for the gather only
    epi = None
    owner = FusedAdam.fused_owner(ctx.params) if not acc else None
    if owner is not None and f_dc.is_contiguous() and f_rest.is_contiguous():
        epi = owner.fuse({"dc": f_dc, "rest": f_rest}, summed=True)   # every view's sum: final on every rank
    d_means = _views_means(P, dev) if defer else None
    _C.sh_grad_views(rs.sh_degree, means3D, views, P, 1 + int(f_rest.size(1)), d_dc=sinks[0], d_rest=sinks[1],
                     accumulate=acc, layout=split, adam=epi, sh=(f_dc, f_rest), d_means=d_means)
    if defer:
        flat.add_after_reduce(xyz, d_means)
    if epi is not None:
        for p in (f_dc, f_rest):
            torch.autograd.graph.increment_version(p)
    parallel.mark_reduced(ctx.params)
    return g_m2d, g_op, g_m3d, g_sc, g_rot


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        # frustum (near-plane) test (:176-185)
        with torch.no_grad():
            rs = self.raster_settings
            visible = _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        if shs is None:
            shs = torch.Tensor([])
        if colors_precomp is None:
            colors_precomp = torch.Tensor([])
        if scales is None:
            scales = torch.Tensor([])
        if rotations is None:
            rotations = torch.Tensor([])
        if cov3D_precomp is None:
            cov3D_precomp = torch.Tensor([])
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, rs)
