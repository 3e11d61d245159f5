"""Fused deform/activation preamble of render() as a torch autograd op.

Forward (gaussian_renderer/__init__.py:79-140, gaussian_model.py:761-797):
    means = xyz + dxyz, scales = exp(scaling + dscale), rotations = normalize(rotation + drot),
    opacities = sigmoid(opacity), shs = cat(f_dc, f_rest) + dsh
in two HIP kernels (gsd_activate_forward) instead of ~10 torch kernels, and
the backward in two more instead of ~12.  When a parameter already has a
``.grad`` buffer (e.g. the FlatGrads slab), its gradient is added in place by
the kernel (no separate AccumulateGrad kernel); otherwise it is returned to
autograd as usual.  Offsets may be None (the reference's zero offsets before
iteration 3000, scene/gaussian_model.py:305-313).
"""
from __future__ import annotations

import torch

from . import _C


def _sinks(params):
    """Parameters registered as in-place gradient owners (FlatGrads sets _gsd_inplace_grad) get their .grad
    updated by the kernels; anything else (e.g. torch.autograd.grad calls) gets returned grads.
    -> (sinks or None, accumulate): accumulate False means the views were stale and are stored into."""
    sinks = [p.grad if (getattr(p, "_gsd_inplace_grad", False) and p.grad is not None
                        and p.grad.dtype == torch.float32
                        and (p.grad.is_contiguous() or p.grad.stride() == p.stride())) else None for p in params]
    if not all(s is not None for s in sinks):
        return None, True
    flats = {id(getattr(p, "_gsd_flat", None)): getattr(p, "_gsd_flat", None) for p in params}
    if len(flats) == 1 and None not in flats.values():
        return sinks, next(iter(flats.values())).claim(params)
    return sinks, True


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xyz, scaling, rotation, opacity, f_dc, f_rest, dxyz, dscale, drot, dsh):
        outs = _C.activate_forward(xyz, scaling, rotation, opacity, f_dc, f_rest, dxyz, dscale, drot, dsh)
        ctx.params = (xyz, scaling, rotation, opacity, f_dc, f_rest)
        ctx.save_for_backward(scaling, rotation, opacity, *(t if t is not None else torch.empty(0)
                                                            for t in (dscale, drot)))
        ctx.has_off = tuple(t is not None for t in (dxyz, dscale, drot, dsh))
        ctx.rest_shape = f_rest.shape
        return outs

    @staticmethod
    def backward(ctx, g_means, g_scales, g_rot, g_opac, g_shs):
        scaling, rotation, opacity, dscale, drot = ctx.saved_tensors
        dscale = dscale if ctx.has_off[1] else None
        drot = drot if ctx.has_off[2] else None
        sinks, acc = _sinks(ctx.params)
        grads = _C.activate_backward(scaling, rotation, opacity, dscale, drot, g_means, g_scales, g_rot, g_opac, g_shs,
                                     sinks, ctx.has_off, ctx.rest_shape, accumulate=acc)
        g_params, g_offsets = grads
        if sinks is not None:
            g_params = (None,) * 6
        g_offsets = tuple(g if need else None for g, need in zip(g_offsets, ctx.has_off))
        return (*g_params, *g_offsets)


class _ActivateSplitSH(torch.autograd.Function):
    """The preamble without the SH concat: the SH stay split (features_dc / features_rest / offset) and
    are read in place by the rasterizer (gsd_amd.rasterizer.rasterize_gaussians_split_sh)."""

    @staticmethod
    def forward(ctx, xyz, scaling, rotation, opacity, dxyz, dscale, drot):
        means, scales, rots, opac, _ = _C.activate_forward(xyz, scaling, rotation, opacity, None, None, dxyz, dscale,
                                                           drot, None)
        ctx.params = (xyz, scaling, rotation, opacity)
        ctx.save_for_backward(scaling, rotation, opacity, *(t if t is not None else torch.empty(0)
                                                            for t in (dscale, drot)))
        ctx.has_off = tuple(t is not None for t in (dxyz, dscale, drot)) + (False,)
        return means, scales, rots, opac

    @staticmethod
    def backward(ctx, g_means, g_scales, g_rot, g_opac):
        scaling, rotation, opacity, dscale, drot = ctx.saved_tensors
        dscale = dscale if ctx.has_off[1] else None
        drot = drot if ctx.has_off[2] else None
        sinks, acc = _sinks(ctx.params)
        (g_xyz, g_scaling, g_rotation, g_opacity, _, _), g_offsets = _C.activate_backward(
            scaling, rotation, opacity, dscale, drot, g_means, g_scales, g_rot, g_opac, None, sinks, ctx.has_off,
            None, accumulate=acc)
        g_params = (None,) * 4 if sinks is not None else (g_xyz, g_scaling, g_rotation, g_opacity)
        g_offsets = tuple(g if need else None for g, need in zip(g_offsets[:3], ctx.has_off[:3]))
        return (*g_params, *g_offsets)


def activate(xyz, scaling, rotation, opacity, f_dc, f_rest, dxyz=None, dscale=None, drot=None, dsh=None):
    """-> (means3D, scales, rotations, opacities, shs (P,1+R,3))."""
    return _Activate.apply(xyz, scaling, rotation, opacity, f_dc, f_rest, dxyz, dscale, drot, dsh)


def activate_split_sh(xyz, scaling, rotation, opacity, dxyz=None, dscale=None, drot=None):
    """-> (means3D, scales, rotations, opacities); the SH are not touched (see _ActivateSplitSH)."""
    return _ActivateSplitSH.apply(xyz, scaling, rotation, opacity, dxyz, dscale, drot)
