"""Torch-facing mirror of the reference's pybind module ``_C``.

Same three functions, argument order, return tuples and error messages as
``submodules/diff-gaussian-rasterization/ext.cpp:15-19`` /
``rasterize_points.cu:35-217``; each call unwraps torch tensors into device
pointers and goes through the C-ABI of ``include/gsd_raster.h`` on the
tensors' device and torch's current HIP stream (the reference used the
legacy default stream and the *current* device -- rasterize_points.cu:71).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native

_i64 = ctypes.c_int64

# host-side record of the most recent forward on this process (bench / diagnostics)
last_forward: dict = {}


def _stream(dev: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _absent(t) -> bool:
    """The reference's placeholders are empty tensors (``torch.Tensor([])``) -> nullptr."""
    return t is None or t.numel() == 0


def _dev_f32(t: torch.Tensor, name: str, dev: torch.device) -> torch.Tensor:
    if t.device != dev:
        raise RuntimeError(f"{name} must be on {dev} (got {t.device}); the rasterizer has no CPU path")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


_MATS = {}


def _dev_mat(t: torch.Tensor, name: str, dev: torch.device) -> torch.Tensor:
    """_dev_f32 for the small per-camera tensors (view / projection matrices, camera centre).  The reference's
    Camera stores its matrices transposed (non-contiguous, scene/cameras.py), so the contiguous copy is cached per
    tensor object and version instead of being remade (one copy kernel each) at every call."""
    if t.is_contiguous():
        return _dev_f32(t, name, dev)
    e = _MATS.get(id(t))
    if e is not None and e[0] is t and e[1] == t._version:
        return e[2]
    c = _dev_f32(t, name, dev)
    if len(_MATS) >= 64:
        _MATS.clear()
    _MATS[id(t)] = (t, t._version, c)   # holds t, so its id is not reused while cached
    return c


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


class ShSplit:
    """The split SH operand (gsd_sh_split): features_dc (P,1,3), features_rest (P,R,3) and an optional
    additive offset (P,1+R,3) read in place instead of shs = cat(dc, rest) + offset; for the backward,
    the gradient sinks (any may be None) and whether they are added into (accumulate) or stored."""

    def __init__(self, dc, rest, offset=None, d_dc=None, d_rest=None, d_offset=None, accumulate=False, d_rgb=None,
                 defer_view_dir=False):
        dev = dc.device
        # dc / rest may be strided (P,K,3) views -- e.g. FusedAdam's coefficient-major slabs -- as long as the
        # element e = 3 k + c sits at g * stride(0) + e * stride(2); anything else is copied contiguous
        self.dc, dcs = _sh_operand(dc, "features_dc", dev)
        self.rest, rs = _sh_operand(rest, "features_rest", dev)
        self.offset = None if offset is None else _dev_f32(offset, "sh offset", dev)
        self.sinks = [None if t is None else t for t in (d_dc, d_rest, d_offset)]
        for t, want in zip(self.sinks, (dcs, rs, None)):
            if t is None:
                continue
            if t.dtype != torch.float32 or t.device != dev:
                raise RuntimeError("sh_split gradient sinks must be float32 on the same device")
            if (t.is_contiguous() and want is None) or (want is not None and _sh_strides(t) == want):
                continue
            if not t.is_contiguous() or want is not None:
                raise RuntimeError("sh_split gradient sinks must have their parameter's layout")
        self.M = 1 + int(self.rest.size(1))
        self.d_rgb = d_rgb   # (P*3,) view: the view's masked dL/dRGB instead of the SH gradient (sh_grad_views)
        self.c = _native.ShSplit(dc=_ptr(self.dc).value, rest=_ptr(self.rest).value, offset=_ptr(self.offset).value,
                                 d_dc=_ptr(self.sinks[0]).value, d_rest=_ptr(self.sinks[1]).value,
                                 d_offset=_ptr(self.sinks[2]).value, accumulate=int(bool(accumulate)),
                                 d_rgb=_ptr(d_rgb).value, dc_stride_g=(dcs or (0, 0))[0],
                                 dc_stride_e=(dcs or (0, 0))[1], rest_stride_g=(rs or (0, 0))[0],
                                 rest_stride_e=(rs or (0, 0))[1], defer_view_dir=int(bool(defer_view_dir)))


def _sh_strides(t):
    """(stride_g, stride_e) of a (P,K,3) tensor whose element (g, 3k+c) is at g*stride_g + (3k+c)*stride_e,
    or None when contiguous (the default layout) or not expressible that way."""
    if t.is_contiguous() or t.dim() != 3:
        return None
    sg, sk, sc = t.stride()
    if t.size(1) > 1 and sk != 3 * sc:
        return None
    return (sg, sc)


def _sh_operand(t, name, dev):
    if t.device != dev:
        raise RuntimeError(f"{name} must be on {dev} (got {t.device}); the rasterizer has no CPU path")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    st = _sh_strides(t)
    if st is None and not t.is_contiguous():
        t = t.contiguous()
    return t, st


class _Args:
    """Holds the contiguous device tensors alive for the duration of one native call."""

    def __init__(self, background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                 viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                 prefiltered, debug, sh_split=None, activation=None):
        dev = means3D.device
        if dev.type != "cuda":
            raise RuntimeError("means3D must be a HIP device tensor: this rasterizer has no CPU implementation")
        self.dev = dev
        self.P = int(means3D.size(0))
        self.means3D = _dev_f32(means3D, "means3D", dev)
        self.bg = _dev_f32(background, "bg", dev)
        self.opacity = None if (opacity is None or not self.P) else _dev_f32(opacity, "opacities", dev)
        self.sh = None if _absent(sh) else _dev_f32(sh, "sh", dev)
        self.colors = None if _absent(colors) else _dev_f32(colors, "colors_precomp", dev)
        self.scales = None if _absent(scales) else _dev_f32(scales, "scales", dev)
        self.rotations = None if _absent(rotations) else _dev_f32(rotations, "rotations", dev)
        self.cov3D = None if _absent(cov3D_precomp) else _dev_f32(cov3D_precomp, "cov3D_precomp", dev)
        self.view = _dev_mat(viewmatrix, "viewmatrix", dev)
        self.proj = _dev_mat(projmatrix, "projmatrix", dev)
        self.campos = _dev_mat(campos, "campos", dev)
        self.M = 0 if self.sh is None else int(self.sh.size(1))  # rasterize_points.cu:83-87
        self.sh_split = sh_split
        if sh_split is not None:
            self.M = sh_split.M
        self.H, self.W = int(image_height), int(image_width)
        self.c = _native.RasterArgs(
            P=self.P, D=int(degree), M=self.M, width=self.W, height=self.H,
            scale_modifier=float(scale_modifier), tan_fovx=float(tan_fovx), tan_fovy=float(tan_fovy),
            prefiltered=int(bool(prefiltered)), debug=int(bool(debug)),
            background=_ptr(self.bg).value, means3D=_ptr(self.means3D).value, shs=_ptr(self.sh).value,
            colors_precomp=_ptr(self.colors).value, opacities=_ptr(self.opacity).value,
            scales=_ptr(self.scales).value, rotations=_ptr(self.rotations).value,
            cov3D_precomp=_ptr(self.cov3D).value, viewmatrix=_ptr(self.view).value,
            projmatrix=_ptr(self.proj).value, campos=_ptr(self.campos).value,
            sh_split=None if sh_split is None else ctypes.addressof(sh_split.c),
            activation=None if activation is None else ctypes.addressof(activation), alpha_mode=_ALPHA_MODE[0])
        self.activation = activation


# gsd_raster_args.alpha_mode (ABI 17): "fast" (the default: alpha >= 1/255 decided as power >= t_o, the value from the
# hardware exp) or "reference" (forward.cu:343-345 as written, min(0.99, o * expf(power)) < 1/255: the oracle's
# decisions and final_T to ~2e-6, ~20 % slower compositing).  GSD_ALPHA_MODE=reference selects it at
# import; a backward must run in its forward's mode.
_ALPHA_MODES = {"fast": 0, "reference": 1}
_ALPHA_MODE = [_ALPHA_MODES[os.environ.get("GSD_ALPHA_MODE", "fast")]]


def set_alpha_mode(mode: str) -> None:
    """Select how the compositing kernels evaluate alpha: "fast" or "reference" (see above)."""
    if mode not in _ALPHA_MODES:
        raise ValueError(f"alpha mode must be one of {sorted(_ALPHA_MODES)}, got {mode!r}")
    _ALPHA_MODE[0] = _ALPHA_MODES[mode]


def alpha_mode() -> str:
    return "reference" if _ALPHA_MODE[0] else "fast"


_K_GUESS = {}   # device -> last num_rendered


def backward_scratch_bytes(P):
    """gsd_backward_scratch_bytes: the backward's gradient-record scratch (ABI 14: zeroed by a forward given it)."""
    return int(_native.load().gsd_backward_scratch_bytes(int(P)))


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug, sh_split=None, activation=None, grad_scratch=None):
    """RasterizeGaussiansCUDA (rasterize_points.cu:35-115):
    -> (num_rendered, color (3,H,W), radii (P,) int32, geomBuffer, binningBuffer, imgBuffer).
    ``sh_split`` (a ShSplit, with ``sh`` empty) is this library's extension for the fused render path.
    ``grad_scratch`` (ABI 14): a uint8 device tensor of backward_scratch_bytes(P) that the forward zeroes for one
    rasterize_gaussians_backward(..., scratch=grad_scratch) of this view (no memset in that backward)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    lib = _native.load()
    a = _Args(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
              projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, debug,
              sh_split, activation)
    dev, P, H, W = a.dev, a.P, a.H, a.W
    if grad_scratch is not None:
        if (grad_scratch.device != dev or grad_scratch.dtype != torch.uint8
                or grad_scratch.numel() < backward_scratch_bytes(P)):
            raise RuntimeError("grad_scratch must be a uint8 device tensor of backward_scratch_bytes(P) bytes")
        a.c.grad_scratch = grad_scratch.data_ptr()
    radii = torch.empty(P, dtype=torch.int32, device=dev)   # preprocess writes every entry (forward.cu:174)
    byte = dict(dtype=torch.uint8, device=dev)
    if P == 0:
        empty = torch.empty(0, **byte)
        return 0, torch.zeros(3, H, W, dtype=torch.float32, device=dev), radii, empty, empty.clone(), empty.clone()
    with torch.cuda.device(dev):
        stream = _stream(dev)
        geom = torch.empty(lib.gsd_geom_buffer_bytes(P, W, H), **byte)
        img = torch.empty(lib.gsd_image_buffer_bytes(W, H), **byte)
        color = torch.empty(3, H, W, dtype=torch.float32, device=dev)
        # the binning buffer is sized before num_rendered is known (the last count on this device plus
        # headroom, or 4 instances per Gaussian), so both phases run in one native call and the device idles
        # only for the count's read-back; a short buffer costs one more allocation and call
        guess = max(_K_GUESS.get(dev, 4 * P), 1)
        binning = torch.empty(lib.gsd_binning_buffer_bytes(guess + guess // 4), **byte)
        K = _i64(0)
        rc = lib.gsd_rasterize_forward(ctypes.byref(a.c), _ptr(geom), _ptr(img), _ptr(binning), binning.numel(),
                                       _ptr(radii), _ptr(color), ctypes.byref(K), stream)
        num_rendered = int(K.value)
        if rc == _native.GSD_NEED_BINNING:
            binning = torch.empty(lib.gsd_binning_buffer_bytes(num_rendered), **byte)
            rc = lib.gsd_rasterize_forward_render(ctypes.byref(a.c), _ptr(geom), _ptr(img), _ptr(binning),
                                                  num_rendered, _ptr(radii), _ptr(color), stream)
        _native.check(rc)
        _K_GUESS[dev] = num_rendered
        last_forward.update(P=P, W=W, H=H, num_rendered=num_rendered)
    return num_rendered, color, radii, geom, binning, img


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree,
                                 campos, geomBuffer, R, binningBuffer, imageBuffer, debug, sh_split=None,
                                 activation=None, raw_opacity=None, adam=None, scratch=None):
    """RasterizeGaussiansBackwardCUDA (rasterize_points.cu:117-196):
    -> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations).
    With ``sh_split`` the SH gradients go to its sinks and dL_dsh is None; so is dL_dcov3D when no
    cov3D_precomp was given (the scales/rotations gradients are what such a caller uses).  With
    ``activation`` (a _native.Activation; scales / rotations and ``raw_opacity`` are then the raw parameters)
    the parameter gradients go to its sinks and only dL_dmeans2D (and dL_dcov3D, dL_dsh) are returned.
    ``adam`` (a _native.AdamEpilogue) fuses the Adam step of the SH pieces / raw parameters it names into this
    backward: those are updated in place and their sinks are not written.  ``scratch``: the ``grad_scratch`` the
    forward of this view zeroed (used once), or None (allocated and zeroed here)."""
    lib = _native.load()
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))  # rasterize_points.cu:142-143
    a = _Args(background, means3D, colors, raw_opacity if activation is not None else None, scales, rotations,
              scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, sh, degree, campos,
              False, debug, sh_split, activation)
    if adam is not None:
        a.c.adam = ctypes.addressof(adam)
    dev, P, M = a.dev, a.P, a.M
    split = sh_split is not None
    want_cov = not split or a.cov3D is not None
    # every output is written by the backward for every Gaussian, so one unfilled slab holds them all (the
    # float4-accessed rotation first, 16-B aligned); the library zeroes its own scratch (the gradient records)
    act = activation is not None   # raw parameters: their gradients go to the activation sinks
    widths = [0 if act else 4, 3, 0 if act else 3, 0 if act else 1, 0 if act else 3, 6 if want_cov else 0,
              0 if split else M * 3, 0 if act else 3]
    slab = torch.empty(P * sum(widths), dtype=torch.float32, device=dev)
    views, off = [], 0
    for w in widths:
        views.append(slab[off:off + P * w].view(P, w) if w else None)
        off += P * w
    drot, dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales = views
    if scratch is not None and scratch.numel() >= lib.gsd_backward_scratch_bytes(P) and scratch.device == dev:
        a.c.grad_scratch = scratch.data_ptr()   # zeroed by the forward: the backward skips its memset
    else:
        scratch = torch.empty(lib.gsd_backward_scratch_bytes(P), dtype=torch.uint8, device=dev)
    if dsh is not None:
        dsh = dsh.view(P, M, 3)
    if P != 0:
        dout = _dev_f32(dL_dout_color, "dL_dout_color", dev)
        radii_c = radii.contiguous()
        with torch.cuda.device(dev):
            _native.check(lib.gsd_rasterize_backward(
                ctypes.byref(a.c), _ptr(radii_c), _ptr(geomBuffer), _ptr(binningBuffer), _ptr(imageBuffer), int(R),
                _ptr(dout), _ptr(dmeans2D), _ptr(scratch), _ptr(dopacity), _ptr(dcolors), _ptr(dmeans3D),
                _ptr(dcov3D), _ptr(dsh if M else None), _ptr(dscales), _ptr(drot), _stream(dev)))
    return dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot


def sh_grad_views(D, means3D, views, P, M, d_dc=None, d_rest=None, d_offset=None, accumulate=False, layout=None,
                  adam=None, sh=None, d_means=None):
    """gsd_sh_grad_views(_ex): the SH gradient summed over the views whose rows views (n_views, view_stride) hold
    [masked dL/dRGB (P*3) | campos (3) | pad] -> written into / added to the given sinks (or, for the pieces
    ``adam`` (a _native.AdamEpilogue) names, their Adam step applied in place).  ``d_means`` (P,3): also the
    views' summed view-direction term that a defer_view_dir backward left out of dL/dmeans3D, from the SH
    coefficients ``sh`` = (features_dc, features_rest) the views rendered."""
    lib = _native.load()
    dev = means3D.device
    if views.dim() != 2 or not views.is_contiguous() or views.dtype != torch.float32 or views.device != dev:
        raise RuntimeError("sh_grad_views: views must be a contiguous (n_views, stride) float32 device tensor")
    m = _dev_f32(means3D, "means3D", dev)
    lay = None if layout is None else ctypes.byref(layout.c)
    ad = None if adam is None else ctypes.byref(adam)
    with torch.cuda.device(dev):
        if d_means is None:
            _native.check(lib.gsd_sh_grad_views(int(P), int(D), int(M), int(views.size(0)), _ptr(m), _ptr(views),
                                                int(views.size(1)), _ptr(d_dc), _ptr(d_rest), _ptr(d_offset),
                                                int(bool(accumulate)), lay, ad, _stream(dev)))
            return
        if sh is None or not all(t.is_contiguous() for t in sh) or not d_means.is_contiguous():
            raise RuntimeError("sh_grad_views: d_means needs the contiguous SH pieces sh=(dc, rest)")
        _native.check(lib.gsd_sh_grad_views_ex(int(P), int(D), int(M), int(views.size(0)), _ptr(m), _ptr(views),
                                               int(views.size(1)), _ptr(sh[0]), _ptr(sh[1]), _ptr(d_dc),
                                               _ptr(d_rest), _ptr(d_offset), _ptr(d_means), int(bool(accumulate)),
                                               lay, ad, _stream(dev)))


def mark_visible(means3D, viewmatrix, projmatrix):
    """markVisible (rasterize_points.cu:198-217) -> bool (P,)."""
    lib = _native.load()
    P = int(means3D.size(0))
    dev = means3D.device
    present = torch.zeros(P, dtype=torch.bool, device=dev)
    if P != 0:
        if dev.type != "cuda":
            raise RuntimeError("means3D must be a HIP device tensor: this rasterizer has no CPU implementation")
        m = _dev_f32(means3D, "means3D", dev)
        v = _dev_f32(viewmatrix, "viewmatrix", dev)
        p = _dev_f32(projmatrix, "projmatrix", dev)
        with torch.cuda.device(dev):
            _native.check(lib.gsd_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(dev)))
    return present


def se3_deform_forward(twist, means, rotations=None):
    """Fused per-Gaussian SE(3) deform (gsd_se3_deform_forward) -> (means', rotations' or None)."""
    lib = _native.load()
    dev = means.device
    P = int(means.size(0))
    tw = _dev_f32(twist, "twist", dev)
    m = _dev_f32(means, "means3D", dev)
    q = None if rotations is None else _dev_f32(rotations, "rotations", dev)
    mo = torch.empty_like(m)
    qo = None if q is None else torch.empty_like(q)
    with torch.cuda.device(dev):
        _native.check(lib.gsd_se3_deform_forward(P, _ptr(tw), _ptr(m), _ptr(q), _ptr(mo), _ptr(qo), _stream(dev)))
    return mo, qo


def se3_deform_backward(twist, means, rotations, dL_dmeans_out, dL_drot_out):
    lib = _native.load()
    dev = means.device
    P = int(means.size(0))
    tw = _dev_f32(twist, "twist", dev)
    m = _dev_f32(means, "means3D", dev)
    q = None if rotations is None else _dev_f32(rotations, "rotations", dev)
    gm = _dev_f32(dL_dmeans_out, "dL_dmeans", dev)
    gq = None
    if q is not None:
        gq = torch.zeros_like(q) if dL_drot_out is None else _dev_f32(dL_drot_out, "dL_drot", dev)
    dtw = torch.empty_like(tw)
    dm = torch.empty_like(m)
    dq = None if q is None else torch.empty_like(q)
    with torch.cuda.device(dev):
        _native.check(lib.gsd_se3_deform_backward(P, _ptr(tw), _ptr(m), _ptr(q), _ptr(gm), _ptr(gq), _ptr(dtw),
                                                  _ptr(dm), _ptr(dq), _stream(dev)))
    return dtw, dm, dq


def _opt_f32(t, name, dev):
    return None if t is None else _dev_f32(t, name, dev)


def activate_forward(xyz, scaling, rotation, opacity, f_dc, f_rest, dxyz=None, dscale=None, drot=None, dsh=None):
    """Fused render() preamble (gsd_activate_forward) -> (means3D, scales, rotations, opacities, shs).
    With f_dc = f_rest = None the SH are left split (shs is None; see ShSplit)."""
    lib = _native.load()
    dev = xyz.device
    P = int(xyz.size(0))
    split = f_dc is None
    R = 0 if split else (int(f_rest.size(1)) if f_rest.dim() == 3 else int(f_rest.numel() // max(P * 3, 1)))
    ins = [_opt_f32(t, n, dev) for t, n in ((xyz, "xyz"), (scaling, "scaling"), (rotation, "rotation"),
                                           (opacity, "opacity"), (f_dc, "f_dc"), (f_rest, "f_rest"))]
    offs = [_opt_f32(t, n, dev) for t, n in ((dxyz, "dxyz"), (dscale, "dscale"), (drot, "drot"),
                                            (None if split else dsh, "dsh"))]
    means = torch.empty(P, 3, device=dev)
    scales = torch.empty(P, 3, device=dev)
    rots = torch.empty(P, 4, device=dev)
    opac = torch.empty(P, 1, device=dev)
    shs = None if split else torch.empty(P, 1 + R, 3, device=dev)
    x, s, q, o, fdc, frest = ins
    dx, ds, dq, dsh_ = offs
    with torch.cuda.device(dev):
        _native.check(lib.gsd_activate_forward(P, R, _ptr(x), _ptr(dx), _ptr(s), _ptr(ds), _ptr(q), _ptr(dq), _ptr(o),
                                               _ptr(fdc), _ptr(frest), _ptr(dsh_), _ptr(means), _ptr(scales),
                                               _ptr(rots), _ptr(opac), _ptr(shs), _stream(dev)))
    return means, scales, rots, opac, shs


def activate_backward(scaling, rotation, opacity, dscale, drot, g_means, g_scales, g_rot, g_opac, g_shs, sinks,
                      has_off, rest_shape, accumulate=True):
    """Backward of activate_forward.  sinks: None, or the parameter .grad buffers to add into in place
    (6, or 4 when the SH were left split: rest_shape None).
    -> ((g_xyz, g_scaling, g_rotation, g_opacity, g_fdc, g_frest), (g_dxyz, g_dscale, g_drot, g_dsh))."""
    lib = _native.load()
    dev = scaling.device
    P = int(scaling.size(0))
    split = rest_shape is None
    R = 0 if split else int(rest_shape[1])
    z = lambda t, shape: torch.zeros(shape, device=dev) if t is None else t  # noqa: E731  (unused grads)
    gm = _dev_f32(z(g_means, (P, 3)), "g_means", dev)
    gs = _dev_f32(z(g_scales, (P, 3)), "g_scales", dev)
    gr = _dev_f32(z(g_rot, (P, 4)), "g_rot", dev)
    go = _dev_f32(z(g_opac, (P, 1)), "g_opac", dev)
    gsh = None if split else _dev_f32(z(g_shs, (P, 1 + R, 3)), "g_shs", dev)
    if sinks is None:
        outs = [torch.empty(P, 3, device=dev), torch.empty(P, 3, device=dev), torch.empty(P, 4, device=dev),
                torch.empty(P, 1, device=dev)]
        outs += [None, None] if split else [torch.empty(P, 1, 3, device=dev), torch.empty(rest_shape, device=dev)]
        acc = 0
    else:
        outs = list(sinks) + ([None, None] if split else [])
        acc = int(bool(accumulate))
    offg = [torch.empty(P, 3, device=dev) if has_off[0] else None,
            torch.empty(P, 3, device=dev) if has_off[1] else None,
            torch.empty(P, 4, device=dev) if has_off[2] else None,
            torch.empty(P, 1 + R, 3, device=dev) if (has_off[3] and not split) else None]
    with torch.cuda.device(dev):
        _native.check(lib.gsd_activate_backward(
            P, R, acc, _ptr(scaling.contiguous()), _ptr(None if dscale is None else dscale.contiguous()),
            _ptr(rotation.contiguous()), _ptr(None if drot is None else drot.contiguous()),
            _ptr(opacity.contiguous()), _ptr(gm), _ptr(gs), _ptr(gr), _ptr(go), _ptr(gsh),
            *[_ptr(t) for t in outs], *[_ptr(t) for t in offg], _stream(dev)))
    return tuple(outs), tuple(offg)
