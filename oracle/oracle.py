"""CPU oracle for the rasterizer hot path -- TEST INFRASTRUCTURE ONLY.

numpy/ctypes front end of ``raster_oracle.c`` (a float32 restatement of the
reference's ``cuda_rasterizer/{forward,backward,rasterizer_impl}.cu``).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker: the product path
(``gaussian-splatting_deformable_amd/``) never imports it.

Parity pins (DESIGN.md "Oracle"): SH evaluation, the covariance build, the
camera matrices and the SE(3) exp-map are checked against vectors produced by
the reference's own Python modules (tests/golden/); the rasterizer proper is
pinned by a float64 autograd check of the analytic backward
(oracle/torch_ref.py) -- the CUDA build itself cannot run in this container.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

TILE = 16

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p


def build() -> str:
    """Compile oracle/build/liboracle.so (gcc); returns its path."""
    src = os.path.join(_HERE, "raster_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_preprocess.restype = None
        L.orc_preprocess.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _vp, ctypes.c_float, _vp,
                                     _f32p, _vp, _vp, _vp, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_float, ctypes.c_float, _i32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                     _u32p, _u8p]
        L.orc_higher_msb.restype = ctypes.c_uint32
        L.orc_higher_msb.argtypes = [ctypes.c_uint32]
        L.orc_binning.restype = ctypes.c_int64
        L.orc_binning.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _i32p, _u32p, _vp,
                                  _vp, _vp, _vp]
        L.orc_render_fwd.restype = None
        L.orc_render_fwd.argtypes = [ctypes.c_int, ctypes.c_int, _u32p, _u32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                     _f32p, _u32p, _vp]
        L.orc_render_bwd.restype = None
        L.orc_render_bwd.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u32p, _u32p, _f32p, _f32p, _f32p,
                                     _f32p, _f32p, _u32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_preprocess_bwd.restype = None
        L.orc_preprocess_bwd.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _i32p, _vp, _u8p, _vp,
                                         _vp, ctypes.c_float, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_float, ctypes.c_float, _f32p, _f32p, _f32p, _f32p, _f32p,
                                         _f32p, _f32p, _f32p, _f32p]
        L.orc_sh_to_rgb.restype = None
        L.orc_sh_to_rgb.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _u8p]
        L.orc_cov3d.restype = None
        L.orc_cov3d.argtypes = [ctypes.c_int, _f32p, ctypes.c_float, _f32p, _f32p]
        L.orc_mark_visible.restype = None
        L.orc_mark_visible.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _u8p]
        L.orc_set_threads.restype = None
        L.orc_set_threads.argtypes = [ctypes.c_int]
        L.orc_get_threads.restype = ctypes.c_int
        L.orc_get_threads.argtypes = []
        _lib = L
    return _lib


def set_threads(n: int) -> int:
    """Threads of the oracle's parallel loops (0: OpenMP's default); returns the count in effect."""
    lib().orc_set_threads(int(n))
    return int(lib().orc_get_threads())


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _opt(a):
    """Empty / None inputs are 'absent' (nullptr), as in rasterize_points.cu."""
    if a is None:
        return None, None
    a = _f32(a)
    if a.size == 0:
        return None, None
    return a, a.ctypes.data_as(ctypes.c_void_p)


def higher_msb(n: int) -> int:
    return int(lib().orc_higher_msb(n))


def grid_dims(W: int, H: int):
    return (W + TILE - 1) // TILE, (H + TILE - 1) // TILE


def sh_to_rgb(deg, pos, campos, sh):
    """forward.cu:20-71 for N points: sh (N,M,3) -> (rgb (N,3) clamped >= 0, clamped flags (N,3))."""
    pos = _f32(pos).reshape(-1, 3)
    sh = _f32(sh)
    N, M = sh.shape[0], sh.shape[1]
    rgb = np.zeros((N, 3), np.float32)
    cl = np.zeros((N, 3), np.uint8)
    lib().orc_sh_to_rgb(N, int(deg), M, pos, _f32(campos).reshape(3), sh, rgb, cl)
    return rgb, cl.astype(bool)


def cov3d(scales, rotations, scale_modifier=1.0):
    """forward.cu:118-152 -> (N,6) upper triangle."""
    s = _f32(scales).reshape(-1, 3)
    out = np.zeros((s.shape[0], 6), np.float32)
    lib().orc_cov3d(s.shape[0], s, float(scale_modifier), _f32(rotations).reshape(-1, 4), out)
    return out


def mark_visible(means3D, viewmatrix, projmatrix):
    m = _f32(means3D).reshape(-1, 3)
    out = np.zeros(m.shape[0], np.uint8)
    lib().orc_mark_visible(m.shape[0], m, _f32(viewmatrix).reshape(16), _f32(projmatrix).reshape(16), out)
    return out.astype(bool)


def forward(means3D, opacities, *, shs=None, colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
            viewmatrix, projmatrix, campos, W, H, tanfovx, tanfovy, sh_degree, scale_modifier=1.0, bg=(0, 0, 0)):
    """Reference forward (rasterizer_impl.cu:198-336).  Returns every intermediate."""
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    shs_a, shs_p = _opt(shs)
    M = 0 if shs_a is None else shs_a.reshape(P, -1, 3).shape[1]
    sc_a, sc_p = _opt(scales)
    ro_a, ro_p = _opt(rotations)
    cp_a, cp_p = _opt(cov3D_precomp)
    col_a, col_p = _opt(colors_precomp)
    view = _f32(viewmatrix).reshape(16)
    proj = _f32(projmatrix).reshape(16)
    cam = _f32(campos).reshape(3)
    bg = _f32(bg).reshape(3)
    opac = _f32(opacities).reshape(P)
    radii = np.zeros(P, np.int32)
    means2D = np.zeros((P, 2), np.float32)
    depths = np.zeros(P, np.float32)
    cov3D = np.zeros((P, 6), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    conic = np.zeros((P, 4), np.float32)
    touched = np.zeros(P, np.uint32)
    clamped = np.zeros((P, 3), np.uint8)
    L.orc_preprocess(P, int(sh_degree), M, means3D, sc_p, float(scale_modifier), ro_p, opac, shs_p, cp_p, col_p,
                     view, proj, cam, int(W), int(H), float(tanfovx), float(tanfovy), radii, means2D, depths,
                     cov3D, rgb, conic, touched, clamped)
    offsets = np.zeros(P, np.uint32)
    K = int(L.orc_binning(P, W, H, means2D, depths, radii, touched, offsets.ctypes.data_as(_vp), None, None, None))
    gx, gy = grid_dims(W, H)
    keys = np.zeros(max(K, 1), np.uint64)
    vals = np.zeros(max(K, 1), np.uint32)
    ranges = np.zeros((gx * gy, 2), np.uint32)
    L.orc_binning(P, W, H, means2D, depths, radii, touched, offsets.ctypes.data_as(_vp), keys.ctypes.data_as(_vp),
                  vals.ctypes.data_as(_vp), ranges.ctypes.data_as(_vp))
    keys, vals = keys[:K], vals[:K]
    feats = col_a.reshape(P, 3) if col_a is not None else rgb
    color = np.zeros((3, H, W), np.float32)
    final_T = np.zeros(H * W, np.float32)
    n_contrib = np.zeros(H * W, np.uint32)
    margin = np.zeros((H * W, 2), np.float32)
    L.orc_render_fwd(W, H, ranges, np.ascontiguousarray(vals), means2D, np.ascontiguousarray(feats), conic, bg,
                     color, final_T, n_contrib, margin.ctypes.data_as(_vp))
    return dict(num_rendered=K, color=color, radii=radii, means2D=means2D, depths=depths, cov3D=cov3D, rgb=rgb,
                conic_opacity=conic, tiles_touched=touched, clamped=clamped, point_offsets=offsets, keys=keys,
                point_list=vals, ranges=ranges, final_T=final_T.reshape(H, W), n_contrib=n_contrib.reshape(H, W),
                margin_alpha=margin[:, 0].reshape(H, W), margin_T=margin[:, 1].reshape(H, W), M=M, P=P)


def backward(fwd, dL_dpix, means3D, *, shs=None, colors_precomp=None, scales=None, rotations=None,
             cov3D_precomp=None, viewmatrix, projmatrix, campos, W, H, tanfovx, tanfovy, sh_degree,
             scale_modifier=1.0, bg=(0, 0, 0)):
    """Reference backward (rasterizer_impl.cu:340-434).  Returns the 8 gradients of
    rasterize_points.cu:195 plus dL_dconic (the float4 view of (P,2,2))."""
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    col_a, _ = _opt(colors_precomp)
    bg = _f32(bg).reshape(3)
    feats = col_a.reshape(P, 3) if col_a is not None else fwd["rgb"]
    dpix = _f32(dL_dpix).reshape(3, H, W)
    dmean2D = np.zeros((P, 3), np.float32)
    dconic = np.zeros((P, 4), np.float32)
    dopac = np.zeros((P, 1), np.float32)
    dcolor = np.zeros((P, 3), np.float32)
    L.orc_render_bwd(P, W, H, fwd["ranges"], np.ascontiguousarray(fwd["point_list"]), bg, fwd["means2D"],
                     fwd["conic_opacity"], np.ascontiguousarray(feats), fwd["final_T"].reshape(-1),
                     fwd["n_contrib"].reshape(-1), dpix, dmean2D, dconic, dopac, dcolor)
    pre = preprocess_backward(fwd, dmean2D, dconic, dcolor, means3D, shs=shs, scales=scales, rotations=rotations,
                              cov3D_precomp=cov3D_precomp, viewmatrix=viewmatrix, projmatrix=projmatrix,
                              campos=campos, W=W, H=H, tanfovx=tanfovx, tanfovy=tanfovy, sh_degree=sh_degree,
                              scale_modifier=scale_modifier)
    return dict(dL_dmeans2D=dmean2D, dL_dcolors=dcolor, dL_dopacity=dopac, dL_dconic=dconic, **pre)


def preprocess_backward(fwd, dL_dmean2D, dL_dconic, dL_dcolor, means3D, *, shs=None, scales=None, rotations=None,
                        cov3D_precomp=None, viewmatrix, projmatrix, campos, W, H, tanfovx, tanfovy, sh_degree,
                        scale_modifier=1.0, **_):
    """The per-Gaussian half of the reference backward alone (computeCov2DCUDA + preprocessCUDA bwd,
    backward.cu:144-396, rasterizer_impl.cu:405-434) from given render-level gradients: dL/dmean2D (P,3),
    dL/dconic in the reference's float4 layout (P,4: .x, .y with the 1/2 factor of backward.cu:550, .w) and
    dL/dcolor (P,3).  Fed with a HIP run's own render gradients it checks the HIP preprocess backward's chain
    without the render kernel's float-atomic order noise in its input."""
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    M = fwd["M"]
    _, shs_p = _opt(shs)
    _, sc_p = _opt(scales)
    _, ro_p = _opt(rotations)
    cp_a, _ = _opt(cov3D_precomp)
    dmean2D = np.ascontiguousarray(_f32(dL_dmean2D).reshape(P, 3))
    dconic = np.ascontiguousarray(_f32(dL_dconic).reshape(P, 4))
    dcolor = np.ascontiguousarray(_f32(dL_dcolor).reshape(P, 3))
    dmean3D = np.zeros((P, 3), np.float32)
    dcov3D = np.zeros((P, 6), np.float32)
    dsh = np.zeros((P, max(M, 0), 3), np.float32)
    dscale = np.zeros((P, 3), np.float32)
    drot = np.zeros((P, 4), np.float32)
    cov_used = cp_a.reshape(P, 6) if cp_a is not None else fwd["cov3D"]
    L.orc_preprocess_bwd(P, int(sh_degree), M, means3D, fwd["radii"], shs_p, fwd["clamped"], sc_p, ro_p,
                         float(scale_modifier), np.ascontiguousarray(cov_used), _f32(viewmatrix).reshape(16),
                         _f32(projmatrix).reshape(16), int(W), int(H), float(tanfovx), float(tanfovy),
                         _f32(campos).reshape(3), dmean2D, dconic, dcolor, dmean3D, dcov3D, dsh, dscale, drot)
    return dict(dL_dmeans3D=dmean3D, dL_dcov3D=dcov3D, dL_dsh=dsh, dL_dscales=dscale, dL_drotations=drot)
