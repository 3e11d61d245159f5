"""Loader for libgsd_hip.so -- the C-ABI of include/gsd_raster.h.

There is no fallback: if the HIP library is missing or stale the import of the
product path fails loudly (the parity claims rest on the HIP kernels being the
code that runs).
"""
from __future__ import annotations

import ctypes
import hashlib
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GSD_HIP_LIB", os.path.join(_PKG_ROOT, "build", "libgsd_hip.so"))
ABI_VERSION = 17
CSRC_DIR = os.path.join(_PKG_ROOT, "csrc")

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_sz = ctypes.c_size_t


class ShSplit(ctypes.Structure):
    """Mirror of ``gsd_sh_split`` (include/gsd_raster.h)."""

    _fields_ = [("dc", _vp), ("rest", _vp), ("offset", _vp), ("d_dc", _vp), ("d_rest", _vp), ("d_offset", _vp),
                ("accumulate", _i32), ("d_rgb", _vp), ("dc_stride_g", _i64), ("dc_stride_e", _i64),
                ("rest_stride_g", _i64), ("rest_stride_e", _i64), ("defer_view_dir", _i32)]


class Activation(ctypes.Structure):
    """Mirror of ``gsd_activation`` (include/gsd_raster.h)."""

    _fields_ = [("d_xyz", _vp), ("d_scaling", _vp), ("d_rotation", _vp), ("d_opacity", _vp), ("accumulate", _i32)]


class AdamSink(ctypes.Structure):
    """Mirror of ``gsd_adam_sink`` (include/gsd_raster.h)."""

    _fields_ = [("param", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("lr", ctypes.c_double), ("step", _i64)]


class AdamEpilogue(ctypes.Structure):
    """Mirror of ``gsd_adam_epilogue``: the Adam step fused into the rasterizer backward."""

    _fields_ = [("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double),
                ("dc", AdamSink), ("rest", AdamSink), ("xyz", AdamSink), ("scaling", AdamSink),
                ("rotation", AdamSink), ("opacity", AdamSink)]


class RasterArgs(ctypes.Structure):
    """Mirror of ``gsd_raster_args`` (include/gsd_raster.h)."""

    _fields_ = [
        ("P", _i32), ("D", _i32), ("M", _i32), ("width", _i32), ("height", _i32),
        ("scale_modifier", _f32), ("tan_fovx", _f32), ("tan_fovy", _f32),
        ("prefiltered", _i32), ("debug", _i32),
        ("background", _vp), ("means3D", _vp), ("shs", _vp), ("colors_precomp", _vp), ("opacities", _vp),
        ("scales", _vp), ("rotations", _vp), ("cov3D_precomp", _vp), ("viewmatrix", _vp), ("projmatrix", _vp),
        ("campos", _vp), ("sh_split", _vp), ("activation", _vp), ("adam", _vp), ("grad_scratch", _vp),
        ("alpha_mode", _i32),
    ]


class TrainStepArgs(ctypes.Structure):
    """Mirror of ``gsd_train_step_args`` (include/gsd_raster.h, ABI 17)."""

    _fields_ = [
        ("raster", RasterArgs), ("geom_buffer", _vp), ("image_buffer", _vp), ("binning_buffer", _vp),
        ("binning_bytes", _sz), ("radii", _vp), ("out_color", _vp), ("gt", _vp), ("lambda_dssim", _f32),
        ("loss_out3", _vp), ("loss_workspace", _vp), ("dL_dimg", _vp), ("grad_seed", _vp), ("dL_dmeans2D", _vp),
        ("dL_dcolors", _vp), ("scratch", _vp), ("grad_accum", _vp), ("grad_accum_3vec", _vp), ("denom", _vp),
        ("max_radii2D", _vp),
    ]


# name -> (restype, argtypes); every symbol include/gsd_raster.h declares
SIGNATURES = {
    "gsd_abi_version": (_i32, []),
    "gsd_last_error": (ctypes.c_char_p, []),
    "gsd_build_id": (ctypes.c_char_p, []),
    "gsd_build_flags": (ctypes.c_char_p, []),
    "gsd_geom_buffer_bytes": (_sz, [_i32, _i32, _i32]),
    "gsd_image_buffer_bytes": (_sz, [_i32, _i32]),
    "gsd_backward_scratch_bytes": (_sz, [_i32]),
    "gsd_binning_buffer_bytes": (_sz, [_i64]),
    "gsd_state_layout": (None, [_i32, _i32, _i32, _i64, ctypes.POINTER(_sz), ctypes.POINTER(_sz),
                                ctypes.POINTER(_sz)]),
    "gsd_rasterize_forward_bin": (_i32, [ctypes.POINTER(RasterArgs), _vp, _vp, _vp, ctypes.POINTER(_i64), _vp]),
    "gsd_rasterize_forward_render": (_i32, [ctypes.POINTER(RasterArgs), _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "gsd_rasterize_forward": (_i32, [ctypes.POINTER(RasterArgs), _vp, _vp, _vp, _sz, _vp, _vp, ctypes.POINTER(_i64), _vp]),
    "gsd_sh_grad_views": (_i32, [_i32, _i32, _i32, _i32, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "gsd_sh_grad_views_ex": (_i32, [_i32, _i32, _i32, _i32, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp,
                                    _vp, _vp]),
    "gsd_rasterize_backward": (_i32, [ctypes.POINTER(RasterArgs), _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsd_mark_visible": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp]),
    "gsd_se3_deform_forward": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsd_se3_deform_backward": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsd_activate_forward": (_i32, [_i32, _i32] + [_vp] * 15 + [_vp]),
    "gsd_activate_backward": (_i32, [_i32, _i32, _i32] + [_vp] * 20 + [_vp]),
    "gsd_l1_ssim_workspace_bytes": (_sz, [_i32, _i32, _i32]),
    "gsd_l1_ssim": (_i32, [_i32, _i32, _i32, _vp, _vp, _f32, _vp, _vp, _vp, _vp]),
    "gsd_l1_ssim_backward": (_i32, [_i32, _i32, _i32, _vp, _vp, _f32, _vp, _f32, _vp, _vp, _vp]),
    "gsd_offset_norm_workspace_bytes": (_sz, [_i64]),
    "gsd_offset_norm": (_i32, [_i64, _vp, _f32, _vp, _vp, _vp]),
    "gsd_offset_norm_backward": (_i32, [_i64, _vp, _vp, _f32, _vp, _vp]),
    "gsd_adam_step": (_i32, [_i64, _vp, _vp, _vp, _vp, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_f32),
                             ctypes.POINTER(_i64), ctypes.c_double, ctypes.c_double, ctypes.c_double, _i32, _vp]),
    "gsd_adam_step_ex": (_i32, [_i64, _vp, _vp, _vp, _vp, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_f32),
                                ctypes.POINTER(_i64), ctypes.c_double, ctypes.c_double, ctypes.c_double, _i32, _vp,
                                _i64, _i64, _vp]),
    "gsd_densify_stats": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsd_train_step": (_i32, [ctypes.POINTER(TrainStepArgs), ctypes.POINTER(_i64), _vp]),
    "gsd_knn_workspace_bytes": (_sz, [_i32]),
    "gsd_knn_mean_dist2": (_i32, [_i32, _vp, _vp, _vp, _vp]),
    "gsd_deform_mlp_fragments": (_i32, []),
    "gsd_deform_mlp_biases": (_i32, []),
    "gsd_deform_mlp_forward_bf16": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsd_relu_backward_bias_blocks": (_i32, [_i64, _i32]),
    "gsd_relu_backward_bias": (_i32, [_i64, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp]),
    "gsd_deform_mlp_train_workspace_bytes": (_sz, [_i64]),
    "gsd_deform_mlp_train_forward": (_i32, [_i64, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _vp, _vp]),
    "gsd_deform_mlp_train_backward": (_i32, [_i64, _vp, ctypes.POINTER(_vp), _vp, _vp, ctypes.POINTER(_vp),
                                             ctypes.POINTER(_vp), _vp]),
    "gsd_deform_mlp_train_forward_heads": (_i32, [_i64, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp,
                                                  ctypes.POINTER(_vp), _vp]),
    "gsd_deform_mlp_train_backward_heads": (_i32, [_i64, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _vp, _i32,
                                                   ctypes.POINTER(_vp), ctypes.POINTER(_vp), _i32, _vp]),
    "gsd_deform_mlp_eval_workspace_bytes": (_sz, [_i64]),
    "gsd_deform_mlp_eval_forward_heads": (_i32, [_i64, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp,
                                                 ctypes.POINTER(_vp), _vp]),
    "gsd_work_counters": (_i32, [_i32, ctypes.POINTER(ctypes.c_uint64), _i32]),
    "gsd_timing_enable": (_i32, [_i32]),
    "gsd_timing_collect": (_i32, [_i32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64)]),
    "gsd_timing_reset": (None, []),
}


def kernel_times(enable: bool | None = None, reset: bool = False) -> dict:
    """Per-kernel device time of this library's launches: {name: (total_ms, launches)}.
    Synchronises on the last timed launch.  enable=True/False switches recording."""
    lib = load()
    out = {}
    n_max = 32
    names = ctypes.create_string_buffer(32 * n_max)
    tot = (ctypes.c_double * n_max)()
    cnt = (_i64 * n_max)()
    n = lib.gsd_timing_collect(n_max, names, tot, cnt)
    for i in range(n):
        nm = names.raw[32 * i:32 * (i + 1)].split(b"\0", 1)[0].decode()
        out[nm] = (tot[i], int(cnt[i]))
    if reset:
        lib.gsd_timing_reset()
    if enable is not None:
        lib.gsd_timing_enable(1 if enable else 0)
    return out

_lib = None


class NativeError(RuntimeError):
    pass


def source_build_id(csrc: str = CSRC_DIR) -> str:
    """SHA-256 of the sources a library built from `csrc` carries as gsd_build_id(): csrc/*.hip and *.h in name
    order, include/gsd_raster.h, csrc/Makefile -- the same bytes, in the same order, as the Makefile's
    `cat $(ID_SRCS) | sha256sum`."""
    names = sorted(n for n in os.listdir(csrc) if n.endswith((".hip", ".h")))
    paths = [os.path.join(csrc, n) for n in names]
    paths += [os.path.join(csrc, "..", "..", "include", "gsd_raster.h"), os.path.join(csrc, "Makefile")]
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def check_build_id(lib, csrc: str = CSRC_DIR, path: str = LIB_PATH) -> str:
    """Refuse a library whose gsd_build_id() is not the hash of the sources in `csrc` (a stale or foreign build:
    the parity and timing claims are about the kernels of this tree).  GSD_SKIP_BUILD_ID=1 lifts the check for
    A/B experiments that load libraries built from older snapshots (scripts/ab_bench.sh); nothing else sets it."""
    got = lib.gsd_build_id().decode()
    if os.environ.get("GSD_SKIP_BUILD_ID") == "1":
        return got
    want = source_build_id(csrc)
    if got != want:
        raise ImportError(f"gsd: {path} was built from other sources (build id {got[:16]}..., this tree "
                          f"{want[:16]}...); rebuild it with `make -C gaussian-splatting_deformable_amd/csrc`")
    # the source hash does not cover HIPFLAGS_EXTRA: a timing-only build (-DGSD_BWD_ABLATE, -DGSD_COUNT_WORK, ...)
    # of this very tree computes wrong results, so the product path takes only the plain build
    flags = lib.gsd_build_flags().decode().strip()
    if flags:
        raise ImportError(f"gsd: {path} was built with extra flags ({flags!r}); the product path loads only the "
                          "plain build (experiments set GSD_SKIP_BUILD_ID=1)")
    return got


def build_info() -> dict:
    """The loaded library's provenance: path, build id (source hash) and extra compiler flags."""
    lib = load()
    return {"path": LIB_PATH, "build_id": lib.gsd_build_id().decode(), "flags": lib.gsd_build_flags().decode()}


def load():
    """Load and type the library once; raises if it is absent, ABI-mismatched or built from other sources."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"gsd: HIP library not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (make -C gaussian-splatting_deformable_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gsd_abi_version() != ABI_VERSION:
        raise ImportError(f"gsd: {LIB_PATH} has ABI {lib.gsd_abi_version()}, expected {ABI_VERSION}")
    check_build_id(lib)
    _lib = lib
    return lib


GSD_NEED_BINNING = 4


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.gsd_last_error().decode("utf-8", "replace")
        raise NativeError(msg)
