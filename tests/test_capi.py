"""The C-ABI library: loads without a GPU, exports every symbol include/*.h
declares, and its struct layout matches the ctypes mirror (no compute calls)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gsd_raster.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gsd_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from gsd_amd import _native
    lib = _native.load()
    names = declared_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
        assert n in _native.SIGNATURES, f"{n} has no ctypes signature"
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (gsd_\w+)", out))
    assert set(names) <= exported


def test_abi_version_and_sizes():
    from gsd_amd import _native
    lib = _native.load()
    assert lib.gsd_abi_version() == _native.ABI_VERSION
    assert lib.gsd_geom_buffer_bytes(0, 64, 64) > 0
    assert lib.gsd_geom_buffer_bytes(1000, 64, 64) > lib.gsd_geom_buffer_bytes(10, 64, 64)
    assert lib.gsd_binning_buffer_bytes(1_000_000) >= 20_000_000    # 8 + 8 + 4 B per instance
    assert lib.gsd_image_buffer_bytes(1920, 1080) >= 1920 * 1080 * 8


def test_state_layout_is_aligned_and_disjoint():
    from gsd_amd import _native
    lib = _native.load()
    go, io, bo = (ctypes.c_size_t * 6)(), (ctypes.c_size_t * 6)(), (ctypes.c_size_t * 3)()
    lib.gsd_state_layout(1001, 333, 217, 12345, go, io, bo)
    # binning: point_list first (the backward's part, at a K-independent offset), then keys, scratch
    for arr in (list(go), list(io), [bo[2], bo[0], bo[1]]):
        assert arr == sorted(arr) and len(set(arr)) == len(arr)
    # conic + opacity and rgb are fields of the 64-B render records (one 256-aligned array)
    assert go[1] - 8 == go[2] - 24 and (go[1] - 8) % 256 == 0
    assert go[3] - (go[1] - 8) >= 64 * 1001
    for arr in ([go[0], go[3], go[4], go[5]], list(io), list(bo)):
        assert all(o % 256 == 0 for o in arr)
    assert bo[2] == 0
    assert go[5] + 1001 <= lib.gsd_geom_buffer_bytes(1001, 333, 217) - 256


def test_struct_layout_matches_c(tmp_path):
    from gsd_amd._native import RasterArgs
    c = tmp_path / "sz.c"
    c.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\nint main(){printf("%%zu %%zu %%zu %%zu",'
                 ' sizeof(gsd_raster_args), offsetof(gsd_raster_args, scale_modifier),'
                 ' offsetof(gsd_raster_args, background), offsetof(gsd_raster_args, campos));}\n' % HEADER)
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", str(c), "-o", str(exe)])
    size, sm, bgo, cpo = map(int, subprocess.check_output([str(exe)]).split())
    assert size == ctypes.sizeof(RasterArgs)
    assert (sm, bgo, cpo) == (RasterArgs.scale_modifier.offset, RasterArgs.background.offset,
                              RasterArgs.campos.offset)


def test_argument_errors_without_gpu():
    """Validation happens before any device work, with the reference's messages."""
    from gsd_amd import _native
    lib = _native.load()
    a = _native.RasterArgs(P=10, D=3, M=16, width=64, height=64, scale_modifier=1.0, tan_fovx=0.5, tan_fovy=0.5,
                           means3D=8, opacities=8, viewmatrix=8, projmatrix=8, background=8, campos=8,
                           scales=8, rotations=8)
    K = ctypes.c_int64(0)
    rc = lib.gsd_rasterize_forward_bin(ctypes.byref(a), None, None, None, ctypes.byref(K), None)
    assert rc == 1 and b"excatly one of either SHs or precomputed colors" in lib.gsd_last_error()
    a.shs = 8
    a.cov3D_precomp = 8
    rc = lib.gsd_rasterize_forward_bin(ctypes.byref(a), None, None, None, ctypes.byref(K), None)
    assert rc == 1 and b"scale/rotation pair or precomputed 3D covariance" in lib.gsd_last_error()
    a.cov3D_precomp = None
    a.M = 9
    rc = lib.gsd_rasterize_forward_bin(ctypes.byref(a), None, None, None, ctypes.byref(K), None)
    assert rc == 1 and b"fewer coefficients" in lib.gsd_last_error()
    a.P = -1
    rc = lib.gsd_rasterize_forward_bin(ctypes.byref(a), None, None, None, ctypes.byref(K), None)
    assert rc == 1 and b"means3D must have dimensions (num_points, 3)" in lib.gsd_last_error()
    a.P = 0
    assert lib.gsd_rasterize_forward_bin(ctypes.byref(a), None, None, None, ctypes.byref(K), None) == 0
    assert K.value == 0


def test_mlp_training_heads_argument_errors_without_gpu():
    """The ABI-15 head-wise training entry points validate before any device work: a null head-pointer array, a
    null head output, and (backward) null gradient sinks fail with GSD_ERR_ARG and a message; a NULL head GRADIENT
    is legal (a zero gradient) and never reaches that check."""
    from gsd_amd import _native
    lib = _native.load()
    vp = ctypes.c_void_p
    W = (vp * 12)(*([8] * 12))
    heads = (vp * 4)(8, 8, None, 8)
    rc = lib.gsd_deform_mlp_train_forward_heads(10, 8, 8, W, W, 8, None, None)
    assert rc == 1 and b"null pointer" in lib.gsd_last_error()
    rc = lib.gsd_deform_mlp_train_forward_heads(10, 8, 8, W, W, 8, heads, None)
    assert rc == 1 and b"4 head outputs" in lib.gsd_last_error()
    rc = lib.gsd_deform_mlp_train_backward_heads(10, None, W, 8, 8, 0, W, W, 0, None)
    assert rc == 1 and b"null pointer" in lib.gsd_last_error()
    dW = (vp * 12)(*([8] * 11 + [None]))
    rc = lib.gsd_deform_mlp_train_backward_heads(10, heads, W, 8, 8, 0, dW, W, 0, None)
    assert rc == 1 and b"weight / bias gradients" in lib.gsd_last_error()
    rc = lib.gsd_deform_mlp_train_backward_heads(0, heads, W, 8, 8, 0, W, W, 0, None)
    assert rc == 1 and b"0 < P" in lib.gsd_last_error()


def test_build_id_is_the_hash_of_this_tree():
    """gsd_build_id() (ABI 16) is the SHA-256 the Makefile took of the sources; load() recomputed it from this
    tree and accepted the library."""
    from gsd_amd import _native
    lib = _native.load()
    info = _native.build_info()
    assert info["build_id"] == _native.source_build_id() and len(info["build_id"]) == 64
    assert info["flags"] == lib.gsd_build_flags().decode()


def test_library_built_from_other_sources_is_refused(tmp_path):
    """A copy of the tree with one source byte changed no longer matches the library: check_build_id raises (the
    same check load() runs), while the unchanged copy passes."""
    import shutil

    import pytest

    from gsd_amd import _native
    lib = _native.load()
    csrc = tmp_path / "pkg" / "csrc"
    shutil.copytree(_native.CSRC_DIR, csrc)
    (tmp_path / "include").mkdir()
    shutil.copy(HEADER, tmp_path / "include" / "gsd_raster.h")
    assert _native.check_build_id(lib, csrc=str(csrc)) == _native.source_build_id()
    src = csrc / "gsd_render.hip"
    data = bytearray(src.read_bytes())
    data[100] ^= 0x20
    src.write_bytes(bytes(data))
    with pytest.raises(ImportError, match="built from other sources"):
        _native.check_build_id(lib, csrc=str(csrc))
