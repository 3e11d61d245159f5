"""Decode the opaque state buffers of one forward (debugging / parity tests).

Uses ``gsd_state_layout`` of the C-ABI; returns torch views (on the buffers'
device) of every internal array, so tests can compare intermediate state --
keys, ranges, point_list, radii, depths -- bit for bit with the oracle.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native


def _aligned_base(buf: torch.Tensor) -> int:
    return ((buf.data_ptr() + 255) // 256) * 256 - buf.data_ptr()


def _view(buf, start, dtype, count, cols=None):
    nbytes = count * torch.tensor([], dtype=dtype).element_size() * (cols or 1)
    t = buf[start:start + nbytes].view(dtype)
    return t.view(count, cols) if cols else t


def decode(P, W, H, num_rendered, geom, binning, img):
    lib = _native.load()
    go = (ctypes.c_size_t * 6)()
    io = (ctypes.c_size_t * 6)()
    bo = (ctypes.c_size_t * 3)()
    lib.gsd_state_layout(P, W, H, num_rendered, go, io, bo)
    gb, ib, bb = _aligned_base(geom), _aligned_base(img), _aligned_base(binning) if binning.numel() else 0
    T = ((W + 15) // 16) * ((H + 15) // 16)
    K = int(num_rendered)
    out = dict(
        means2D=_view(geom, gb + go[0], torch.float32, P, 2),
        # conic + opacity and rgb sit inside the 64-B render records (16 floats per Gaussian)
        conic_opacity=_view(geom, gb + go[1] - 8, torch.float32, P, 16)[:, 2:6],
        rgb=_view(geom, gb + go[2] - 24, torch.float32, P, 16)[:, 6:9],
        depths=_view(geom, gb + go[3], torch.float32, P),
        radii_internal=_view(geom, gb + go[4], torch.int32, P),
        clamped=_view(geom, gb + go[5], torch.uint8, P),
        final_T=_view(img, ib + io[0], torch.float32, H * W).view(H, W),
        n_contrib=_view(img, ib + io[1], torch.int32, H * W).view(H, W),
        ranges=_view(img, ib + io[2], torch.int32, T, 2),
        tile_count=_view(img, ib + io[3], torch.int32, T),
    )
    if K > 0:
        out["point_list"] = _view(binning, bb + bo[2], torch.int32, K)
    else:
        out["point_list"] = torch.zeros(0, dtype=torch.int32, device=geom.device)
    return out
