#!/usr/bin/env python
"""Host-side cost of one forward through gsd_amd._C (cfg 4): time spent in each phase of
rasterize_gaussians, measured with perf_counter (the device work is synchronised first)."""
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import ctypes  # noqa: E402

import torch  # noqa: E402

from gsd_amd import _C, _native  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402

cfg = CONFIGS[4]
P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
dev = torch.device("cuda:0")
g = make_gaussians(P, W, H, seed=4)
cam = synthetic_camera(W, H).to(dev)
means = g.xyz.to(dev)
scales = torch.exp(g.scaling).to(dev)
rots = torch.nn.functional.normalize(g.rotation, dim=1).to(dev)
opac = torch.sigmoid(g.opacity).to(dev)
shs = torch.cat([g.features_dc, g.features_rest], 1).to(dev)
bg = torch.zeros(3, device=dev)
tx, ty = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
lib = _native.load()
ph = {k: [] for k in ["args", "alloc1", "bin_call", "alloc2", "render_call", "total_gpu_idle_est"]}
for it in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = _C._Args(bg, means, None, opac, scales, rots, 1.0, None, cam.world_view_transform, cam.full_proj_transform,
                 tx, ty, H, W, shs, D, cam.camera_center, False, False)
    t1 = time.perf_counter()
    radii = torch.zeros(P, dtype=torch.int32, device=dev)
    geom = torch.empty(lib.gsd_geom_buffer_bytes(P, W, H), dtype=torch.uint8, device=dev)
    img = torch.empty(lib.gsd_image_buffer_bytes(W, H), dtype=torch.uint8, device=dev)
    K = ctypes.c_int64(0)
    stream = _C._stream(dev)
    t2 = time.perf_counter()
    _native.check(lib.gsd_rasterize_forward_bin(ctypes.byref(a.c), _C._ptr(geom), _C._ptr(img), _C._ptr(radii),
                                                ctypes.byref(K), stream))
    t3 = time.perf_counter()
    binning = torch.empty(lib.gsd_binning_buffer_bytes(K.value), dtype=torch.uint8, device=dev)
    color = torch.empty(3, H, W, dtype=torch.float32, device=dev)
    t4 = time.perf_counter()
    _native.check(lib.gsd_rasterize_forward_render(ctypes.byref(a.c), _C._ptr(geom), _C._ptr(img), _C._ptr(binning),
                                                   K.value, _C._ptr(radii), _C._ptr(color), stream))
    t5 = time.perf_counter()
    torch.cuda.synchronize()
    if it >= 10:
        for k, v in zip(["args", "alloc1", "bin_call", "alloc2", "render_call"], [t1 - t0, t2 - t1, t3 - t2, t4 - t3,
                                                                                   t5 - t4]):
            ph[k].append(v * 1e6)
for k, v in ph.items():
    if v:
        v.sort()
        print("%-12s median %8.1f us" % (k, v[len(v) // 2]))
