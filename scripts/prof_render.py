#!/usr/bin/env python
"""Profiling harness: N forward+backward passes of the rasterizer on the bench
workload (cfg 4 by default), nothing else -- short enough for rocprofv3 --pmc
passes.   python scripts/prof_render.py [--config 4] [--iters 5]"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd import _C  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--timing", action="store_true", help="print per-kernel device times (gsd_timing_*)")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    dev = torch.device("cuda:0")
    g = make_gaussians(P, W, H, seed=a.config)
    cam = synthetic_camera(W, H).to(dev)
    means = g.xyz.to(dev)
    scales = torch.exp(g.scaling).to(dev)
    rots = torch.nn.functional.normalize(g.rotation, dim=1).to(dev)
    opac = torch.sigmoid(g.opacity).to(dev)
    shs = torch.cat([g.features_dc, g.features_rest], 1).to(dev)
    bg = torch.zeros(3, device=dev)
    e = torch.empty(0)
    tx, ty = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
    dpix = torch.randn(3, H, W, device=dev) * 1e-3
    from gsd_amd._native import kernel_times
    for it in range(a.iters):
        if a.timing and it == 1:
            kernel_times(enable=True, reset=True)
        K, color, radii, geom, binning, img = _C.rasterize_gaussians(
            bg, means, e, opac, scales, rots, 1.0, e, cam.world_view_transform, cam.full_proj_transform, tx, ty, H, W,
            shs, D, cam.camera_center, False, False)
        _C.rasterize_gaussians_backward(bg, means, radii, e, scales, rots, 1.0, e, cam.world_view_transform,
                                        cam.full_proj_transform, tx, ty, dpix, shs, D, cam.camera_center, geom, K,
                                        binning, img, False)
    torch.cuda.synchronize()
    if a.timing:
        for k, (tot, n) in kernel_times(enable=False).items():
            print("%-16s %8.4f ms/launch (%d launches)" % (k, tot / n, n))
    print("done K=%d" % K)


if __name__ == "__main__":
    main()
