#!/usr/bin/env python
"""Useful-work counts of the compositing kernels on a BASELINE configuration: one forward + backward of the
bench's view with a library built with -DGSD_COUNT_WORK (gsd_work_counters), e.g.

  make -C gaussian-splatting_deformable_amd/csrc OUT=/tmp/gsdcount HIPFLAGS_EXTRA=-DGSD_COUNT_WORK
  GSD_HIP_LIB=/tmp/gsdcount/libgsd_hip.so python scripts/count_work.py --config 4 --out work_counts_cfg4.json

Writes {"_workload": "cfgN", "render_fwd": {...}, "render_bwd": {...}}: (wave, record) steps, (pixel, record)
pairs and the useful-lane fraction pairs / (64 steps) -- the figures bench.py's roofline block reports beside the
counted VALU issue (profiles/**/work_counts.json).  The scene is the bench's (seed = configuration, camera yaw 0,
the initial parameters), so the counts are those of the bench's first timed view."""
import argparse
import ctypes
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd import _C, _native  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--out", default=None)
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
    dpix = torch.randn(3, H, W, device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 1e-3
    lib = _native.load()
    lib.gsd_work_counters.restype = ctypes.c_int
    lib.gsd_work_counters.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    buf = (ctypes.c_uint64 * 4)()
    _native.check(lib.gsd_work_counters(4, buf, 1))   # zero the counters
    K, color, radii, geom, binning, img = _C.rasterize_gaussians(
        bg, means, e, opac, scales, rots, 1.0, e, cam.world_view_transform, cam.full_proj_transform, tx, ty, H, W,
        shs, D, cam.camera_center, False, False)
    _C.rasterize_gaussians_backward(bg, means, radii, e, scales, rots, 1.0, e, cam.world_view_transform,
                                    cam.full_proj_transform, tx, ty, dpix, shs, D, cam.camera_center, geom, K,
                                    binning, img, False)
    torch.cuda.synchronize()
    _native.check(lib.gsd_work_counters(4, buf, 1))
    c = [int(v) for v in buf]
    if not any(c):
        raise SystemExit("count_work.py: all counters are 0 -- the library was not built with -DGSD_COUNT_WORK")
    res = {"_workload": f"cfg{a.config}", "num_rendered": int(K), "visible": int((radii > 0).sum()),
           "render_fwd": {"wave_record_steps": c[0], "pixel_record_pairs": c[1],
                          "useful_lane_fraction": round(c[1] / (64.0 * c[0]), 4)},
           "render_bwd": {"wave_record_steps": c[2], "pixel_record_pairs": c[3],
                          "useful_lane_fraction": round(c[3] / (64.0 * c[2]), 4)}}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
