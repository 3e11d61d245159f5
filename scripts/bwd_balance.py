#!/usr/bin/env python
"""Load balance of k_render_bwd_quadrant's four waves (one 8x8 quadrant each) on the bench workload: per 256-record
batch every wave walks its own compacted list, and the workgroup's barrier after the batch makes the three
shorter waves wait for the longest.  Counts, from the forward's state (alpha-box test only, the backward's
exact-ellipse test trims ~11 % more), sum over batches of max-over-waves vs mean-over-waves list length.
    python scripts/bwd_balance.py [--config 4]"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsd_amd import _C  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.introspect import decode  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    dev = torch.device("cuda:0")
    g = make_gaussians(P, W, H, seed=a.config)
    cam = synthetic_camera(W, H).to(dev)
    e = torch.empty(0)
    K, color, radii, geom, binning, img = _C.rasterize_gaussians(
        torch.zeros(3, device=dev), g.xyz.to(dev), e, torch.sigmoid(g.opacity).to(dev),
        torch.exp(g.scaling).to(dev), torch.nn.functional.normalize(g.rotation, dim=1).to(dev), 1.0, e,
        cam.world_view_transform, cam.full_proj_transform, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), H, W,
        torch.cat([g.features_dc, g.features_rest], 1).to(dev), D, cam.camera_center, False, False)
    st = {k: v.cpu().numpy() for k, v in decode(P, W, H, K, geom, binning, img).items()}
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    rng = st["ranges"].astype(np.int64)
    nc = np.zeros((gy * 16, gx * 16), np.int64)
    nc[:H, :W] = st["n_contrib"]
    tile_lc = nc.reshape(gy, 16, gx, 16).max(axis=(1, 3)).reshape(T)
    length = np.minimum(rng[:, 1] - rng[:, 0], tile_lc)
    # instances of the backward walk: tile t, list positions rng[t,0] .. rng[t,0] + length - 1
    tiles = np.repeat(np.arange(T), length)
    starts = np.repeat(rng[:, 0], length)
    pos = np.arange(length.sum()) - np.repeat(np.cumsum(length) - length, length)
    back = np.repeat(length, length) - 1 - pos           # index counted from the back (the backward's order)
    batch = back // 256
    gid = st["point_list"].astype(np.int64)[starts + pos]
    xy = st["means2D"][gid]
    co = st["conic_opacity"][gid]
    a_, b_, c_, o_ = co[:, 0], co[:, 1], co[:, 2], co[:, 3]
    det = a_ * c_ - b_ * b_
    t = 2.0 * np.log(np.maximum(255.0 * o_, 1e-30))
    ok = (255.0 * o_ >= 0.999)
    ex = np.sqrt(np.maximum(t, 0) * c_ / np.where(det > 0, det, 1)) * 1.001 + 0.02
    ey = np.sqrt(np.maximum(t, 0) * a_ / np.where(det > 0, det, 1)) * 1.001 + 0.02
    tx0 = (tiles % gx) * 16.0
    ty0 = (tiles // gx) * 16.0
    hits = np.zeros((len(tiles), 4), bool)
    for q in range(4):
        qx0 = tx0 + (q & 1) * 8
        qy0 = ty0 + (q >> 1) * 8
        hits[:, q] = ok & (xy[:, 0] + ex >= qx0) & (xy[:, 0] - ex <= qx0 + 7) & (xy[:, 1] + ey >= qy0) & \
            (xy[:, 1] - ey <= qy0 + 7)
    nb = int(batch.max()) + 1
    key = tiles * nb + batch
    cnt = np.stack([np.bincount(key, weights=hits[:, q], minlength=T * nb) for q in range(4)], 1)
    used = cnt.sum(1) > 0
    cnt = cnt[used]
    s_max, s_mean = cnt.max(1).sum(), cnt.mean(1).sum()
    groups_max = np.ceil(cnt / 4).max(1).sum()
    groups_mean = np.ceil(cnt / 4).mean(1).sum()
    print(f"K={K} walked={len(tiles)} (wave, record) pairs={int(cnt.sum())} batches={len(cnt)}")
    print(f"sum over batches of max-over-waves list length {s_max:.0f}, of the mean {s_mean:.0f}: "
          f"waves busy {s_mean / s_max:.3f} of the batch time (records)")
    print(f"in groups of 4: max {groups_max:.0f} mean {groups_mean:.0f} -> {groups_mean / groups_max:.3f}")
    per_tile = np.bincount(tiles, minlength=T)
    print("records per tile: mean %.1f p50 %d p90 %d p99 %d max %d" % (
        per_tile.mean(), np.percentile(per_tile, 50), np.percentile(per_tile, 90), np.percentile(per_tile, 99),
        per_tile.max()))


if __name__ == "__main__":
    main()
