#!/usr/bin/env python
"""Design study for k_render_bwd's record lists (CPU only, the C oracle's forward of a BASELINE workload).

Counts, per culling granularity, the wave steps the backward would take: per 256-record batch of a tile (back to
front, cut at the tile's largest n_contrib), each wave walks its 8x8 quadrant; with per-lane-group lists the wave
advances as the longest of its groups' lists.  Tests per group rectangle: the alpha box, the exact ellipse, or the
box plus a linear bound of Q over the group (min Q >= Q(c) - |grad Q(c)| . h).  Each group's list is also cut at the
group's largest last contributor (backward.cu:487-488).
    python scripts/sim_bwd_lists.py [--config 4]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT, os.path.join(ROOT, "tests")]


def ellipse_min_q(mx, my, a, b, c, x0, x1, y0, y1):
    """min of Q(d) = a dx^2 + 2 b dx dy + c dy^2 over the rectangle, d = p - m (exact, float64)."""
    dx0, dx1, dy0, dy1 = x0 - mx, x1 - mx, y0 - my, y1 - my
    inside = (dx0 <= 0) & (dx1 >= 0) & (dy0 <= 0) & (dy1 >= 0)

    def edge(a_, b_, c_, dx, lo, hi):
        dy = np.clip(-b_ * dx / c_, lo, hi)
        return a_ * dx * dx + 2 * b_ * dx * dy + c_ * dy * dy

    q = np.minimum(np.minimum(edge(a, b, c, dx0, dy0, dy1), edge(a, b, c, dx1, dy0, dy1)),
                   np.minimum(edge(c, b, a, dy0, dx0, dx1), edge(c, b, a, dy1, dx0, dx1)))
    return np.where(inside, 0.0, q)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256, help="records staged per batch")
    ap.add_argument("--chunks", action="store_true", help="also the union-chunked walks")
    ap.add_argument("--fine", action="store_true", help="also 2x2 and 4x2 lane groups")
    ap.add_argument("--balance", action="store_true", help="only: blocks dealt to waves by list length per batch")
    ap.add_argument("--linonly", action="store_true", help="also 4x4 groups culled by the linear bound alone (no box)")
    a = ap.parse_args()
    from conftest import oracle_kwargs, scene_inputs
    from gsd_amd.scene import CONFIGS
    from oracle import oracle
    cfg = CONFIGS[a.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    d = scene_inputs(P, W, H, D, seed=a.config)
    kw = oracle_kwargs(d)
    t0 = time.time()
    o = oracle.forward(d["means3D"].numpy(), kw["opacities"], shs=kw["shs"], scales=kw["scales"],
                       rotations=kw["rotations"], viewmatrix=kw["viewmatrix"], projmatrix=kw["projmatrix"],
                       campos=kw["campos"], W=W, H=H, tanfovx=kw["tanfovx"], tanfovy=kw["tanfovy"], sh_degree=D)
    print(f"oracle forward {time.time() - t0:.1f} s, K={o['num_rendered']}")
    gx = (W + 15) // 16
    ranges = o["ranges"].astype(np.int64)
    pl = o["point_list"].astype(np.int64)
    K = pl.size
    tile_of = np.repeat(np.arange(ranges.shape[0]), ranges[:, 1] - ranges[:, 0])
    pos = np.arange(K) - ranges[tile_of, 0]
    nc = np.zeros((((H + 15) // 16) * 16, gx * 16), np.int64)
    nc[:H, :W] = o["n_contrib"]
    # per-pixel n_contrib as [tile][16][16]
    nct = nc.reshape(-1, 16, gx, 16).transpose(0, 2, 1, 3).reshape(-1, 16, 16)
    tile_lc = nct.reshape(nct.shape[0], -1).max(1)
    total = np.minimum(ranges[:, 1] - ranges[:, 0], tile_lc)
    keep = pos < total[tile_of]
    tile_of, pos, g = tile_of[keep], pos[keep], pl[keep]
    batch = (total[tile_of] - 1 - pos) // a.batch
    co = o["conic_opacity"].astype(np.float64)[g]
    m2 = o["means2D"].astype(np.float64)[g]
    A, B, C, O = co[:, 0], co[:, 1], co[:, 2], co[:, 3]
    thr = -2.0 * -np.log(255.0 * O)            # Q <= 2 ln(255 o)
    det = A * C - B * B
    tpos = np.maximum(thr, 0)
    ex = np.sqrt(tpos * C / det) * 1.001 + 0.02
    ey = np.sqrt(tpos * A / det) * 1.001 + 0.02
    bx0, bx1, by0, by1 = m2[:, 0] - ex, m2[:, 0] + ex, m2[:, 1] - ey, m2[:, 1] + ey
    tx = (tile_of % gx) * 16.0
    ty = (tile_of // gx) * 16.0
    nb = int(batch.max()) + 1
    print(f"instances replayed {tile_of.size}, batches up to {nb}")

    def count(rw, rh, test):
        """wave steps with groups of rw x rh pixels inside each 8x8 quadrant; returns (wave steps, group list sum)."""
        steps = 0
        lsum = 0
        ng = (8 // rw) * (8 // rh)
        for wq in range(4):
            qx, qy = (wq & 1) * 8, (wq >> 1) * 8
            lens = []
            for gi in range(ng):
                ox, oy = qx + (gi % (8 // rw)) * rw, qy + (gi // (8 // rw)) * rh
                x0, y0 = tx + ox, ty + oy
                x1, y1 = x0 + rw - 1, y0 + rh - 1
                hit = (bx1 >= x0) & (bx0 <= x1) & (by1 >= y0) & (by0 <= y1)
                if test == "exact":
                    hit &= ellipse_min_q(m2[:, 0], m2[:, 1], A, B, C, x0, x1, y0, y1) <= thr * 1.001 + 0.05
                elif test in ("linear", "linonly"):
                    if test == "linonly":
                        hit = np.ones_like(hit)
                    cx, cy = (x0 + x1) * 0.5, (y0 + y1) * 0.5
                    dx, dy = cx - m2[:, 0], cy - m2[:, 1]
                    u, v = A * dx + B * dy, B * dx + C * dy
                    q = dx * u + dy * v
                    hit &= q - (rw - 1) * np.abs(u) - (rh - 1) * np.abs(v) <= thr * 1.001 + 0.05
                elif test == "quadexact":   # the exact test against the quadrant, then the group box
                    hit &= ellipse_min_q(m2[:, 0], m2[:, 1], A, B, C, tx + qx, tx + qx + 7, ty + qy,
                                         ty + qy + 7) <= thr * 1.001 + 0.05
                # group last contributor
                glc = nct[:, oy:oy + rh, ox:ox + rw].reshape(nct.shape[0], -1).max(1)
                hit &= pos < glc[tile_of]
                key = tile_of * nb + batch
                lens.append(np.bincount(key[hit], minlength=ranges.shape[0] * nb))
            L = np.stack(lens)
            steps += int(L.max(0).sum())
            lsum += int(L.sum())
        return steps, lsum

    def count_chunked(C, test="linear"):
        """per-row lists (4x4 blocks) walked in chunks of C entries of the wave's union list: each chunk costs the
        largest number of its entries any one row holds"""
        steps = 0
        for wq in range(4):
            qx, qy = (wq & 1) * 8, (wq >> 1) * 8
            hits = []
            for gi in range(4):
                ox, oy = qx + (gi % 2) * 4, qy + (gi // 2) * 4
                x0, y0 = tx + ox, ty + oy
                x1, y1 = x0 + 3, y0 + 3
                hit = (bx1 >= x0) & (bx0 <= x1) & (by1 >= y0) & (by0 <= y1)
                cx, cy = (x0 + x1) * 0.5, (y0 + y1) * 0.5
                dx, dy = cx - m2[:, 0], cy - m2[:, 1]
                u, v = A * dx + B * dy, B * dx + C_ * dy
                q = dx * u + dy * v
                hit &= q - 3 * np.abs(u) - 3 * np.abs(v) <= thr * 1.001 + 0.05
                glc = nct[:, oy:oy + 4, ox:ox + 4].reshape(nct.shape[0], -1).max(1)
                hit &= pos < glc[tile_of]
                hits.append(hit)
            H4 = np.stack(hits)            # [4][instances], instances in tile order (front to back)
            uni = H4.any(0)
            key = tile_of * nb + batch
            # union index from the back within (tile, batch): instances are in front-to-back order, the walk goes
            # back to front; count union members per key in reverse
            idx = np.nonzero(uni)[0][::-1]
            k = key[idx]
            # rank within key (back to front)
            order = np.argsort(k, kind="stable")
            ks = k[order]
            starts = np.r_[0, np.nonzero(np.diff(ks))[0] + 1]
            rank = np.empty(len(ks), np.int64)
            for a_, b_ in zip(starts, np.r_[starts[1:], len(ks)]):
                rank[a_:b_] = np.arange(b_ - a_)
            chunk = np.empty(len(idx), np.int64)
            chunk[order] = rank // C
            ck = k * 100000 + chunk
            cnt = np.stack([np.bincount(np.searchsorted(np.unique(ck), ck), weights=H4[g][idx]) for g in range(4)])
            steps += int(cnt.max(0).sum())
        return steps

    def count_balance():
        """4x4 linear lists: wave steps with the fixed block -> (wave, row) map against blocks dealt to waves by list
        length per batch (sorted, four consecutive per wave), and the lower bound sum / 4"""
        lens = []
        for blk in range(16):
            ox, oy = (blk % 4) * 4, (blk // 4) * 4
            x0, y0 = tx + ox, ty + oy
            x1, y1 = x0 + 3, y0 + 3
            hit = (bx1 >= x0) & (bx0 <= x1) & (by1 >= y0) & (by0 <= y1)
            cx, cy = (x0 + x1) * 0.5, (y0 + y1) * 0.5
            dx, dy = cx - m2[:, 0], cy - m2[:, 1]
            u, v = A * dx + B * dy, B * dx + C_ * dy
            q = dx * u + dy * v
            hit &= q - 3 * np.abs(u) - 3 * np.abs(v) <= thr * 1.001 + 0.05
            glc = nct[:, oy:oy + 4, ox:ox + 4].reshape(nct.shape[0], -1).max(1)
            hit &= pos < glc[tile_of]
            key = tile_of * nb + batch
            lens.append(np.bincount(key[hit], minlength=ranges.shape[0] * nb))
        L = np.stack(lens)  # [16 blocks][tile * nb + batch]; block = 4 * by + bx
        # the kernel's map: wave w = quadrant (qx, qy), rows = its four 4x4 blocks
        fixed = 0
        for wq in range(4):
            qx, qy = (wq & 1) * 2, (wq >> 1) * 2
            blks = [(qy + j) * 4 + qx + i for j in range(2) for i in range(2)]
            fixed += int(L[blks].max(0).sum())
        Ls = -np.sort(-L, axis=0)
        dealt = int((Ls[0] + Ls[4] + Ls[8] + Ls[12]).sum())
        print(f"4x4 linear lists, batch {a.batch}: wave steps fixed map {fixed}, dealt by length {dealt} "
              f"({dealt / fixed:.3f}), lower bound {int(L.sum()) / 4:.0f} ({L.sum() / 4 / fixed:.3f})")

    C_ = C
    if a.balance:
        count_balance()
        return
    for Cc in ((4, 8, 16, 32) if a.chunks else ()):
        print(f"per-row lists in union chunks of {Cc}: wave steps {count_chunked(Cc)}")
    base = None
    for rw, rh, test in [(8, 8, "exact"), (4, 4, "linear")] + ([(2, 2, "linear"), (4, 2, "linear"), (2, 2, "exact")]
                                                              if a.fine else []) + ([(4, 4, "linonly")] if a.linonly else []):
        t0 = time.time()
        s, ls = count(rw, rh, test)
        base = base or s
        print(f"groups {rw}x{rh} {test:9s}: wave steps {s:>9d} ({s / base:.3f} of 8x8 exact)  "
              f"group-list entries {ls:>9d}  [{time.time() - t0:.1f} s]")


if __name__ == "__main__":
    main()
