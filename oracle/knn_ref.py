"""Test infrastructure only.  Brute-force float32 restatement of simple-knn's distCUDA2
(submodules/simple-knn/simple_knn.cu:125-163): for each point, the three smallest squared distances
dx*dx + dy*dy + dz*dz (float32, in that order, differences other - self) to the other points, padded with
FLT_MAX when there are fewer than three, summed in ascending order and divided by 3.  The reference's
Morton-box search only prunes boxes whose lower-bound distance exceeds the running third best, so it returns
exactly these values."""
from __future__ import annotations

import numpy as np

FLT_MAX = np.float32(np.finfo(np.float32).max)


def mean_dist2(points: np.ndarray) -> np.ndarray:
    pts = np.asarray(points, dtype=np.float32)
    P = pts.shape[0]
    out = np.empty(P, dtype=np.float32)
    for i in range(P):
        d = pts - pts[i]
        dist = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        dist = np.delete(dist, i)
        best = np.sort(dist)[:3]
        if best.size < 3:
            best = np.concatenate((best, np.full(3 - best.size, FLT_MAX, dtype=np.float32)))
        with np.errstate(over="ignore"):
            out[i] = np.float32(np.float32(best[0] + best[1]) + best[2]) / np.float32(3.0)
    return out
