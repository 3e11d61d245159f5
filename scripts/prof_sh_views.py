#!/usr/bin/env python
"""Times gsd_sh_grad_views (the data-parallel SH gradient assembled from N exchanged views) on the bench's scale:
1M Gaussians, SH3, N views.   python scripts/prof_sh_views.py [--views 8] [--iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    P, N = a.P, a.views
    means = torch.randn(P, 3, device=dev, generator=g) + torch.tensor([0.0, 0.0, 6.0], device=dev)
    stride = 3 * P + 4
    views = torch.zeros(N, stride, device=dev)
    views[:, :3 * P] = torch.randn(N, 3 * P, device=dev, generator=g) * 1e-3
    views[:, 3 * P:3 * P + 3] = torch.randn(N, 3, device=dev, generator=g) * 0.1
    d_dc = torch.empty(P, 1, 3, device=dev)
    d_rest = torch.empty(P, 15, 3, device=dev)
    for _ in range(3):
        _C.sh_grad_views(3, means, views, P, 16, d_dc=d_dc, d_rest=d_rest)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        _C.sh_grad_views(3, means, views, P, 16, d_dc=d_dc, d_rest=d_rest)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    nbytes = P * (12 + N * 12 + 192)
    print(f"sh_grad_views P={P} views={N}: {ms:.4f} ms, {nbytes / ms / 1e6:.0f} GB/s algorithmic; "
          f"checksum {float(d_rest.double().abs().sum()):.6e}")


if __name__ == "__main__":
    main()
