#!/usr/bin/env python
"""Loss kernels alone (gsd_loss.hip): --iters forward + backward passes of l1_ssim_loss on a (3, H, W) image,
for rocprofv3 --kernel-trace --stats (k_ssim_fwd, k_loss_sum, k_ssim_bwd), plus a host-event median.
    python scripts/prof_loss.py [--width 1920 --height 1080 --iters 200]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd import l1_ssim_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    y = torch.rand(3, a.height, a.width, generator=g).cuda()
    x = (y + 0.1 * torch.randn(3, a.height, a.width, generator=g).cuda()).clamp(0, 1).requires_grad_(True)
    ts = []
    for _ in range(a.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        l1_ssim_loss(x, y, 0.2).backward()
        e1.record()
        ts.append((e0, e1))
        x.grad = None
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ts)
    print("loss fwd+bwd median %.4f ms" % ms[len(ms) // 2])


if __name__ == "__main__":
    main()
