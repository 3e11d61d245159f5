#!/usr/bin/env python
"""Profiling harness for the fused loss (gsd_loss.hip): N value+gradient passes at 3x1080x1920."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch  # noqa: E402

from gsd_amd.loss import l1_ssim_loss  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
gt = torch.rand(3, 1080, 1920, generator=g).to(dev)
x = (gt + 0.05 * torch.randn(3, 1080, 1920, generator=g).to(dev)).clamp(0, 1).requires_grad_(True)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    l1_ssim_loss(x, gt, 0.2).backward()
    x.grad = None
torch.cuda.synchronize()
print("done")
