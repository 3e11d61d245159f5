#!/usr/bin/env python
"""One fused deformation-network forward (gsd_mlp.hip) at P Gaussians, for rocprofv3 kernel traces.
    python scripts/prof_mlp_once.py [--P 1000000 --iters 5]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd.deform_mlp import DirectTemporalNeRF  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
net = DirectTemporalNeRF(dtype=torch.bfloat16).cuda()
x = torch.rand(a.P, 3, device="cuda") * 2 - 1
t = torch.full((a.P, 1), 0.3, device="cuda")
with torch.no_grad():
    for _ in range(a.iters):
        out = net(x, t, 10_000)
torch.cuda.synchronize()
print("done", float(out[3].abs().sum()))
