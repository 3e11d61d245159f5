#!/usr/bin/env python
"""The deformation network's f32 training path alone (gsd_mlp_train.hip, GSD_MLP_TORCH unset): N forward+backward
passes at P Gaussians with dL/dx, for rocprofv3 kernel traces.   python scripts/prof_mlp_train.py [--P 1000000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd.deform_mlp import DirectTemporalNeRF  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    net = DirectTemporalNeRF().to(dev)
    x = (torch.rand(a.P, 3, device=dev) * 2 - 1).requires_grad_(True)
    t = torch.full((a.P, 1), 0.3, device=dev)
    for _ in range(a.iters):
        outs = net(x, t, 10_000)
        sum(o.sum() for o in outs).backward()
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
