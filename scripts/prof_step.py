#!/usr/bin/env python
"""Profiling harness: N full bench steps (cfg 4 by default: render, loss, backward with the fused Adam step),
nothing else -- short enough for rocprofv3 --pmc passes over the step's kernels (the Adam-bearing preprocess
backward halves above all, which scripts/prof_render.py does not run).
    python scripts/prof_step.py [--config 4] [--steps 3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from bench import make_optimizer  # noqa: E402
from gsd_amd import DeformableGaussians, default_pipe, l1_ssim_loss, render  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    dev = torch.device("cuda:0")
    pc = DeformableGaussians(make_gaussians(P, W, H, seed=a.config).to(dev), sh_degree=D)
    cam = synthetic_camera(W, H).to(dev)
    bg = torch.zeros(3, device=dev)
    pipe = default_pipe()
    with torch.no_grad():
        target = render(cam, pc, pipe, bg)["render"].clamp(0.0, 1.0)
    opt = make_optimizer(pc)
    for _ in range(a.steps):
        with opt.step_in_backward():
            l1_ssim_loss(render(cam, pc, pipe, bg)["render"], target, 0.2).backward()
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
