#!/usr/bin/env python
"""Host-timed pieces of a densification step on the bench's configuration 5 (2M Gaussians, 4K): a few fused
training steps, densify_and_prune (GaussianDensifier), and the steps right after it.
    python scripts/prof_densify.py [--config 5] [--steps 4]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from bench import make_optimizer  # noqa: E402
from gsd_amd import DeformableGaussians, default_pipe, l1_ssim_loss, render  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.densify import GaussianDensifier  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--steps", type=int, default=4)
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
    dens = GaussianDensifier(pc, opt)

    def step():
        out = render(cam, pc, pipe, bg)
        with opt.step_in_backward():
            l1_ssim_loss(out["render"], target, 0.2).backward()
        dens.add_densification_stats(out["viewspace_points"], out["radii"])

    def timed(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        print("%-28s %8.2f ms" % (name, 1e3 * (time.perf_counter() - t0)), flush=True)

    for i in range(a.steps):
        timed(f"step {i}", step)
    if os.environ.get("PROF_OPS"):   # torch.profiler over the densification: where its host time goes
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            timed("densify_and_prune", lambda: dens.densify_and_prune(0.0002, 0.005, 10.0, None))
        print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25))
    else:
        timed("densify_and_prune", lambda: dens.densify_and_prune(0.0002, 0.005, 10.0, None))
    for i in range(a.steps):
        timed(f"step after {i}", step)
    # the first call above includes PyTorch's one-time code-object loads for its elementwise kernels
    if os.environ.get("PROF_OPS2"):   # torch.profiler over the warm call
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            timed("densify_and_prune (2nd)", lambda: dens.densify_and_prune(0.0002, 0.005, 10.0, None))
        print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=30))
    else:
        timed("densify_and_prune (2nd)", lambda: dens.densify_and_prune(0.0002, 0.005, 10.0, None))
    for i in range(a.steps):
        timed(f"step after 2nd {i}", step)
    print("P", pc._xyz.shape[0])


if __name__ == "__main__":
    main()
