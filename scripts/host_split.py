#!/usr/bin/env python
"""Where the host's time goes in bench.py's step (cfg 4, the fused N = 1 step): per step, the host wall time of
step(), the part before the forward's native call, the native call itself (enqueue of both phases + the wait for the
num_rendered read-back) and everything after it (loss, backward, Adam enqueue).  The device is host-bound when the
read-back wait is no longer than phase 1's own device time: the device had drained the previous step's work before
the host enqueued this one.
    python scripts/host_split.py [--steps 40]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from gsd_amd import DeformableGaussians, _native, default_pipe, render, training_loss  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--config", type=int, default=4)
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    dev = torch.device("cuda:0")
    pc = DeformableGaussians(make_gaussians(P, W, H, seed=args.config).to(dev), sh_degree=D)
    cam = synthetic_camera(W, H).to(dev)
    bg = torch.zeros(3, device=dev)
    pipe = default_pipe()
    with torch.no_grad():
        target = render(cam, pc, pipe, bg)["render"].clone()
    opt = bench.make_optimizer(pc)
    seed = torch.ones((), device=dev)
    lib = _native.load()
    orig = lib.gsd_rasterize_forward
    marks = {}

    def timed_forward(*a):
        marks["f0"] = time.perf_counter()
        rc = orig(*a)
        marks["f1"] = time.perf_counter()
        return rc

    lib.gsd_rasterize_forward = timed_forward

    def step():
        out = render(cam, pc, pipe, bg)
        loss = training_loss(out["render"], target, out["means3D_offset"], 0.2)
        with opt.step_in_backward():
            loss.backward(seed)

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    rows = []
    import gc
    gc.disable()
    t_all = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        rows.append((t1 - t0, marks["f0"] - t0, marks["f1"] - marks["f0"], t1 - marks["f1"]))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) / args.steps
    gc.enable()
    med = [statistics.median(r[i] for r in rows) * 1e3 for i in range(4)]
    print(f"steps {args.steps}: wall {wall * 1e3:.3f} ms/step; host medians (ms): step {med[0]:.3f}, "
          f"before forward call {med[1]:.3f}, forward call (enqueue + read-back wait) {med[2]:.3f}, "
          f"after it {med[3]:.3f}")
    # the same steps with the device kept busy ahead of the host: a long spin kernel first, so the host never
    # waits on an idle device for the enqueue part; the read-back wait then includes the spin
    torch.cuda.synchronize()
    post = []
    for _ in range(10):
        torch.cuda._sleep(2_000_000)
        t0 = time.perf_counter()
        step()
        post.append(time.perf_counter() - marks["f1"])
        torch.cuda.synchronize()
    print(f"after-forward host time with the device busy ahead: {statistics.median(post) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
