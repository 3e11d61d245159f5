#!/usr/bin/env python
"""Host-side (Python) cost of the bench step: cProfile over N steps of cfg 4 after warm-up, top functions by
internal time -- where the host spends the time the GPU may wait on after the num_rendered read-back."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch  # noqa: E402

from bench import make_optimizer  # noqa: E402
from gsd_amd import DeformableGaussians, default_pipe, render, training_loss  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402

CFG = int(sys.argv[1]) if len(sys.argv) > 1 else 4   # python scripts/host_profile.py [config]
cfg = CONFIGS[CFG]
P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
dev = torch.device("cuda:0")
pc = DeformableGaussians(make_gaussians(P, W, H, seed=CFG).to(dev), sh_degree=D)
cam = synthetic_camera(W, H).to(dev)
bg = torch.zeros(3, device=dev)
pipe = default_pipe()
with torch.no_grad():
    target = render(cam, pc, pipe, bg)["render"].clone()
opt = make_optimizer(pc)
seed = torch.ones((), device=dev)


def step():   # bench.py's fused N = 1 step
    out = render(cam, pc, pipe, bg)
    loss = training_loss(out["render"], target, out["means3D_offset"], 0.2)
    with opt.step_in_backward():
        loss.backward(seed)


for _ in range(10):
    step()
torch.cuda.synchronize()
import time  # noqa: E402
T0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
print("host+device per step under cProfile: %.3f ms" % (1e3 * (time.perf_counter() - T0) / 50))
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumulative").print_stats(40)
