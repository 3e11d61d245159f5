#!/usr/bin/env python
"""Which aten op launches each small kernel of the bench step: torch.profiler over a few bench steps (cfg 4),
device time grouped by op and by (op, kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench import make_optimizer  # noqa: E402
from gsd_amd import DeformableGaussians, default_pipe, l1_ssim_loss, render  # noqa: E402
from gsd_amd.camera import synthetic_camera  # noqa: E402
from gsd_amd.scene import CONFIGS, make_gaussians  # noqa: E402

cfg = CONFIGS[int(os.environ.get("CFG", "4"))]
P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
dev = torch.device("cuda:0")
pc = DeformableGaussians(make_gaussians(P, W, H, seed=4).to(dev), sh_degree=D)
cam = synthetic_camera(W, H).to(dev)
bg = torch.zeros(3, device=dev)
pipe = default_pipe()
with torch.no_grad():
    target = render(cam, pc, pipe, bg)["render"].clone()
opt = make_optimizer(pc)
flat = opt.flat


def step():
    out = render(cam, pc, pipe, bg)
    loss = l1_ssim_loss(out["render"], target, 0.2)
    loss.backward()
    flat.allreduce()
    opt.step(zero_grad=True)


for _ in range(5):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(5):
        step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=70))
print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=30,
                                                    max_name_column_width=60, max_src_column_width=120))
