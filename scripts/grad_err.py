#!/usr/bin/env python
"""Relative L2 error of every rasterizer gradient against the C oracle on the parity-test shapes
(tests/test_gpu_parity.py CASES), to see how much room a backward change leaves under the 1e-4 bar.
GSD_HIP_LIB selects a library variant (scripts/exp_variant.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from conftest import scene_inputs  # noqa: E402
from test_gpu_parity import CASES, gpu_backward, gpu_forward, oracle_fwd_bwd, rel_l2  # noqa: E402
from oracle import oracle  # noqa: E402

oracle.build()
names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
         "dL_drotations"]
for P, W, H, deg, seed in CASES + [(100_000, 800, 800, 2, 2)]:
    d = scene_inputs(P, W, H, deg, seed=seed, device="cuda:0")
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(seed)).mul_(1e-3).to("cuda:0")
    _, ob = oracle_fwd_bwd(oracle, d, dpix)
    grads = gpu_backward(d, gpu_forward(d), dpix)
    errs = {n: rel_l2(g.cpu().numpy().reshape(ob[n].shape), ob[n]) for n, g in zip(names, grads)}
    print(f"P={P} {W}x{H} D={deg}: " + " ".join(f"{n[3:]}={e:.2e}" for n, e in errs.items()), flush=True)
