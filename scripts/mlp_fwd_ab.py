#!/usr/bin/env python
"""A/B of the deformation network's layer-fused training kernels (round 6): k_mlp_fwd_fused + k_mlp_bwd_chain (w32,
32 Gaussians per wave, one wave per SIMD) against k_mlp_fwd_fused16 + k_mlp_bwd_chain16 (w16, 16 per wave, two per
SIMD; f16c32: the new forward with the old chain) at P Gaussians,
alternating, with the C-ABI's hipEvent times of the forward and backward calls, and the heads / gradients of the
two compared.   python scripts/mlp_fwd_ab.py [--P 1000000] [--reps 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd._native import kernel_times  # noqa: E402
from gsd_amd.deform_mlp import DirectTemporalNeRF  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="w32,w16,f16c32")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    net = DirectTemporalNeRF().to(dev)
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.rand(a.P, 3, device=dev, generator=g) * 2 - 1
    t = torch.full((a.P, 1), 0.3, device=dev)
    w = [torch.randn(a.P, n, device=dev, generator=g) for n in (3, 3, 4, 48)]
    modes = a.modes.split(",")

    def run(mode):   # "w32" / "w16": both the forward and the chain; "f16c32" etc.: each its own
        fwd, chain = (mode, mode) if mode in ("w32", "w16") else ("w" + mode[1:3], "w" + mode[4:6])
        os.environ["GSD_MLP_FWD"], os.environ["GSD_MLP_CHAIN"] = fwd, chain
        net.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        outs = net(xx, t, 10_000)
        sum((o * wi).sum() for o, wi in zip(outs, w)).backward()
        return torch.cat(outs, -1).detach(), [xx.grad] + [p.grad.clone() for p in net.parameters()]

    res = {m: run(m) for m in modes}   # warm + results
    base = res[modes[0]]
    cmp = {}
    for m in modes[1:]:
        o, gr = res[m]
        cmp[m] = {"out": float((o - base[0]).abs().max() / base[0].abs().max())}
        names = ["x"] + [k for k, _ in net.named_parameters()]
        cmp[m]["grads_max_rel"] = max(float((h - r).abs().max() / r.abs().max().clamp_min(1e-30))
                                      for h, r in zip(gr, base[1]))
        cmp[m]["worst"] = max(zip(((float((h - r).abs().max() / r.abs().max().clamp_min(1e-30))) for h, r in
                                   zip(gr, base[1])), names))[1]
    times = {m: [] for m in modes}
    for _ in range(a.reps):
        for m in modes:
            kernel_times(enable=True, reset=True)
            run(m)
            torch.cuda.synchronize()
            kt = kernel_times(enable=False, reset=True)
            times[m].append({k: round(v[0], 4) for k, v in kt.items() if "mlp" in k})
    out = {"P": a.P, "compare_vs_" + modes[0]: cmp, "times_ms": times}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
