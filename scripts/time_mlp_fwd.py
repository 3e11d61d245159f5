#!/usr/bin/env python
"""Median time of the f32 training forward of DirectTemporalNeRF (gsd_deform_mlp_train_forward) at P Gaussians,
or with --bwd of forward + backward (dL/dx included), or with --eval of the evaluation without autograd
(gsd_deform_mlp_eval_forward_heads; with GSD_MLP_TORCH=1: torch's f32 GEMMs), for A/B runs of library builds.
    python scripts/time_mlp_fwd.py [--P 1000000 --iters 20 --bwd | --eval]"""
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--eval", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(0)
    net = DirectTemporalNeRF().cuda()
    x = torch.rand(a.P, 3, device="cuda") * 2 - 1
    t = torch.full((a.P, 1), 0.3, device="cuda")
    xg = x.clone().requires_grad_(True)

    def step():
        if a.eval:
            with torch.no_grad():
                net(x, t, 10_000)
        elif a.bwd:
            sum(o.sum() for o in net(xg, t, 10_000)).backward()
        else:   # the training forward (a backward may follow: the HIP path stores the hidden layers)
            net(xg, t, 10_000)

    for _ in range(3):
        step()
    ev = []
    for _ in range(a.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    print("%s  P=%d  %s median %.3f ms  min %.3f" % (os.environ.get("GSD_HIP_LIB", "default"), a.P, "fwd+bwd" if a.bwd else ("eval" + (" torch" if os.environ.get("GSD_MLP_TORCH") else "") if a.eval else "fwd"),
                                                        ms[len(ms) // 2], ms[0]), flush=True)


if __name__ == "__main__":
    main()
