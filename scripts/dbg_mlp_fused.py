#!/usr/bin/env python
"""Debug: the f32 training forward (and dx) of DirectTemporalNeRF against the torch path at one P, reporting
where they differ.  python scripts/dbg_mlp_fused.py [--P 20000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd.deform_mlp import DirectTemporalNeRF  # noqa: E402


def run(net, x, t, w):
    xx = x.clone().requires_grad_(True)
    outs = net(xx, t, 5000)
    sum((o * wi).sum() for o, wi in zip(outs, w)).backward()
    return torch.cat([o.detach() for o in outs], -1), xx.grad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=20000)
    ap.add_argument("--seed", type=int, default=14)
    a = ap.parse_args()
    torch.manual_seed(a.seed)
    net = DirectTemporalNeRF().cuda()
    P = a.P
    x = torch.rand(P, 3, device="cuda") * 2 - 1
    t = torch.full((P, 1), 0.2, device="cuda")
    w = [torch.randn(P, n, device="cuda") for n in (3, 3, 4, 48)]
    o_h, dx_h = run(net, x, t, w)
    os.environ["GSD_MLP_TORCH"] = "1"
    o_t, dx_t = run(net, x, t, w)
    for name, a_, b_ in (("out", o_h, o_t), ("dx", dx_h, dx_t)):
        err = (a_ - b_).abs().amax(-1)
        bad = torch.nonzero(err > 1e-4 * float(b_.abs().max()) + 1e-7).flatten()
        print("%s: max err %.3g (scale %.3g), %d bad Gaussians" % (name, float(err.max()), float(b_.abs().max()),
                                                                   bad.numel()))
        if bad.numel():
            b = bad.cpu()
            print("   first", b[:20].tolist(), "last", b[-5:].tolist())
            print("   by 32-column group:", sorted(set((b // 32).tolist()))[:40])


if __name__ == "__main__":
    main()
