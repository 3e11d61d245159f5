#!/usr/bin/env python
"""Timing harness for the deformation network's training call: REPS forward + backward passes of
DirectTemporalNeRF at P Gaussians through gsd_deform_mlp_train_* (run under rocprofv3 --kernel-trace --stats, with
GSD_HIP_LIB pointing at a -DGSD_ABLATE=<bits> build to see what each part of a kernel costs; see
gsd_mlp_train.hip)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd.deform_mlp import DirectTemporalNeRF  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = DirectTemporalNeRF().to(dev)
    x = torch.randn(a.P, 3, device=dev).requires_grad_(True)
    t = torch.full((a.P, 1), 0.25, device=dev)
    gh = [torch.randn(a.P, n, device=dev) * 1e-3 for n in (3, 3, 4, 48)]
    for i in range(a.reps + 1):
        if i == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        outs = net(x, t, 5000)
        torch.autograd.backward(outs, gh)
    torch.cuda.synchronize()
    print(f"P={a.P}: {(time.perf_counter() - t0) / a.reps * 1e3:.3f} ms per forward + backward", flush=True)


if __name__ == "__main__":
    main()
