#!/usr/bin/env python
"""The deformation network (gsd_amd.deform_mlp.DirectTemporalNeRF) alone: forward and
forward+backward at P Gaussians in f32 and bf16 (autocast on the hidden layers), hipEvent medians, and the
achieved TFLOP/s against the dense MFMA peaks (MI355X: ~157 TFLOP/s f32 matrix, ~2.5 PFLOP/s bf16).
    python scripts/prof_deform_mlp.py [--P 1000000 --iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]

import torch  # noqa: E402

from gsd_amd.deform_mlp import DirectTemporalNeRF  # noqa: E402


def flops_per_gaussian(net):
    """2 x multiply-adds of every Linear (the encoding and ReLUs are not counted)."""
    return 2 * sum(m.in_features * m.out_features for m in net.modules() if isinstance(m, torch.nn.Linear))


def median_ms(fn, iters):
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ts)
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(a.P, 3, generator=g) * 2 - 1).to(dev)
    t = torch.full((a.P, 1), 0.3, device=dev)
    peaks = {torch.float32: 157.3, torch.bfloat16: 2516.6}
    xg = x.clone().requires_grad_(True)   # the reference feeds the trained means (dL/dx computed)
    for dt in (torch.float32, torch.bfloat16):
        net = DirectTemporalNeRF(dtype=dt).to(dev)
        fpg = flops_per_gaussian(net)

        def fwd():
            if dt == torch.float32:   # the training forward: the HIP path only runs when a backward can follow
                net(xg, t, 10_000)
                return
            with torch.no_grad():
                net(x, t, 10_000)

        def fwd_bwd():
            outs = net(xg, t, 10_000)
            sum(o.float().sum() for o in outs).backward()

        if dt == torch.float32:   # the HIP training path (BF16x6) vs torch's f32 GEMMs (GSD_MLP_TORCH=1)
            os.environ["GSD_MLP_TORCH"] = "1"
            for _ in range(2):
                fwd_bwd()
            tf_ms, tfb_ms = median_ms(fwd, a.iters), median_ms(fwd_bwd, a.iters)
            del os.environ["GSD_MLP_TORCH"]
            print("float32   P=%d  torch f32 GEMMs: fwd %.3f ms  fwd+bwd %.3f ms" % (a.P, tf_ms, tfb_ms), flush=True)

        for _ in range(3):
            fwd_bwd()
        if dt == torch.bfloat16:   # no-grad forward: the fused HIP kernel (gsd_mlp.hip) vs torch layer by layer
            os.environ["GSD_MLP_TORCH"] = "1"
            fwd()
            t_ms = median_ms(fwd, a.iters)
            del os.environ["GSD_MLP_TORCH"]
            fwd()
            print("bfloat16  P=%d  no-grad fwd torch %.3f ms (%.1f TFLOP/s)" % (a.P, t_ms, fpg * a.P / (t_ms * 1e-3) / 1e12))
        f_ms = median_ms(fwd, a.iters)
        fb_ms = median_ms(fwd_bwd, a.iters)
        f_tf = fpg * a.P / (f_ms * 1e-3) / 1e12
        fb_tf = 3 * fpg * a.P / (fb_ms * 1e-3) / 1e12
        print("%-9s P=%d  fwd %.3f ms (%.1f TFLOP/s, %.1f %% of %.0f)  fwd+bwd %.3f ms (%.1f TFLOP/s, %.1f %%)"
              % (str(dt).replace("torch.", ""), a.P, f_ms, f_tf, 100 * f_tf / peaks[dt], peaks[dt], fb_ms, fb_tf,
                 100 * fb_tf / peaks[dt]), flush=True)
        if dt == torch.float32:   # BF16x6: six bf16 MFMAs per f32 product -> the f32-accurate roof is 2516.6 / 6
            print("          HIP f32 path vs its BF16x6 roof (419.4 TFLOP/s): fwd %.1f %%  fwd+bwd %.1f %%"
                  % (100 * f_tf / 419.4, 100 * fb_tf / 419.4), flush=True)


if __name__ == "__main__":
    main()
