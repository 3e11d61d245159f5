#!/usr/bin/env python
"""Training-throughput bench (BASELINE.json metric): views/s and fwd+bwd ms/view,
1M Gaussians @ 1920x1080, SH degree 3, one view per GPU.

A step = on every rank (one process per GPU): render() of that rank's view
(activation preamble + HIP rasterizer forward), the reference's training loss
0.8 L1 + 0.2 (1 - SSIM) against a synthetic target (train.py:529, fused HIP
kernel), backward (HIP rasterizer backward + the fused activation backward),
the RCCL all-reduce of the flat per-Gaussian gradient slab (the SH gradient
exchanged as per-view dL/dRGB rows inside the backward; the rest in 32-MB
buckets) overlapped with the reference's Adam step (scene/gaussian_model.py:
834-864 param groups, eps 1e-15), which updates each bucket as its sum
arrives.  Inputs live in HBM before the timed region.  ``value`` = views
processed by all ranks / max-over-ranks wall time of the K timed steps.

Also reported (rank 0): fwd+bwd ms/view (hipEvents, median over >= 100 views,
SURVEY.md 8(d)); per-kernel device times (hipEvents around each launch inside
the C-ABI, from a separate pass so they do not perturb the timed steps); the
roofline of the dominant kernel -- its binding roof from the committed PMC pass
of the same workload (VALU issue for the render kernels, HBM otherwise; traffic
null when no PMC pass of that workload exists); and the CPU baseline -- the
OpenMP C oracle on the host's cores, full views of the same workload for ~10 s.

Every step also updates the densification statistics (max_radii2D and add_densification_stats, train.py:610-618,
which the reference runs every iteration below densify_until_iter); configuration 5 also runs densify_and_prune.

``--with-mlp``: the whole reference training step -- the deformation network DirectTemporalNeRF
(gaussian_model.py:242-316) live in render() at iteration 5000 (offsets on means, scales, rotations and SH), the
offset-norm term of the loss (train.py:329-332) and the network's Adam group (training_setup :843, the offset
schedule's rate at that iteration).  A separate line (config.workload says "MLP live"); the headline is without.

  python bench.py [--gpus N --steps K --warmup W --config 4 --cpu-baseline auto|off --with-mlp]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

``--gpus N`` means N ranks: without a launcher (no WORLD_SIZE in the environment) and N > 1, this process
starts ``torch.distributed.run`` with N ranks on this node and exits with its status, before anything touches
the GPU.  Under a launcher, WORLD_SIZE must equal N; fewer visible devices than ranks is refused unless
GSD_DIST_BACKEND=gloo (the one-GPU rehearsal).

Failure bound at N > 1 (gsd_amd.parallel.DIST_TIMEOUT_S): a rank that raises prints its traceback and exits with
status 1 at once (no interpreter teardown of the process groups, which can block on a dead peer), and
torch.distributed.run then stops the other ranks; a rank that hangs leaves its peers waiting in a collective for
at most GSD_DIST_TIMEOUT_S (default 120 s: every process group is created with it, and RCCL's watchdog aborts the
communicator, TORCH_NCCL_ASYNC_ERROR_HANDLING=1).  So the worst case is about 2 minutes plus start-up, not the
default 10 (RCCL) or 30 (gloo) minutes.
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training views/sec + fwd+bwd ms/view, 1M Gaussians @1080p SH3, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue roof: 256 CUs x 4 SIMDs, a wave64 v_fma_f32 every 2 cycles per SIMD with more than one wave resident
# (MI355X_MICROARCH.md), at the 2.4 GHz peak engine clock -> 1228.8 G wave-instructions/s
VALU_PEAK_GINST = 1024 * 0.5 * 2.4


# Adam's per-Gaussian parameter floats (xyz 3, f_dc 3, f_rest 45, opacity 1, scaling 3, rotation 4) and its bytes per
# float when fused into the preprocess backward: param, exp_avg, exp_avg_sq each read and written (the gradient is
# formed in registers, never stored)
ADAM_FLOATS_PER_G = 59
FUSED_ADAM_BYTES_PER_FLOAT = 24


def algorithmic_bytes(P, V, K, W, H, C, adam_fused=False):
    """Per-launch algorithmic HBM bytes of each kernel (DESIGN.md 'Roofline');
    P Gaussians, V visible, K instances, C = (D+1)^2 SH coefficients.  adam_fused: the bench step at N = 1, where
    the preprocess backward carries the Adam step (gsd_adam_epilogue) -- its bytes are then Adam's 24 B per
    parameter float over all P (the parameter reads serve the backward's own inputs: means, scales, rotations,
    opacities, SH), plus radii 4, the gradient record 48, the clamp flags 1 read and dL/dmean2D 12 written per
    Gaussian; no gradient of a parameter is stored."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    npix = W * H
    return {
        "preprocess_fwd": 44 * P + 12 * C * V + 4 * P + 81 * V,   # 64-B render record per visible Gaussian
        # + the per-chunk tile histograms (B = 512 chunks x T u32): written by the histogram pass, read and
        # rewritten as chunk offsets by the column scans (gsd_binning.hip)
        "tile_hist": 4 * P + 8 * V + 4 * 4 * 512 * T,
        "tile_scan": 16 * T,
        "scatter_keys": 4 * P + 12 * V + 8 * K,
        "tile_sort": 8 * T + 8 * K + 4 * K,
        "render_fwd": 8 * T + 44 * K + 20 * npix,
        "render_bwd": 8 * T + 44 * K + 20 * npix + 44 * V,
        "preprocess_bwd": (FUSED_ADAM_BYTES_PER_FLOAT * ADAM_FLOATS_PER_G * P + (4 + 48 + 1 + 12) * P if adam_fused
                           else 4 * P + (85 + 12 * C) * V + (64 + 12 * C) * V),
        "l1_ssim": 3 * npix * (8 + 12),         # img, gt in; window adjoints out
        "l1_ssim_bwd": 3 * npix * (12 + 8 + 4),  # adjoints, img, gt in; dL/dimg out
        "adam": 32 * P * (3 + 3 + 45 + 1 + 3 + 4),
    }


# the deformation network (DirectTemporalNeRF): multiply-adds per Gaussian of one forward -- 84 -> 256, six
# 256 -> 256, the skip layer 319 -> 256, the four heads 256 -> 58
MLP_MACS_PER_GAUSSIAN = 84 * 256 + 6 * 256 * 256 + 319 * 256 + 256 * 58
# f32 training GEMMs on the bf16 matrix cores at f32 accuracy (BF16x6: six bf16 MFMAs per f32 product): the f32-
# equivalent roof is the dense bf16 peak (MI355X_MICROARCH.md, 2.5166 PFLOP/s) / 6
BF16X6_PEAK_TFLOPS = 2516.6 / 6.0


def mfma_flops(P):
    """Algorithmic FLOPs per call of the deformation network's training kernels: the forward's GEMMs, and the
    backward's dX GEMMs (dL/dx included, as the reference's autograd computes it) plus its weight gradients."""
    f = 2.0 * MLP_MACS_PER_GAUSSIAN * P
    return {"deform_mlp_train_fwd": f, "deform_mlp_train_bwd": 2.0 * f}


def pmc_traffic(kernel, workload):
    """HBM bytes (and the VALU issue figures) per launch of ``kernel`` from the newest committed PMC summary of
    the same workload (profiles/**/pmc_traffic.json whose "_workload" is ``workload``, e.g. "cfg4"; written by
    scripts/pmc_traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE / SQ_* passes over that configuration), or None
    -- a summary of another workload or without a workload tag is never used."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_traffic.json"), recursive=True))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("_workload") == workload and kernel in d:
            return {"hbm_bytes": d[kernel].get("hbm_bytes"), "valu": d[kernel].get("valu"),
                    "source": os.path.relpath(f, ROOT)}
    return None


# FP32 vector peak (MI355X_MICROARCH.md: 157.3 TFLOP/s, v_pk_fma_f32) for the compositing kernels' useful-work figure
FP32_VALU_PEAK_TFLOPS = 157.3
# the reference's arithmetic per useful (pixel, Gaussian) pair, counted from its expressions: forward.cu:332-357 for a
# composited pair (offset 2, power 9, alpha 3, test_T 2, colour 9) and backward.cu:490-555 for a replayed pair
# (offset, power, G, alpha 14; T and alpha T 3; the three channels' accum_rec / dL/dalpha / dL/dcolor 27; dL/dalpha
# scaling and the background term 5; dL/dG, G dx, G dy, dG/d delta 9; the nine gradient sums with their factors 20),
# loop invariants (bg . dL/dpixel) excluded
FLOP_PER_PAIR = {"render_fwd": 25, "render_bwd": 78}


def work_counts(kernel, workload):
    """The useful-work counts of ``kernel`` on ``workload`` from the newest committed count
    (profiles/**/work_counts*.json, scripts/count_work.py with a -DGSD_COUNT_WORK build), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "work_counts*.json"), recursive=True))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("_workload") == workload and kernel in d:
            return dict(d[kernel], source=os.path.relpath(f, ROOT))
    return None


# the kernels behind each C-ABI timing slot (gsd_capi.hip kKernelNames), by their PMC short names (pmc_traffic.py)
TIMING_SLOT_KERNELS = {
    "preprocess_fwd": ["preprocess_fwd"], "tile_hist": ["tile_hist", "colscan_partial", "colscan_final"],
    "tile_scan": ["tile_scan"], "scatter_keys": ["scatter_hist"], "tile_sort": ["tile_sort"],
    "render_fwd": ["render_fwd"], "render_bwd": ["render_bwd"],
    "preprocess_bwd": ["preprocess_bwd_sh_adam", "preprocess_bwd"], "l1_ssim": ["ssim_fwd", "loss_sum"],
    "l1_ssim_bwd": ["ssim_bwd"], "densify_stats": ["densify_stats"],
}


def kernels_vs_hbm(per_kernel, ab, workload):
    """Every timed slot of the step against HBM: algorithmic bytes / live launch time vs 8 TB/s, and -- where a
    committed PMC summary of the bench step itself (workload "cfgN-step", rocprofv3 --pmc over bench.py) holds every
    kernel of the slot -- the measured bytes and their ratio to the algorithmic ones."""
    out = {}
    for k, ms in per_kernel.items():
        if k not in ab or ms <= 0:
            continue
        gbs = ab[k] / (ms * 1e-3) / 1e9
        e = {"algorithmic_bytes": int(ab[k]), "gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
        trs = [pmc_traffic(n, workload) for n in TIMING_SLOT_KERNELS.get(k, [k])]
        if trs and all(t is not None and t.get("hbm_bytes") is not None for t in trs):
            e["traffic"] = int(sum(t["hbm_bytes"] for t in trs))
            e["traffic_over_algorithmic"] = round(e["traffic"] / max(ab[k], 1), 3)
            e["traffic_source"] = trs[0]["source"]
        out[k] = e
    return out


def roofline(kernel, ms, nbytes, workload):
    """The dominant kernel against its binding roof.  HBM: algorithmic bytes / the live average launch time vs
    8 TB/s.  VALU issue (when a PMC pass of this workload counted the kernel's instructions): the counted wave64
    VALU instructions per launch / the live launch time vs VALU_PEAK_GINST.  ``bound`` is whichever of the two
    the kernel is closer to; the other stays in the block as a secondary figure."""
    ach = nbytes / (ms * 1e-3) / 1e9
    hbm = {"achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}
    roof = {"kernel": kernel, "bound": "hbm", **hbm, "traffic": None, "algorithmic_bytes": int(nbytes),
            "avg_launch_ms": round(ms, 4), "workload": workload}
    tr = pmc_traffic(kernel, workload)
    if tr is None:
        return roof
    roof["traffic"] = tr["hbm_bytes"]
    roof["traffic_source"] = tr["source"]
    v = tr.get("valu")
    if v and v.get("instructions"):
        rate = v["instructions"] / (ms * 1e-3) / 1e9
        valu = {"achieved": round(rate, 2), "peak": VALU_PEAK_GINST, "unit": "G wave64-VALU-instr/s",
                "frac": round(rate / VALU_PEAK_GINST, 4), "instructions_per_launch": int(v["instructions"]),
                "pmc_issue_per_simd_cycle": v.get("issue_per_simd_cycle"),
                "pmc_lds_issue_wait_frac": v.get("lds_issue_wait_frac")}
        if valu["frac"] > hbm["frac"]:
            roof.update(bound="valu", achieved=valu["achieved"], peak=valu["peak"], unit=valu["unit"],
                        frac=valu["frac"])
            roof["valu"] = valu
            roof["hbm"] = hbm
        else:
            roof["valu"] = valu
    wc = work_counts(kernel, workload)
    if wc and kernel in FLOP_PER_PAIR:
        # SURVEY.md 8(d)'s secondary figure: useful (pixel, Gaussian) pairs x the reference's FLOPs per pair / the
        # live launch time, against the FP32 vector peak; and the issue figure scaled by the fraction of lanes
        # doing useful work (counted pairs / (64 x counted wave-steps))
        fl = wc["pixel_record_pairs"] * FLOP_PER_PAIR[kernel]
        ach = fl / (ms * 1e-3) / 1e12
        pairs = {"pairs_per_launch": wc["pixel_record_pairs"], "flop_per_pair": FLOP_PER_PAIR[kernel],
                 "achieved": round(ach, 3), "peak": FP32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(ach / FP32_VALU_PEAK_TFLOPS, 4), "wave_record_steps": wc["wave_record_steps"],
                 "useful_lane_fraction": wc["useful_lane_fraction"], "source": wc["source"]}
        if roof.get("valu"):
            pairs["valu_issue_x_useful_lanes"] = round(roof["valu"]["frac"] * wc["useful_lane_fraction"], 4)
        roof["pairs"] = pairs
    return roof


def mfma_roofline(kernel, ms, flops, workload):
    """A matrix-core kernel against the BF16x6 f32-equivalent roof: algorithmic FLOPs / live launch time."""
    ach = flops / (ms * 1e-3) / 1e12
    return {"kernel": kernel, "bound": "mfma", "achieved": round(ach, 2), "peak": round(BF16X6_PEAK_TFLOPS, 1),
            "unit": "TFLOP/s", "frac": round(ach / BF16X6_PEAK_TFLOPS, 4), "traffic": None,
            "algorithmic_flops": flops, "avg_launch_ms": round(ms, 4), "workload": workload}


FUSED_STEP = os.environ.get("GSD_FUSED_STEP", "1") != "0"
MLP_ITERATION = 5000   # >= 3000: the network's offsets are live (gaussian_model.py:308-313)


def make_optimizer(pc, net=None):
    """training_setup (scene/gaussian_model.py:834-864) param groups, spatial_lr_scale = 1, eps 1e-15, as one
    fused HIP Adam over flat slabs (gsd_amd.optim.FusedAdam; torch.optim.Adam semantics).  In the SE(3) mode the
    per-Gaussian twist (the deformation network's output in the dormant reference path,
    scene/gaussian_model.py:99-173) is a trained parameter of its own group, so d_se3 reaches the optimizer."""
    from gsd_amd.optim import FusedAdam
    groups = [{"params": [pc._xyz], "lr": 0.00016, "name": "xyz"}]
    if net is not None:   # training_setup :843, at the offset schedule's rate of the bench's iteration
        from gsd_amd.schedule import offset_schedule
        groups.append({"params": list(net.parameters()), "lr": float(offset_schedule()(MLP_ITERATION)),
                       "name": "offset_model"})
    groups += [
        {"params": [pc._features_dc], "lr": 0.0025, "name": "f_dc"},
        {"params": [pc._features_rest], "lr": 0.0025 / 20.0, "name": "f_rest"},
        {"params": [pc._opacity], "lr": 0.05, "name": "opacity"},
        {"params": [pc._scaling], "lr": 0.005, "name": "scaling"},
        {"params": [pc._rotation], "lr": 0.001, "name": "rotation"},
    ]
    if getattr(pc, "deform", "additive") == "se3" and pc._twist is not None:
        groups.append({"params": [pc._twist], "lr": 0.0008, "name": "twist"})
    return FusedAdam(groups, lr=0.0, eps=1e-15)


def host_cpu():
    """CPU model name and the CPUs this process may run on (lscpu's "Model name" and the affinity mask)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, avail


def cpu_baseline(cfg, seed, min_seconds=10.0, max_views=64):
    """The C oracle (oracle/raster_oracle.c) on the host cores: OpenMP over Gaussians and tiles with OpenMP's
    default thread count (OMP_NUM_THREADS: 16 on the GPU box, this process's CPU share there), full views
    forward + backward of the same workload repeated until ~``min_seconds`` have passed."""
    import numpy as np

    from gsd_amd.camera import synthetic_camera
    from gsd_amd.scene import make_gaussians
    from oracle import oracle

    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
    g = make_gaussians(P, W, H, seed=seed)
    cam = synthetic_camera(W, H)
    kw = dict(shs=torch.cat([g.features_dc, g.features_rest], 1).numpy(), scales=torch.exp(g.scaling).numpy(),
              rotations=torch.nn.functional.normalize(g.rotation, dim=1).numpy(),
              viewmatrix=cam.world_view_transform.numpy(), projmatrix=cam.full_proj_transform.numpy(),
              campos=cam.camera_center.numpy(), W=W, H=H, tanfovx=math.tan(cam.FoVx / 2),
              tanfovy=math.tan(cam.FoVy / 2), sh_degree=D)
    opac = torch.sigmoid(g.opacity).numpy()
    dpix = np.random.default_rng(0).standard_normal((3, H, W)).astype(np.float32) * 1e-3
    oracle.build()
    threads = oracle.set_threads(0)
    model, avail = host_cpu()
    xyz = g.xyz.numpy()
    n = 0
    t0 = time.perf_counter()
    while True:
        fwd = oracle.forward(xyz, opac, **kw)
        oracle.backward(fwd, dpix, xyz, **kw)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds or n >= max_views:
            break
    share = os.environ.get("OMP_NUM_THREADS")
    return {"value": n / dt, "unit": "views/s", "cores": threads, "kind": "port",
            "host": {"model": model, "cpus_available": avail, "omp_threads": threads,
                     "threads_why": (f"OMP_NUM_THREADS={share}: the CPU share of one GPU's process on this host (the "
                                     "GPU box sets it; its affinity mask shows every CPU of the machine, shared by the "
                                     "other GPUs' jobs) -- the baseline uses the cores a one-GPU job owns"
                                     if share else "OpenMP's default: every CPU in the affinity mask")},
            "sample": f"{n} full views of the bench workload (P={P}, {W}x{H}, SH{D}) forward+backward with the "
                      f"OpenMP C oracle on {threads} threads ({model}): {dt:.1f} s"}


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launcher_argv(n, argv, port):
    """The torch.distributed.run command that runs this script as ``n`` ranks on this node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def check_ranks(gpus, env=None):
    """Refusals of --gpus N (before anything touches the GPU): returns an error message or None.
    Under a launcher WORLD_SIZE must be N; N ranks need N visible devices unless GSD_DIST_BACKEND=gloo (several
    ranks on one GPU, the rehearsal of the data-parallel path)."""
    env = os.environ if env is None else env
    if gpus < 1:
        return f"--gpus must be >= 1, got {gpus}"
    ws = env.get("WORLD_SIZE")
    if ws is not None and int(ws) != gpus:
        return f"--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks"
    if gpus > 1 and env.get("GSD_DIST_BACKEND") != "gloo":
        ndev = torch.cuda.device_count()   # counts devices without initialising HIP in this process
        if ndev < gpus:
            return f"--gpus {gpus} needs {gpus} visible GPUs, found {ndev} (GSD_DIST_BACKEND=gloo rehearses on fewer)"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--densify-interval", type=int, default=None,
                    help="densify_and_prune every N steps (train.py:610-648); default 100 for config 5, else off")
    ap.add_argument("--with-mlp", action="store_true",
                    help="DirectTemporalNeRF live in the step (iteration 5000): offsets, offset-norm loss, its Adam")
    args = ap.parse_args()
    err = check_ranks(args.gpus)
    if err:
        print(f"bench.py: {err}", file=sys.stderr)
        sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # N ranks on this node: a child launcher, started before this process initialises the GPU
        sys.exit(subprocess.call(launcher_argv(args.gpus, sys.argv[1:], free_port())))

    from gsd_amd import DeformableGaussians, default_pipe, render, training_loss
    from gsd_amd import _C as gsdC
    from gsd_amd._native import kernel_times
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.parallel import dp_active, init_from_env
    from gsd_amd.scene import CONFIGS, make_gaussians

    rank, local, world = init_from_env()
    if os.environ.get("GSD_DIST_BACKEND") == "gloo":   # rehearsal of the N > 1 path on fewer GPUs
        local %= max(1, torch.cuda.device_count())
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    cfg = CONFIGS[args.config]
    P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]

    se3 = cfg.get("se3") is not None   # configurations 1 and 3: the per-Gaussian SE(3) deform and its gradient
    # configuration 5: "densification/prune step active" -- densify_and_prune every 100 views, so P changes
    densify_every = args.densify_interval if args.densify_interval is not None else (100 if args.config == 5 else 0)
    params = make_gaussians(P, W, H, seed=args.config, se3=cfg.get("se3")).to(dev)   # replicated on every rank
    net = None
    if args.with_mlp:
        if se3:
            print("bench.py: --with-mlp runs the reference's additive deform (configurations 2, 4, 5)", file=sys.stderr)
            sys.exit(2)
        from gsd_amd.deform_mlp import DirectTemporalNeRF
        torch.manual_seed(1234)   # the same initial network on every rank
        net = DirectTemporalNeRF().to(dev)
    iteration = MLP_ITERATION if net is not None else 0
    pc = DeformableGaussians(params, sh_degree=D, deform="se3" if se3 else "additive", offset_model=net)
    cam = synthetic_camera(W, H, yaw_deg=2.0 * rank).to(dev)     # one view per GPU, yaw offsets k*2 deg
    bg = torch.zeros(3, device=dev)
    pipe = default_pipe()
    # synthetic ground truth consistent with the scene: the initial render of this view plus N(0, 0.02) noise,
    # so the optimisation stays near the configured workload (a random target drives opacities and scales
    # away from it within tens of steps, shrinking num_rendered while the bench runs)
    with torch.no_grad():
        target = render(cam, pc, pipe, bg, iteration)["render"]
        noise = torch.randn(3, H, W, generator=torch.Generator().manual_seed(100 + rank)).to(dev)
        target = (target + 0.02 * noise).clamp_(0.0, 1.0)
    opt = make_optimizer(pc, net)
    # every .grad is a view of one slab (opt.flat): the one buffer the all-reduce sums
    from gsd_amd.densify import GaussianDensifier
    dens = GaussianDensifier(pc, opt)   # the statistics run every step; densify_and_prune every densify_every
    nstep = [0]

    # autograd's seed gradient d loss / d loss = 1, allocated once (a bare loss.backward() launches a fill each
    # step; identical semantics)
    seed = torch.ones((), device=dev)

    # The step as one native call (gsd_amd.train_step.FusedTrainStep: the drop-in path's kernels with the same
    # arguments, its argument structures built once) where it applies -- one rank, no offsets / SE(3) -- so the host
    # does not pace small views; GSD_TRAIN_STEP=0 times the drop-in API path (render + training_loss +
    # step_in_backward + add_densification_stats) instead.  Both are timed below (value: the former).
    fused_step = None
    if FUSED_STEP and world == 1 and net is None and not se3 and os.environ.get("GSD_TRAIN_STEP", "1") != "0":
        from gsd_amd.train_step import FusedTrainStep
        fused_step = FusedTrainStep(pc, opt, cam, target, bg, 0.2, densifier=dens)

    def step():
        if fused_step is not None:
            out = fused_step()
            nstep[0] += 1
            if densify_every and nstep[0] % densify_every == 0:
                dens.densify_and_prune(0.0002, 0.005, 10.0, None)
            return out
        return dropin_step()

    def dropin_step():
        out = render(cam, pc, pipe, bg, iteration)
        # train.py:323-332 + :529, lambda_dssim = 0.2: the offset-norm term is 0 (and skipped) when nothing moves
        # the means (configurations 2, 4, 5); in the SE(3) mode (1, 3) it is the moved distance's mean norm
        loss = training_loss(out["render"], target, out["means3D_offset"], 0.2)
        if FUSED_STEP:
            # backward + Adam: at N = 1 every gradient is final inside the preprocess backward, which applies
            # the Adam step there (FusedAdam.step_in_backward, gsd_adam_epilogue); with N > 1 the gradients
            # are summed first, and leaving the block runs allreduce_step as below
            with opt.step_in_backward():
                loss.backward(seed)
        else:
            loss.backward(seed)
            # the gradient all-reduce (RCCL, bucketed, asynchronous) overlapped with the Adam pass, which runs
            # over each bucket as its sum arrives; a no-op collective at N = 1.  The gradient slab is marked
            # stale for the next step instead of cleared.
            opt.allreduce_step(zero_grad=True)
        # train.py:610-618, every iteration below densify_until_iter: max_radii2D + add_densification_stats (one
        # fused pass); train.py:640-644 with the reference's thresholds (densify_grad_threshold 0.0002, min opacity
        # 0.005) every densify_every steps; the synthetic scene's extent is its depth range (z in [2, 10])
        dens.add_densification_stats(out["viewspace_points"], out["radii"])
        nstep[0] += 1
        if densify_every and nstep[0] % densify_every == 0:
            dens.densify_and_prune(0.0002, 0.005, 10.0, None)   # new slabs (FusedAdam.rebuild): opt.flat
        return out

    # Adam moves every parameter by ~lr per step whatever the gradient, so the scene drifts from the configured
    # workload as steps accumulate; each measurement below starts from the initial parameters and optimizer
    # state (restored outside the timed regions; with densification the initial scene is rebuilt, P included)
    trained = list(pc.parameters()) + (list(net.parameters()) if net is not None else [])
    snapshot = [p.detach().clone() for p in trained]

    def restore():
        with torch.no_grad():
            if pc._xyz.shape[0] != snapshot[0].shape[0]:   # densified: the initial P back
                init = dict(zip(dens._names(), snapshot))
                dens._apply(lambda n, d, m, v: (init[n].clone(), torch.zeros_like(init[n]), torch.zeros_like(init[n])))
            for p, s0 in zip(trained, snapshot):
                p.copy_(s0)
            opt.reset_state()
            dens._reset_stats()
        nstep[0] = 0
        opt.flat.invalidate()   # as a fresh optimizer: no gradients yet

    gc.collect()   # before the warmup, so the device is busy again when the timed steps start
    restore_first = os.environ.get("GSD_BENCH_RESTORE_FIRST") == "1"   # diagnostics: no restore after the warmup
    for _ in range(args.warmup):
        step()
    if densify_every:
        # one densification in the warmup as well: PyTorch loads each elementwise kernel's code object on its
        # first launch (~0.1 s over densify_and_prune's ops on a fresh process), a one-time cost, not a step's
        dens.densify_and_prune(0.0002, 0.005, 10.0, None)
    if not restore_first:
        restore()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    step_ev = [] if os.environ.get("GSD_BENCH_STEP_TIMES") else None   # diagnostics: per-step device times
    step_host = []
    # Python's cyclic garbage collector off inside the timed steps (as timeit does): a collection pass stalls the
    # host, which paces the device through the per-step num_rendered read-back (+0.15 ms on one step of every
    # ~10 at 1M Gaussians).  The collection is done before the warmup: a pause of the host here, with the device
    # idle, let its clocks drop for the first timed steps.
    no_gc = os.environ.get("GSD_BENCH_GC", "off") == "off"
    if no_gc:
        gc.disable()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if step_ev is not None:
            step_ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
            step_ev[-1][0].record()
            th = time.perf_counter()
        out = step()
        if step_ev is not None:
            step_ev[-1][1].record()
            step_host.append(1000.0 * (time.perf_counter() - th))
        if i == 0:
            K_start = int(gsdC.last_forward.get("num_rendered", 0))  # host value, already read by the forward
    torch.cuda.synchronize()
    if no_gc:
        gc.enable()
    if step_ev is not None and rank == 0:
        print("step ms:", " ".join("%.3f" % a.elapsed_time(b) for a, b in step_ev), file=sys.stderr)
        print("host ms:", " ".join("%.3f" % h for h in step_host), file=sys.stderr)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    K_end = int(gsdC.last_forward.get("num_rendered", 0))
    P_end = int(pc._xyz.shape[0])   # densified count at the end of the timed steps
    # data parallel: the replicated parameters must still be bit-identical on every rank after the timed steps
    # (every rank applies the same summed gradients): a bit-pattern checksum of the parameter slab, min == max
    replicas = None
    if world > 1:
        with torch.no_grad():
            ck = opt.param_slab.view(torch.int32).to(torch.int64).sum().reshape(1)
            lo, hi = ck.clone(), ck.clone()
            if dist.get_backend() == "nccl":
                dist.all_reduce(lo, op=dist.ReduceOp.MIN)
                dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            else:
                lo, hi = lo.cpu(), hi.cpu()
                dist.all_reduce(lo, op=dist.ReduceOp.MIN)
                dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            replicas = bool(int(lo.item()) == int(hi.item()))
    # GSD_BENCH_STEP_ONLY=1 (profiling: rocprofv3 --pmc over this script): only the warmup and the timed steps, so
    # every launch the counters see is a bench step's; the line then carries no fwd+bwd or per-kernel figures
    if os.environ.get("GSD_BENCH_STEP_ONLY") == "1":
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": round(world * args.steps / elapsed, 3), "unit": "views/s",
                              "n_gpus": world, "steps": args.steps, "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
                              "step_only": True}), flush=True)
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        return
    # the drop-in API's step (render + training_loss + step_in_backward + add_densification_stats, what a user of
    # the reference's interface runs) over the same number of steps, for comparison with the one-call step above
    dropin = None
    if fused_step is not None:
        restore()
        for _ in range(3):
            dropin_step()
        restore()
        torch.cuda.synchronize()
        if no_gc:
            gc.disable()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            dropin_step()
        torch.cuda.synchronize()
        dropin_s = time.perf_counter() - t1
        if no_gc:
            gc.enable()
        dropin = {"ms_per_step": round(1000.0 * dropin_s / args.steps, 4),
                  "views_per_s": round(args.steps / dropin_s, 3)}
    restore()
    # fwd+bwd ms/view: render + loss + backward of one view (no optimizer / collective),
    # hipEvents on the current stream, median over >= 100 views, two ways:
    #   queued  -- a ~1 ms spin kernel ahead of the first event holds the stream while the host enqueues the
    #              view, so the time is the device's (the host still waits for num_rendered mid-forward, as the
    #              reference does, and whatever it does after that read-back is on the clock);
    #   synced  -- the host starts enqueueing after the first event: its Python prologue is on the clock too.
    def fwd_bwd(queued):
        ts = []
        opt.flat.invalidate()
        for _ in range(max(100, args.steps)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if queued:
                torch.cuda._sleep(2_000_000)
            e0.record()
            o = render(cam, pc, pipe, bg, iteration)
            training_loss(o["render"], target, o["means3D_offset"], 0.2).backward(seed)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
            opt.flat.invalidate()   # as after the optimizer step: the next backward stores into the slab
        ts.sort()
        return ts[len(ts) // 2]

    fwd_bwd_ms = fwd_bwd(True)
    fwd_bwd_synced_ms = fwd_bwd(False)

    # the data-parallel exchange on its own (SURVEY.md 8(e) "all-reduce ms"), at the sizes of the step's: the
    # all-gather of the per-view masked dL/dRGB rows (3P + 3 floats per rank) and the all-reduce of the rest of the
    # gradient slab (every parameter but the SH pieces, which the ranks assemble from the gathered views); medians
    # of 10 after 2 warm-ups, hipEvents on the current stream around the (synchronous) collective
    exchange = None
    if world > 1:
        n_red = sum(p.numel() for p in pc.parameters()) - pc._features_dc.numel() - pc._features_rest.numel()
        red = torch.zeros(n_red, device=dev)
        row = torch.zeros(3 * P + 3, device=dev)
        rows = torch.empty(world, 3 * P + 3, device=dev)
        nccl = dist.get_backend() == "nccl"

        def gather():
            if nccl:
                dist.all_gather_into_tensor(rows, row)
            else:
                dist.all_gather(list(rows.unbind(0)), row)

        def timed_ms(fn):
            ts = []
            for it in range(12):
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(e0.elapsed_time(e1))
            ts.sort()
            return ts[len(ts) // 2]

        exchange = {"backend": dist.get_backend(),
                    "allreduce_floats": int(n_red), "allreduce_ms": round(timed_ms(lambda: dist.all_reduce(red)), 4),
                    "allgather_floats_per_rank": 3 * P + 3, "allgather_ms": round(timed_ms(gather), 4)}
        del red, row, rows

    # per-kernel device times: a separate pass of full steps with the C-ABI's hipEvent timing on
    restore()
    kernel_times(enable=True, reset=True)
    n_timing_steps = min(20, max(5, args.steps))
    for _ in range(n_timing_steps):
        out = step()
    torch.cuda.synchronize()
    kt = kernel_times(enable=False, reset=True)

    if rank == 0:
        V = int((out["radii"] > 0).sum())
        K = int(gsdC.last_forward.get("num_rendered", 0))
        steps = args.steps
        per_kernel = {k: tot / max(n, 1) for k, (tot, n) in kt.items()}
        dom = max(kt, key=lambda k: kt[k][0]) if kt else None
        roof = None
        adam_fused = FUSED_STEP and net is None and world == 1 and not dp_active()
        kernel_hbm = kernels_vs_hbm(per_kernel, algorithmic_bytes(int(pc._xyz.shape[0]), V, K, W, H,
                                                                  (min(D, 3) + 1) ** 2, adam_fused=adam_fused),
                                    f"cfg{args.config}-step")
        if dom in mfma_flops(1):   # the deformation network's training call (--with-mlp): the matrix cores
            roof = mfma_roofline(dom, per_kernel[dom], mfma_flops(int(pc._xyz.shape[0]))[dom],
                                 f"cfg{args.config}+mlp")
        elif dom:
            # the kernel-timing pass's scene: V and K of its last view, P of that view (no densification in it)
            nbytes = algorithmic_bytes(int(pc._xyz.shape[0]), V, K, W, H, (min(D, 3) + 1) ** 2,
                                       adam_fused=adam_fused).get(dom)
            if nbytes:
                roof = roofline(dom, per_kernel[dom], nbytes, f"cfg{args.config}")
        cpu = None
        if args.cpu_baseline == "auto" and world == 1:   # rank 0 at N = 1 only; a bounded CPU sample
            cpu = cpu_baseline(cfg, args.config)
        res = {
            "metric": METRIC,
            "value": round(world * steps / elapsed, 3),
            "unit": "views/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"cfg{args.config}: {P} Gaussians, SH deg {D}, {W}x{H}, 1 view/GPU; "
                                   + ("per-Gaussian SE(3) deform (fused exp-map) + " if se3 else "")
                                   + ("MLP live: DirectTemporalNeRF offsets (iteration 5000) + " if net is not None
                                      else "")
                                   + "render fwd + 0.8 L1 + 0.2 (1 - SSIM)"
                                   + (" + 0.1 mean |offset|" if net is not None else "") + " + bwd"
                                   + (" + d_se3" if se3 else "")
                                   + (" + MLP bwd" if net is not None else "")
                                   + " + densification statistics + RCCL all-reduce of per-Gaussian grads + Adam"
                                   + (" (incl. the MLP's group)" if net is not None else "")
                                   + (f"; densify_and_prune every {densify_every} steps" if densify_every else ""),
                       "P": P, "width": W, "height": H, "sh_degree": D, "views_per_step": world,
                       "parallelism": f"dp{world}", "visible": V, "num_rendered": K,
                       "num_rendered_timed_first": K_start, "num_rendered_timed_last": K_end,
                       "densify_interval": densify_every or None, "deform_mlp": net is not None,
                       "P_timed_last": P_end},
            "fwd_bwd_ms_per_view": round(fwd_bwd_ms, 4),
            "fwd_bwd_ms_per_view_host_synced": round(fwd_bwd_synced_ms, 4),
            "kernels_ms": {k: round(v, 4) for k, v in per_kernel.items()},
            "kernel_launches_per_step": {k: round(n / n_timing_steps, 2) for k, (tot, n) in kt.items()},
            "kernels_hbm": kernel_hbm,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        res["step_path"] = "gsd_train_step (one native call)" if fused_step is not None else "drop-in API"
        if dropin is not None:
            res["dropin_api_step"] = dropin
        if exchange is not None:
            res["exchange"] = exchange
        if replicas is not None:
            res["replicas_identical"] = replicas
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        try:
            main()
        except SystemExit as e:   # a rank that stops early must not wait in teardown either
            if e.code is None:
                code = 0
            elif isinstance(e.code, int):
                code = e.code
            else:   # sys.exit("message"): print it as the interpreter would, status 1
                print(e.code, file=sys.stderr)
                code = 1
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(code)
        except BaseException:
            import traceback
            traceback.print_exc()
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(1)
    else:
        main()
