"""Two data-parallel ranks on one GPU (gloo through host memory, 2 processes): one render + backward per rank,
then FlatGrads.allreduce.  The SH gradient takes the per-view exchange path (rasterizer._backward_sh_views: the
ranks all-gather masked dL/dRGB rows and each runs gsd_sh_grad_views); the rest is all-reduced.  Both ranks'
slabs must equal one process accumulating both views."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu

WORKER = r'''
import os, sys
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch, torch.distributed as dist
from gsd_amd import DeformableGaussians, default_pipe, render
from gsd_amd.camera import synthetic_camera
from gsd_amd.parallel import FlatGrads
from gsd_amd.scene import make_gaussians

def step(pc, yaw):
    cam = synthetic_camera(320, 240, yaw_deg=yaw).to("cuda:0")
    out = render(cam, pc, default_pipe(), torch.zeros(3, device="cuda:0"))
    w = torch.linspace(0.5, 1.5, 320, device="cuda:0")
    (out["render"] * w).sum().backward()

rank, world, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
torch.cuda.set_device(0)
params = make_gaussians(20_000, 320, 240, seed=21, device="cuda:0")
pc = DeformableGaussians(params, sh_degree=3)
flat = FlatGrads(pc.parameters())
flat.slab.fill_(7.0)
flat.invalidate()
if rank >= 0:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[4], RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    step(pc, 4.0 * rank)
    flat.allreduce()
    dist.barrier()   # no rank tears the group down while a peer's last exchange is still in flight
    dist.destroy_process_group()
else:                      # the single-process reference: both views into one slab
    for r in range(world):
        step(pc, 4.0 * r)
    flat.allreduce()
torch.save(flat.slab.cpu(), out)
'''


def test_two_ranks_match_one_process(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text("ROOT = %r\n" % ROOT + WORKER)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    port = str(29600 + os.getpid() % 200)
    procs = [subprocess.Popen([sys.executable, str(script), str(r), "2", str(tmp_path / f"r{r}.pt"), port], env=env)
             for r in range(2)]
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0, 0]
    ref = subprocess.run([sys.executable, str(script), "-1", "2", str(tmp_path / "ref.pt"), port], env=env,
                         timeout=300)
    assert ref.returncode == 0
    want = torch.load(tmp_path / "ref.pt", weights_only=True)
    for r in range(2):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.isfinite(got).all()
        rel = float((got - want).norm() / want.norm())
        assert rel <= 1e-5, (r, rel)


WORKER_ADAM = r'''
import os, sys
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch, torch.distributed as dist
from gsd_amd import DeformableGaussians, default_pipe, render
from gsd_amd.camera import synthetic_camera
from gsd_amd.optim import FusedAdam
from gsd_amd.scene import make_gaussians

def step(pc, yaw):
    cam = synthetic_camera(320, 240, yaw_deg=yaw).to("cuda:0")
    out = render(cam, pc, default_pipe(), torch.zeros(3, device="cuda:0"))
    w = torch.linspace(0.5, 1.5, 320, device="cuda:0")
    (out["render"] * w).sum().backward()

rank, world, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
torch.cuda.set_device(0)
params = make_gaussians(20_000, 320, 240, seed=22, device="cuda:0")
pc = DeformableGaussians(params, sh_degree=3)
opt = FusedAdam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(pc.parameters())])
for it in range(2):
    if rank >= 0:
        if it == 0:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[4], RANK=str(rank), WORLD_SIZE=str(world))
            dist.init_process_group("gloo", rank=rank, world_size=world)
        if len(sys.argv) > 5 and sys.argv[5] == "fused":   # SH pieces stepped inside sh_grad_views
            with opt.step_in_backward():
                step(pc, 4.0 * rank + it)
        else:
            step(pc, 4.0 * rank + it)
            opt.allreduce_step(zero_grad=True, bucket_floats=50_000)   # several buckets, partial ones included
    else:                      # the single-process reference: both views into one slab, then a plain step
        for r in range(world):
            step(pc, 4.0 * r + it)
        opt.step(zero_grad=True)
if rank >= 0:
    dist.barrier()   # no rank tears the group down while a peer's last exchange is still in flight
    dist.destroy_process_group()
torch.save({"p": opt.param_slab.cpu(), "m": opt.exp_avg.cpu(), "v": opt.exp_avg_sq.cpu()}, out)
'''


@pytest.mark.parametrize("mode", ["plain", "fused"])
def test_two_ranks_overlapped_allreduce_adam_matches_one_process(tmp_path, mode):
    """FusedAdam.allreduce_step (bucketed asynchronous all-reduce, Adam per bucket as it arrives, the exchanged
    SH gradient first) over two gloo ranks == one process summing both views and taking a plain Adam step;
    two steps, so the second runs on moments the first left.  "fused": FusedAdam.step_in_backward, whose SH
    pieces take their Adam step inside gsd_sh_grad_views (the assembled gradient is final on every rank) and
    whose other parameters are all-reduced and stepped on leaving the block."""
    script = tmp_path / "worker_adam.py"
    script.write_text("ROOT = %r\n" % ROOT + WORKER_ADAM)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    port = str(29800 + os.getpid() % 150 + (7 if mode == "fused" else 0))
    procs = [subprocess.Popen([sys.executable, str(script), str(r), "2", str(tmp_path / f"a{r}.pt"), port, mode],
                              env=env) for r in range(2)]
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0, 0]
    ref = subprocess.run([sys.executable, str(script), "-1", "2", str(tmp_path / "aref.pt"), port], env=env,
                         timeout=300)
    assert ref.returncode == 0
    want = torch.load(tmp_path / "aref.pt", weights_only=True)
    for r in range(2):
        got = torch.load(tmp_path / f"a{r}.pt", weights_only=True)
        for k in ("m", "v"):   # the moments are (quadratic in) the summed gradients
            assert torch.isfinite(got[k]).all()
            rel = float((got[k] - want[k]).norm() / want[k].norm())
            assert rel <= 1e-5, (r, k, rel)
        # the parameters move by ~lr m / sqrt(v); only gradients within rounding of zero may flip a sign
        d = (got["p"] - want["p"]).abs()
        assert float(d.max()) <= 2 * 6e-3 + 1e-6
        assert float((d > 1e-6).float().mean()) <= 1e-4


WORKER_ONE_RANK = r'''
import os, sys
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch, torch.distributed as dist
from gsd_amd import DeformableGaussians, default_pipe, render
from gsd_amd.camera import synthetic_camera
from gsd_amd.optim import FusedAdam
from gsd_amd.parallel import dp_active, init_from_env
from gsd_amd.scene import make_gaussians

rank, local, world = init_from_env()
torch.cuda.set_device(0)
assert dp_active() == (os.environ.get("GSD_DP_ONE_RANK") == "1")
if dp_active():
    assert dist.get_backend() == "nccl" and world == 1
params = make_gaussians(20_000, 320, 240, seed=23, device="cuda:0")
pc = DeformableGaussians(params, sh_degree=3)
opt = FusedAdam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(pc.parameters())])
w = torch.linspace(0.5, 1.5, 320, device="cuda:0")
for it in range(3):
    cam = synthetic_camera(320, 240, yaw_deg=3.0 * it).to("cuda:0")
    with opt.step_in_backward():
        out = render(cam, pc, default_pipe(), torch.zeros(3, device="cuda:0"))
        (out["render"] * w).sum().backward()
torch.cuda.synchronize()
if dist.is_initialized():
    dist.barrier()   # no rank tears the group down while a peer's last exchange is still in flight
    dist.destroy_process_group()
torch.save({"p": opt.param_slab.cpu(), "m": opt.exp_avg.cpu(), "v": opt.exp_avg_sq.cpu()}, sys.argv[1])
'''


def test_one_rank_rccl_matches_single_process(tmp_path):
    """GSD_DP_ONE_RANK=1: a one-rank RCCL group takes the whole data-parallel path of bench.py's step -- the
    SH-view all_gather_into_tensor, gsd_sh_grad_views with the fused SH Adam, the early all-reduce of the raw
    parameters inside the backward and the bucketed allreduce_step on leaving the block -- with real RCCL
    collectives and their stream ordering, on one GPU.  Three steps must match the single-process path."""
    script = tmp_path / "worker_one.py"
    script.write_text("ROOT = %r\n" % ROOT + WORKER_ONE_RANK)
    port = str(29400 + os.getpid() % 150)
    base = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "GSD_DP_ONE_RANK")}
    env_dp = dict(base, HSA_ENABLE_IPC_MODE_LEGACY="0", GSD_DP_ONE_RANK="1", MASTER_ADDR="127.0.0.1",
                  MASTER_PORT=port, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r1 = subprocess.run([sys.executable, str(script), str(tmp_path / "dp.pt")], env=env_dp, timeout=300)
    assert r1.returncode == 0
    r2 = subprocess.run([sys.executable, str(script), str(tmp_path / "ref.pt")], env=dict(base), timeout=300)
    assert r2.returncode == 0
    got = torch.load(tmp_path / "dp.pt", weights_only=True)
    want = torch.load(tmp_path / "ref.pt", weights_only=True)
    for k in ("m", "v"):
        assert torch.isfinite(got[k]).all()
        rel = float((got[k] - want[k]).norm() / want[k].norm())
        assert rel <= 1e-5, (k, rel)
    d = (got["p"] - want["p"]).abs()
    assert float(d.max()) <= 2 * 1.8e-2 + 1e-6
    assert float((d > 1e-6).float().mean()) <= 1e-4


@pytest.mark.parametrize("sh_views", ["1", "0"])
def test_bench_gpus_2_spawns_two_ranks(sh_views):
    """``bench.py --gpus 2`` without a launcher starts torch.distributed.run with two ranks itself (here both on the
    one GPU, GSD_DIST_BACKEND=gloo: the rehearsal of the data-parallel path); rank 0 prints ONE JSON line with
    n_gpus 2, the data-parallel exchange timed alone, and value = 2 views per step over the max-over-ranks time.
    With the SH gradient exchanged as per-view rows (GSD_SH_VIEWS=1) and all-reduced whole (=0), the replicated
    parameters must be bit-identical on both ranks after the timed steps (bench.py's replicas_identical)."""
    import json
    env = dict(os.environ, GSD_DIST_BACKEND="gloo", GSD_SH_VIEWS=sh_views)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "2", "--steps",
                        "3", "--warmup", "1", "--cpu-baseline", "off"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2" and res["config"]["views_per_step"] == 2
    assert res["exchange"]["backend"] == "gloo" and res["exchange"]["allreduce_ms"] > 0
    assert res["value"] == pytest.approx(2 * 3 / (3 * res["ms_per_step"] / 1000.0), rel=1e-2)
    assert res["replicas_identical"] is True
