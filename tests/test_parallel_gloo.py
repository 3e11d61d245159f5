"""N>1 path on the CPU: world_size-2 gloo.  Each rank renders its own view
(one view per GPU in production) with the oracle, drops the per-Gaussian
gradients into the FlatGrads slab, and one all-reduce must give the sum of
the single-view gradients (SURVEY.md 8(e) parity)."""
from __future__ import annotations

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT, oracle_kwargs, scene_inputs

P, W, H, DEG = 400, 64, 48, 2


def view_grads(yaw):
    from oracle import oracle
    d = scene_inputs(P, W, H, DEG, seed=5, yaw=yaw)
    kw = oracle_kwargs(d)
    fwd = oracle.forward(d["means3D"].numpy(), kw["opacities"], shs=kw["shs"], scales=kw["scales"],
                         rotations=kw["rotations"], viewmatrix=kw["viewmatrix"], projmatrix=kw["projmatrix"],
                         campos=kw["campos"], W=W, H=H, tanfovx=kw["tanfovx"], tanfovy=kw["tanfovy"], sh_degree=DEG)
    dpix = np.random.default_rng(int(yaw * 10)).standard_normal((3, H, W)).astype(np.float32)
    b = oracle.backward(fwd, dpix, d["means3D"].numpy(), shs=kw["shs"], scales=kw["scales"],
                        rotations=kw["rotations"], viewmatrix=kw["viewmatrix"], projmatrix=kw["projmatrix"],
                        campos=kw["campos"], W=W, H=H, tanfovx=kw["tanfovx"], tanfovy=kw["tanfovy"], sh_degree=DEG)
    return [b["dL_dmeans3D"], b["dL_dsh"], b["dL_dopacity"], b["dL_dscales"], b["dL_drotations"]]


def _worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd.parallel import FlatGrads, init_from_env
    r, _, w = init_from_env(backend="gloo")
    grads = view_grads(yaw=2.0 * r)                      # one view per rank, yaw offsets k*2 deg
    params = [torch.nn.Parameter(torch.zeros(g.shape)) for g in grads]
    fg = FlatGrads(params, device="cpu")
    for p, g in zip(params, grads):
        p.grad.copy_(torch.from_numpy(g))
    fg.allreduce()
    np.save(os.path.join(out_dir, f"rank{r}.npy"), fg.slab.numpy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_rank_gradient_allreduce_equals_sum_of_views(tmp_path):
    from oracle import oracle
    oracle.build()
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = sum(np.concatenate([g.reshape(-1) for g in view_grads(2.0 * r)]) for r in range(world))
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)


def _worker_sh_views(rank, world, port, out_dir):
    """The data-parallel protocol of the per-view SH exchange: each rank holds the all-view SH gradient (what
    gsd_sh_grad_views assembles from the gathered dL/dRGB rows -- emulated here from the oracle's per-view SH
    gradients after an all_gather), marks it reduced, and FlatGrads.allreduce sums only the other gradients
    (two contiguous runs around the SH view)."""
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd.parallel import FlatGrads, init_from_env, mark_reduced
    r, _, w = init_from_env(backend="gloo")
    grads = view_grads(yaw=2.0 * r)
    params = [torch.nn.Parameter(torch.zeros(g.shape)) for g in grads]
    fg = FlatGrads(params, device="cpu")
    fg.invalidate()
    sh_mine = torch.from_numpy(grads[1]).contiguous()
    parts = [torch.empty_like(sh_mine) for _ in range(w)]
    dist.all_gather(parts, sh_mine)
    for i, (p, g) in enumerate(zip(params, grads)):
        assert fg.claim([p]) is False
        p.grad.copy_(sum(parts) if i == 1 else torch.from_numpy(g))
    mark_reduced([params[1]])
    fg.allreduce()
    assert not fg.reduced
    np.save(os.path.join(out_dir, f"rank{r}.npy"), fg.slab.numpy())
    dist.destroy_process_group()


def test_two_rank_sh_views_protocol(tmp_path):
    from oracle import oracle
    oracle.build()
    world = 2
    mp.spawn(_worker_sh_views, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = sum(np.concatenate([g.reshape(-1) for g in view_grads(2.0 * r)]) for r in range(world))
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)


def _worker_buckets(rank, world, port, out_dir):
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd.parallel import FlatGrads, init_from_env, mark_reduced
    r, _, w = init_from_env(backend="gloo")
    grads = view_grads(yaw=2.0 * r)
    params = [torch.nn.Parameter(torch.zeros(g.shape)) for g in grads]
    fg = FlatGrads(params, device="cpu")
    for p, g in zip(params, grads):
        p.grad.copy_(torch.from_numpy(g))
    # the SH gradient (params[1]) stands for one the ranks already summed (the per-view exchange): every rank
    # holds the sum, and the bucketed all-reduce must leave it alone
    total_sh = torch.zeros_like(params[1].grad)
    for k in range(w):
        total_sh += torch.from_numpy(view_grads(yaw=2.0 * k)[1])
    params[1].grad.copy_(total_sh)
    mark_reduced([params[1]])
    ranges = fg.allreduce_buckets(bucket_floats=1000)    # several buckets per run, a partial one at each end
    covered = 0
    for a, b, work in ranges:
        assert a == covered and b > a
        covered = b
        if work is not None:
            work.wait()
    assert covered == fg.slab.numel()
    np.save(os.path.join(out_dir, f"brank{r}.npy"), fg.slab.numpy())
    dist.destroy_process_group()


def test_four_rank_bucketed_allreduce_equals_sum_of_views(tmp_path):
    """FlatGrads.allreduce_buckets (the asynchronous, bucketed all-reduce FusedAdam.allreduce_step overlaps with
    Adam) over four gloo ranks: the slab ranges cover it in order, and every rank ends with the sum of the four
    single-view oracle gradients -- including the range marked as already summed, which it must not re-add."""
    world = 4
    mp.spawn(_worker_buckets, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = sum(np.concatenate([g.reshape(-1) for g in view_grads(2.0 * r)]) for r in range(world))
    for r in range(world):
        got = np.load(os.path.join(str(tmp_path), f"brank{r}.npy"))
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)
