"""N>1 path on the CPU: world_size-2 gloo.  Each rank renders its own view
(one view per GPU in production) with the oracle, drops the per-Gaussian
gradients into the FlatGrads slab, and one all-reduce must give the sum of
the single-view gradients (SURVEY.md 8(e) parity)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
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


def _teardown(rank, world, out_dir):
    """End a worker whose results are already on disk without running gloo's or the TCP store's destructors: a
    barrier, then every rank but 0 says so through a file and leaves with os._exit(0), and rank 0 (which hosts the
    TCP store) leaves the same way once all have.  Destroying the groups (at once, or peers first and rank 0 last)
    now and then aborted a rank in a destructor under load ("terminate called without an active exception",
    SIGABRT), which mp.spawn reports as a failed test although every result was written."""
    import sys
    import time
    dist.barrier()
    sys.stdout.flush()
    sys.stderr.flush()
    if rank != 0:
        open(os.path.join(out_dir, ".down%d" % rank), "w").close()
        os._exit(0)
    deadline = time.time() + 60
    while time.time() < deadline and not all(os.path.exists(os.path.join(out_dir, ".down%d" % r))
                                             for r in range(1, world)):
        time.sleep(0.01)
    os._exit(0)


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
    _teardown(rank, world, out_dir)


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
    _teardown(rank, world, out_dir)


def test_two_rank_sh_views_protocol(tmp_path):
    from oracle import oracle
    oracle.build()
    world = 2
    mp.spawn(_worker_sh_views, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = sum(np.concatenate([g.reshape(-1) for g in view_grads(2.0 * r)]) for r in range(world))
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)


def _worker_buckets(rank, world, port, out_dir, early=False):
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
    if early:   # the raw parameters' all-reduce started inside the backward (FusedAdam.reduce_early)
        fg.early_allreduce([params[2], params[0]], bucket_floats=700)
        try:    # a second producer for an early-reduced gradient would miss the sum: refused
            fg.claim([params[0]])
            raise AssertionError("claim of an early-reduced parameter did not raise")
        except RuntimeError:
            pass
    ranges = fg.allreduce_buckets(bucket_floats=1000)    # several buckets per run, a partial one at each end
    assert not fg.early and not fg.early_ids
    covered = 0
    for a, b, work in ranges:
        assert a == covered and b > a
        covered = b
        if work is not None:
            work.wait()
    assert covered == fg.slab.numel()
    np.save(os.path.join(out_dir, f"{'e' if early else 'b'}rank{r}.npy"), fg.slab.numpy())
    _teardown(rank, world, out_dir)


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


def test_four_rank_early_allreduce_then_buckets(tmp_path):
    """FlatGrads.early_allreduce (issued inside the data-parallel backward for the raw parameters, then handed
    to allreduce_buckets) over four gloo ranks: two non-adjacent parameters go out early in their own buckets,
    the rest in allreduce_buckets' -- every element summed exactly once, the ranges covering the slab in order,
    and a second producer of an early-reduced gradient refused."""
    world = 4
    mp.spawn(_worker_buckets, args=(world, _free_port(), str(tmp_path), True), nprocs=world, join=True)
    want = sum(np.concatenate([g.reshape(-1) for g in view_grads(2.0 * r)]) for r in range(world))
    for r in range(world):
        got = np.load(os.path.join(str(tmp_path), f"erank{r}.npy"))
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)


class _SlabOpt:
    """Stand-in for FusedAdam's slab surgery interface (param_groups, moments, rebuild) on CPU tensors."""

    def __init__(self, params):
        self.param_groups = [{"params": [p]} for p in params]
        self.m = {id(p): torch.full_like(p, 0.5) for p in params}
        self.v = {id(p): torch.full_like(p, 0.25) for p in params}

    def moments(self, p):
        return self.m[id(p)], self.v[id(p)]

    def rebuild(self, datas, ms, vs):
        ps = [g["params"][0] for g in self.param_groups]
        self.m, self.v = {}, {}
        for p, d, m, v in zip(ps, datas, ms, vs):
            p.data = d.clone()
            self.m[id(p)], self.v[id(p)] = m.clone(), v.clone()


def _densify_model(P=300):
    from gsd_amd import DeformableGaussians
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.scene import make_gaussians
    pc = DeformableGaussians(make_gaussians(P, 64, 48, seed=3), sh_degree=3)
    ps = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
    with torch.no_grad():   # a spread of scales so that both clone and split select points
        pc._scaling.add_(torch.linspace(-2.0, 1.5, P)[:, None])
    return pc, ps, GaussianDensifier(pc, _SlabOpt(ps))


def _rank_stats(r, P):
    """Rank r's own-view statistics (as add_densification_stats leaves them): different visibility, gradient
    norms and radii per rank."""
    g = torch.Generator().manual_seed(100 + r)
    vis = torch.rand(P, generator=g) < 0.7
    return (vis.float()[:, None], (torch.rand(P, 1, generator=g) * 4e-4) * vis[:, None],
            torch.randint(0, 40, (P,), generator=g).float() * vis, torch.randn(P, 3, generator=g) * vis[:, None])


def _worker_densify(rank, world, port, out_dir):
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd.parallel import init_from_env
    r, _, w = init_from_env(backend="gloo")
    pc, ps, dens = _densify_model()
    dens.denom, dens.xyz_gradient_accum, dens.max_radii2D, dens.xyz_gradient_accum_3vec = _rank_stats(r, 300)
    torch.manual_seed(1000 + r)   # different generators per rank: the split samples must come from rank 0
    dens.densify_and_prune(2e-4, 0.005, 2.0, 30)
    np.savez(os.path.join(out_dir, f"dens{r}.npz"), *[p.detach().numpy() for p in ps])
    _teardown(rank, world, out_dir)


def test_two_rank_densify_keeps_replicas_identical(tmp_path):
    """Data-parallel densify_and_prune (2 ranks, gloo): each rank holds only its own view's statistics and its
    own random generator; both must end with identical parameters, equal to one process holding the combined
    statistics (sums; max of the radii) and rank 0's generator."""
    world = 2
    mp.spawn(_worker_densify, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [np.load(tmp_path / f"dens{r}.npz") for r in range(world)]
    pc, ps, dens = _densify_model()
    st = [_rank_stats(r, 300) for r in range(world)]
    dens.denom = st[0][0] + st[1][0]
    dens.xyz_gradient_accum = st[0][1] + st[1][1]
    dens.max_radii2D = torch.maximum(st[0][2], st[1][2])
    dens.xyz_gradient_accum_3vec = st[0][3] + st[1][3]
    torch.manual_seed(1000)
    dens.densify_and_prune(2e-4, 0.005, 2.0, 30)
    assert ps[0].shape[0] != 300   # the scene changed (clone / split / prune all ran)
    for i, p in enumerate(ps):
        a0, a1 = got[0][f"arr_{i}"], got[1][f"arr_{i}"]
        assert np.array_equal(a0, a1), i
        np.testing.assert_allclose(a0, p.detach().numpy(), rtol=1e-6, atol=1e-7)


def _worker_addend(rank, world, port, out_dir):
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd.parallel import FlatGrads, init_from_env
    r, _, w = init_from_env(backend="gloo")
    grads = view_grads(yaw=2.0 * r)
    params = [torch.nn.Parameter(torch.zeros(g.shape)) for g in grads]
    fg = FlatGrads(params, device="cpu")
    addend = torch.from_numpy(np.random.default_rng(3).standard_normal(grads[0].shape).astype(np.float32))
    for sync in (True, False):
        for p, g in zip(params, grads):
            p.grad.copy_(torch.from_numpy(g))
        fg.add_after_reduce(params[0], addend.clone())   # the same all-rank total on every rank
        try:
            fg.add_after_reduce(params[0], addend.clone())
            raise AssertionError("a second addend for one parameter did not raise")
        except RuntimeError:
            pass
        if sync:   # allreduce adds it once, after the sum
            fg.allreduce()
            np.save(os.path.join(out_dir, f"arank{r}.npy"), fg.slab.numpy())
        else:      # allreduce_buckets leaves it to the consumer (FusedAdam passes it to its Adam pass)
            for _, _, wk in fg.allreduce_buckets(bucket_floats=500):
                if wk is not None:
                    wk.wait()
            (a, b, t), = fg.addend_ranges()
            assert (a, b) == (0, params[0].numel()) and fg.addends == {}
            np.save(os.path.join(out_dir, f"brank{r}.npy"), fg.slab.numpy())
    _teardown(rank, world, out_dir)


def test_two_rank_addend_joins_after_the_sum(tmp_path):
    """FlatGrads.add_after_reduce (the exchanged views' summed mean term, already an all-rank total): the
    synchronous allreduce adds it once after summing the ranks' own gradients; allreduce_buckets sums the
    ranks' parts only and hands the addend's slab range to its consumer."""
    world = 2
    mp.spawn(_worker_addend, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    views = [np.concatenate([g.reshape(-1) for g in view_grads(2.0 * r)]) for r in range(world)]
    plain = sum(views)
    addend = np.random.default_rng(3).standard_normal(view_grads(0.0)[0].shape).astype(np.float32).reshape(-1)
    with_add = plain.copy()
    with_add[:addend.size] += addend
    for r in range(world):
        np.testing.assert_allclose(np.load(os.path.join(str(tmp_path), f"arank{r}.npy")), with_add, rtol=1e-5,
                                   atol=1e-6)
        np.testing.assert_allclose(np.load(os.path.join(str(tmp_path), f"brank{r}.npy")), plain, rtol=1e-5,
                                   atol=1e-6)


def test_single_pass_densify_equals_clone_split_prune():
    """GaussianDensifier.densify_and_prune assembles the reference's result in one optimizer-state surgery; it
    must equal the reference's own sequence -- densify_and_clone, densify_and_split (same torch.normal draw),
    then the opacity / world-size prune over the statistics the postfix reset -- point for point, moments
    included (CPU, the slab stand-in)."""
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    outs = []
    for single in (True, False):
        pc, ps, dens = _densify_model()
        with torch.no_grad():
            pc._opacity[::7] = -8.0   # some points below the prune threshold
        dens.denom, dens.xyz_gradient_accum, dens.max_radii2D, dens.xyz_gradient_accum_3vec = _rank_stats(0, 300)
        for p in ps:   # distinct moments per point, so the row bookkeeping shows
            m, v = dens.opt.moments(p)
            m.copy_(torch.arange(p.numel(), dtype=torch.float32).reshape(p.shape))
            v.copy_(m * 0.5)
        torch.manual_seed(77)
        if single:
            dens.densify_and_prune(2e-4, 0.005, 2.0, 30)
        else:   # gaussian_model.py:1219-1233 step by step
            grads = dens.xyz_gradient_accum / dens.denom
            grads[grads.isnan()] = 0.0
            dens.densify_and_clone(grads, 2e-4, 2.0)
            dens.densify_and_split(grads, 2e-4, 2.0)
            with torch.no_grad():
                prune = (pc.get_opacity < 0.005).squeeze()
                big_vs = dens.max_radii2D > 30
                big_ws = pc.get_scaling.max(dim=1).values > 0.1 * 2.0
                prune = torch.logical_or(torch.logical_or(prune, big_vs), big_ws)
            dens.prune_points(prune)
        outs.append(([p.detach().clone() for p in ps], [torch.cat([t.reshape(-1) for t in dens.opt.moments(p)])
                                                        for p in ps]))
    (pa, ma), (pb, mb) = outs
    assert pa[0].shape[0] not in (300,) and pa[0].shape == pb[0].shape
    for a, b in zip(pa + ma, pb + mb):
        assert torch.equal(a, b)


def _worker_divergent(rank, world, port, out_dir):
    """Ranks whose slabs disagree -- a different Gaussian count (a densification that ran on one rank only), or a
    different bucket size -- must all raise at their first collective of the step (FlatGrads.verify_layout on
    the host-side signature exchange), not enter collectives of different sizes and hang."""
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd import parallel
    from gsd_amd.parallel import FlatGrads, init_from_env
    r, _, w = init_from_env(backend="gloo")
    msgs = []
    for case in ("P", "bucket", "same"):
        n = 100 + (r if case == "P" else 0)
        parallel.BUCKET_FLOATS = 1 << (10 + (r if case == "bucket" else 0))
        params = [torch.nn.Parameter(torch.zeros(n, 3)), torch.nn.Parameter(torch.zeros(n, 1))]
        fg = FlatGrads(params, device="cpu")
        fg.invalidate()            # the start of a step: posts the layout check
        for p in params:
            p.grad.fill_(1.0)
        try:
            for _, _, wk in fg.allreduce_buckets(parallel.BUCKET_FLOATS):
                if wk is not None:
                    wk.wait()
            msgs.append(f"{case}: ok {float(fg.slab.sum()):.1f}")
        except RuntimeError as e:
            msgs.append(f"{case}: raised {'differ' in str(e)}")
    with open(os.path.join(out_dir, f"rank{r}.txt"), "w") as fh:
        fh.write("\n".join(msgs))
    _teardown(rank, world, out_dir)


def test_rank_divergent_layouts_raise_on_every_rank(tmp_path):
    world = 2
    mp.spawn(_worker_divergent, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        got = (tmp_path / f"rank{r}.txt").read_text().splitlines()
        assert got == ["P: raised True", "bucket: raised True", "same: ok 800.0"], (r, got)


def _worker_one_rank_rebuilds(rank, world, port, out_dir):
    """a densification that runs on one rank only (FusedAdam.rebuild -> FlatGrads.successor) between
    steps.  The next step's forward posts the layout check (rasterizer._post_layout_checks) with the new layout on
    that rank and the old one elsewhere, so every rank raises at its first collective -- and because each rank
    makes exactly one exchange per step, the signature group's collectives stay paired: a following step where
    both ranks rebuilt alike passes.  The same without a forward post (verify_layout's synchronous exchange)."""
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd import parallel
    from gsd_amd.parallel import FlatGrads, init_from_env
    from gsd_amd.rasterizer import _post_layout_checks
    r, _, w = init_from_env(backend="gloo")
    parallel.BUCKET_FLOATS = 1 << 10
    params = [torch.nn.Parameter(torch.zeros(100, 3)), torch.nn.Parameter(torch.zeros(100, 1))]
    fg = FlatGrads(params, device="cpu")
    msgs = []

    def run(fg, forward_post, tag):
        if forward_post:
            _post_layout_checks(*fg.params)
        for p in fg.params:
            p.grad.fill_(1.0)
        try:
            for _, _, wk in fg.allreduce_buckets(parallel.BUCKET_FLOATS):
                if wk is not None:
                    wk.wait()
            msgs.append(f"{tag}: ok {float(fg.slab.sum()):.1f}")
        except RuntimeError as e:
            msgs.append(f"{tag}: raised {'differ' in str(e)}")
        fg.invalidate()            # the step's end (FusedAdam marks the slab stale)

    for forward_post in (True, False):
        run(fg, forward_post, f"same{int(forward_post)}")
        if r == 1:                 # densify on rank 1 only: fewer Gaussians
            params = [torch.nn.Parameter(torch.zeros(90, 3)), torch.nn.Parameter(torch.zeros(90, 1))]
            fg = fg.successor(params, device="cpu")
        run(fg, forward_post, f"diverged{int(forward_post)}")
        if r == 0:                 # rank 0 catches up: the layouts agree again
            params = [torch.nn.Parameter(torch.zeros(90, 3)), torch.nn.Parameter(torch.zeros(90, 1))]
            fg = fg.successor(params, device="cpu")
        run(fg, forward_post, f"agreed{int(forward_post)}")
        params = [torch.nn.Parameter(torch.zeros(100, 3)), torch.nn.Parameter(torch.zeros(100, 1))]
        fg = fg.successor(params, device="cpu")
    with open(os.path.join(out_dir, f"rank{r}.txt"), "w") as fh:
        fh.write("\n".join(msgs))
    _teardown(rank, world, out_dir)


def test_one_rank_densify_raises_on_every_rank_and_stays_paired(tmp_path):
    world = 2
    mp.spawn(_worker_one_rank_rebuilds, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = []
    for fp in (1, 0):
        want += [f"same{fp}: ok 800.0", f"diverged{fp}: raised True", f"agreed{fp}: ok 720.0"]
    for r in range(world):
        got = (tmp_path / f"rank{r}.txt").read_text().splitlines()
        assert got == want, (r, got)


def _view_grads_at(params, yaw):
    """The oracle's per-view gradients at the current parameters (activated means / SH / opacity / scales /
    rotations), plus this view's masked dL/dRGB row and camera centre -- what the rasterizer backward hands the
    SH-view exchange (gsd_sh_split.d_rgb)."""
    from gsd_amd.camera import synthetic_camera
    from oracle import oracle
    xyz, sh, op, sc, rot = (p.detach().numpy() for p in params)
    cam = synthetic_camera(W, H, yaw_deg=yaw)
    kw = dict(shs=sh, scales=sc, rotations=rot, viewmatrix=cam.world_view_transform.numpy(),
              projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(), W=W, H=H,
              tanfovx=float(np.tan(cam.FoVx * 0.5)), tanfovy=float(np.tan(cam.FoVy * 0.5)), sh_degree=DEG)
    fwd = oracle.forward(xyz, op, **kw)
    dpix = np.random.default_rng(int(yaw * 10) + 1).standard_normal((3, H, W)).astype(np.float32)
    b = oracle.backward(fwd, dpix, xyz, **kw)
    row = b["dL_dcolors"].reshape(P, 3) * (1 - fwd["clamped"].reshape(P, 3))
    return b, row.astype(np.float32), cam.camera_center.numpy().astype(np.float32)


def _assemble_sh(xyz, sh_shape, rows, campos):
    """sum_v B(dir_v) (x) dL/dRGB_v (backward.cu:20-139 per view, summed) -- a float64 restatement of
    gsd_sh_grad_views: the SH colour is linear in the coefficients, so autograd of it gives the basis."""
    from oracle.torch_ref import sh_rgb
    x = torch.from_numpy(xyz).double()
    total = torch.zeros(sh_shape, dtype=torch.float64)
    for row, c in zip(rows, campos):
        d = x - torch.from_numpy(c).double()
        sh = torch.zeros(sh_shape, dtype=torch.float64, requires_grad=True)
        (sh_rgb(DEG, sh, d / d.norm(dim=1, keepdim=True)) * torch.from_numpy(row).double()).sum().backward()
        total += sh.grad
    return total.float()


def _worker_eight(rank, world, port, out_dir, sh_views):
    """SURVEY.md 8(e) at cfg4's shape: 8 ranks, one view each (yaw k * 2 deg), three data-parallel steps of the
    bench's protocol -- the SH gradient assembled from the all-gathered per-view dL/dRGB rows (sh_views) or
    all-reduced with the rest, the raw parameters' early all-reduce, the bucketed all-reduce of the remainder,
    and an identical Adam step on every rank.  Saves the first step's assembled gradient slab and a checksum of
    the parameters after the three steps."""
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gsd_amd import parallel
    from gsd_amd.parallel import FlatGrads, init_from_env, mark_reduced
    from gsd_amd.rasterizer import _post_layout_checks
    from oracle import oracle
    oracle.set_threads(1)
    r, _, w = init_from_env(backend="gloo")
    parallel.SH_VIEWS = bool(sh_views)
    d = scene_inputs(P, W, H, DEG, seed=5)
    params = [torch.nn.Parameter(d[k].clone().contiguous()) for k in
              ("means3D", "shs", "opacities", "scales", "rotations")]
    fg = FlatGrads(params, device="cpu")
    opt = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(params, (1e-4, 2.5e-3, 5e-2, 5e-3, 1e-3))],
                           eps=1e-15)
    for it in range(3):
        fg.invalidate()
        b, row, campos = _view_grads_at(params, 2.0 * r)
        grads = [b["dL_dmeans3D"], b["dL_dsh"], b["dL_dopacity"], b["dL_dscales"], b["dL_drotations"]]
        _post_layout_checks(*params)                    # the forward's layout check
        for i, (p, g) in enumerate(zip(params, grads)):
            if i == 1 and sh_views:
                continue
            assert fg.claim([p]) is False               # store mode: the first producer of the step
            p.grad.copy_(torch.from_numpy(g).reshape(p.shape))
        if sh_views:   # the row exchange: every rank assembles the all-view SH gradient itself
            fg.verify_layout()
            mine = torch.from_numpy(np.concatenate([row.reshape(-1), campos]))
            parts = [torch.empty_like(mine) for _ in range(w)]
            dist.all_gather(parts, mine)
            rows = [q[:3 * P].numpy().reshape(P, 3) for q in parts]
            cams = [q[3 * P:].numpy() for q in parts]
            assert fg.claim([params[1]]) is False
            params[1].grad.copy_(_assemble_sh(params[0].detach().numpy(), tuple(params[1].shape), rows, cams))
            mark_reduced([params[1]])
        fg.early_allreduce([params[0], params[2]], bucket_floats=700)   # the raw parameters, inside the backward
        for a, bb, work in fg.allreduce_buckets(bucket_floats=900):
            if work is not None:
                work.wait()
        if it == 0:
            np.save(os.path.join(out_dir, f"{sh_views}grad{r}.npy"), fg.slab.numpy().copy())
        opt.step()
    ck = np.concatenate([p.detach().numpy().reshape(-1) for p in params]).view(np.uint32).astype(np.uint64).sum()
    with open(os.path.join(out_dir, f"{sh_views}ck{r}.txt"), "w") as fh:
        fh.write(str(int(ck)))
    _teardown(rank, world, out_dir)


def _eight_rank(tmp_path, sh_views):
    from oracle import oracle
    oracle.build()
    world = 8
    mp.spawn(_worker_eight, args=(world, _free_port(), str(tmp_path), sh_views), nprocs=world, join=True)
    d = scene_inputs(P, W, H, DEG, seed=5)
    params = [d[k].clone().contiguous() for k in ("means3D", "shs", "opacities", "scales", "rotations")]
    want = 0
    for k in range(world):
        b, _, _ = _view_grads_at(params, 2.0 * k)
        want = want + np.concatenate([b[n].reshape(-1) for n in ("dL_dmeans3D", "dL_dsh", "dL_dopacity",
                                                                 "dL_dscales", "dL_drotations")]).astype(np.float64)
    got = [np.load(tmp_path / f"{sh_views}grad{r}.npy") for r in range(world)]
    for r in range(world):   # every rank holds the sum of the eight single-view oracle gradients
        np.testing.assert_allclose(got[r], want, rtol=1e-5, atol=1e-6 * np.abs(want).max())
    cks = {(tmp_path / f"{sh_views}ck{r}.txt").read_text() for r in range(world)}
    assert len(cks) == 1, cks   # replicas bit-identical after three steps


def test_eight_rank_sh_view_exchange_matches_sum_of_views(tmp_path):
    _eight_rank(tmp_path, 1)


def test_eight_rank_plain_allreduce_matches_sum_of_views(tmp_path):
    _eight_rank(tmp_path, 0)


def _worker_fail(rank, world, port, out_dir, mode):
    """Three all-reduce steps; rank 2 exits (mode "exit") or hangs ("hang") before its second step.  A surviving
    rank whose collective raises records the time and exits with status 17."""
    import sys
    import time
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GSD_DIST_TIMEOUT_S="6")
    from gsd_amd.parallel import FlatGrads, init_from_env
    r, _, w = init_from_env(backend="gloo")
    params = [torch.nn.Parameter(torch.zeros(1000)), torch.nn.Parameter(torch.zeros(7, 3))]
    fg = FlatGrads(params, device="cpu")
    t0 = None
    try:
        for step in range(3):
            if step == 1 and r == 2:
                if mode == "exit":
                    os._exit(3)
                time.sleep(3600)
            t0 = time.time()
            for p in params:
                p.grad.fill_(1.0)
            fg.allreduce()
    except Exception as e:   # the peer's failure, seen by this rank's collective
        with open(os.path.join(out_dir, f"err{r}.txt"), "w") as f:
            f.write(f"{time.time() - t0:.3f} {type(e).__name__}: {e}"[:2000])
        os._exit(17)
    os._exit(0)


@pytest.mark.parametrize("mode", ["exit", "hang"])
def test_failed_rank_ends_its_peers_within_the_timeout(tmp_path, mode):
    """Failure bound of the N > 1 path (parallel.DIST_TIMEOUT_S): of four gloo ranks one exits, or hangs, in the
    middle of the step sequence; the three others must leave their collective with an error and exit non-zero
    within the timeout (6 s here) plus a margin, instead of waiting in it for torch's default 30 minutes."""
    import time
    ctx = mp.get_context("spawn")
    world, port = 4, _free_port()
    procs = [ctx.Process(target=_worker_fail, args=(r, world, port, str(tmp_path), mode)) for r in range(world)]
    t0 = time.time()
    for p in procs:
        p.start()
    try:
        for r, p in enumerate(procs):
            if r != 2:
                p.join(timeout=max(1.0, 60.0 - (time.time() - t0)))
        for r, p in enumerate(procs):
            if r == 2:
                continue
            assert p.exitcode == 17, (r, p.exitcode)
            elapsed = float((tmp_path / f"err{r}.txt").read_text().split()[0])
            assert elapsed <= 6.0 + 10.0, (r, (tmp_path / f"err{r}.txt").read_text())
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
            p.join(timeout=10)
