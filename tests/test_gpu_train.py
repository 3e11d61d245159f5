"""GPU parity of the training-step pieces around the rasterizer:
the fused loss (gsd_amd.loss, gsd_loss.hip) against the fp32 torch restatement of utils/loss_utils.py
(oracle/loss_ref.py, itself pinned to the reference's values in tests/test_oracle_golden.py) -- loss
value rel 1e-5, d loss / d image rel L2 1e-4 (separable vs 2-D window, different summation order) --
and the fused Adam step (gsd_amd.optim, gsd_adam.hip) against torch.optim.Adam -- 1e-6."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rel_l2(a, b):
    return float(torch.linalg.vector_norm(a - b) / max(float(torch.linalg.vector_norm(b)), 1e-30))


def test_loss_matches_reference_fixture():
    from gsd_amd.loss import l1_loss, ssim
    g = golden("loss.npz")
    x, y = torch.from_numpy(g["img1"]).to(DEV), torch.from_numpy(g["img2"]).to(DEV)
    assert abs(float(l1_loss(x, y)) - float(g["l1"])) <= 1e-6
    assert abs(float(ssim(x, y)) - float(g["ssim"])) <= 1e-5


@pytest.mark.parametrize("C,H,W,lam", [(3, 64, 96, 0.2), (3, 217, 333, 0.2), (1, 45, 31, 0.5), (3, 1080, 1920, 0.2)])
def test_l1_ssim_value_and_grad(C, H, W, lam):
    from gsd_amd.loss import l1_ssim_loss
    from oracle import loss_ref
    gen = torch.Generator().manual_seed(H * W + C)
    gt = torch.rand(C, H, W, generator=gen).to(DEV)
    base = (gt + 0.1 * torch.randn(C, H, W, generator=gen).to(DEV)).clamp(0, 1)
    x1 = base.clone().requires_grad_(True)
    x2 = base.clone().requires_grad_(True)
    got = l1_ssim_loss(x1, gt, lam)
    ref = loss_ref.l1_ssim_loss(x2, gt, lam)
    assert abs(float(got) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))
    got.backward()
    ref.backward()
    assert rel_l2(x1.grad, x2.grad) <= 1e-4


def test_loss_backward_scaled_and_composed():
    """The backward scales d loss / d img by autograd's incoming gradient inside the kernel: a weighted sum of
    l1_loss, ssim and l1_ssim_loss (train.py:529 written out by hand) against the restatement."""
    from gsd_amd.loss import l1_loss, l1_ssim_loss, ssim
    from oracle import loss_ref
    gen = torch.Generator().manual_seed(7)
    gt = torch.rand(3, 70, 90, generator=gen).to(DEV)
    base = (gt + 0.1 * torch.randn(3, 70, 90, generator=gen).to(DEV)).clamp(0, 1)
    x1 = base.clone().requires_grad_(True)
    x2 = base.clone().requires_grad_(True)
    (0.8 * l1_loss(x1, gt) + 0.2 * (1.0 - ssim(x1, gt)) - 2.5 * l1_ssim_loss(x1, gt, 0.3)).backward()
    (0.8 * loss_ref.l1_loss(x2, gt) + 0.2 * (1.0 - loss_ref.ssim(x2, gt))
     - 2.5 * loss_ref.l1_ssim_loss(x2, gt, 0.3)).backward()
    assert rel_l2(x1.grad, x2.grad) <= 1e-4


def test_identical_images_and_batched_input():
    from gsd_amd.loss import l1_ssim_loss, ssim
    x = torch.rand(1, 3, 50, 70, generator=torch.Generator().manual_seed(1)).to(DEV).requires_grad_(True)
    loss = l1_ssim_loss(x, x.detach(), 0.2)
    assert abs(float(loss)) <= 1e-6 and abs(float(ssim(x, x.detach())) - 1.0) <= 1e-6
    loss.backward()
    assert x.grad.shape == x.shape and float(x.grad.abs().max()) <= 1e-6  # sign(0) = 0, SSIM at its maximum


def test_loss_rejects_cpu_and_mismatch():
    from gsd_amd.loss import l1_ssim_loss
    with pytest.raises(RuntimeError):
        l1_ssim_loss(torch.rand(3, 8, 8), torch.rand(3, 8, 8))
    with pytest.raises(RuntimeError):
        l1_ssim_loss(torch.rand(3, 8, 8, device=DEV), torch.rand(3, 8, 9, device=DEV))


def test_fused_adam_matches_torch_adam():
    """gsd_amd.optim.FusedAdam vs torch.optim.Adam (foreach) with the reference's param groups (different
    learning rates, eps 1e-15), three steps, an lr change between steps (update_learning_rate)."""
    from gsd_amd.optim import FusedAdam
    gen = torch.Generator().manual_seed(5)
    shapes = [(1001, 3), (1001, 1, 3), (1001, 15, 3), (1001, 1), (1001, 3), (1001, 4)]
    lrs = [0.00016, 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]
    init = [torch.randn(*s, generator=gen) for s in shapes]
    grads = [[torch.randn(*s, generator=gen) * (10.0 ** -k) for s in shapes] for k in range(3)]
    a = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    b = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    opt_a = FusedAdam([{"params": [p], "lr": lr, "name": str(i)} for i, (p, lr) in enumerate(zip(a, lrs))],
                      lr=0.0, eps=1e-15)
    opt_b = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(b, lrs)], lr=0.0, eps=1e-15, foreach=True)
    for k in range(3):
        if k == 2:
            opt_a.param_groups[0]["lr"] = opt_b.param_groups[0]["lr"] = 1e-5
        for p, g in zip(a, grads[k]):
            p.grad.copy_(g.to(DEV))
        for p, g in zip(b, grads[k]):
            p.grad = g.to(DEV)
        opt_a.step(zero_grad=(k == 1))
        opt_b.step()
    for pa, pb in zip(a, b):
        assert pa.data_ptr() >= opt_a.param_slab.data_ptr()
        assert rel_l2(pa.detach(), pb.detach()) <= 1e-6
        assert float((pa - pb).abs().max()) <= 1e-6


def _adam_pair(seed=11):
    """Gaussian-like groups (one parameter each) plus an offset-network group holding several parameters
    (scene/gaussian_model.py:839-856 adds offset_model.parameters() as one group), as FusedAdam and as
    torch.optim.Adam (foreach)."""
    from gsd_amd.optim import FusedAdam
    gen = torch.Generator().manual_seed(seed)
    g_shapes = [(701, 3), (701, 15, 3), (701, 1)]
    n_shapes = [(32, 16), (32,), (3, 32)]
    lrs = [0.00016, 0.0025 / 20.0, 0.05]
    init = [torch.randn(*s, generator=gen) for s in g_shapes + n_shapes]
    a = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    b = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]

    def groups(ps):
        return ([{"params": [p], "lr": lr, "name": str(i)} for i, (p, lr) in enumerate(zip(ps[:3], lrs))] +
                [{"params": ps[3:], "lr": 8e-4, "name": "offset_model"}])
    opt_a = FusedAdam(groups(a), lr=0.0, eps=1e-15)
    opt_b = torch.optim.Adam(groups(b), lr=0.0, eps=1e-15, foreach=True)
    return a, b, opt_a, opt_b, gen


def _adam_backward(ps, ws, with_net):
    """A loss linear in every Gaussian parameter and, when ``with_net``, in the network's (autograd producers
    only: without it the network's parameters get no gradient at all -- grad None in torch)."""
    n = len(ps) if with_net else 3
    sum((p * w).sum() for p, w in zip(ps[:n], ws[:n])).backward()


def test_fused_adam_skips_parameters_without_grad():
    """torch.optim.Adam skips a parameter whose grad is None and keeps state['step'] per parameter: the
    offset-network group gets no gradient for its first 4 steps (the reference's DirectTemporalNeRF returns zeros
    before iteration 3000), then its first real update uses step 1's bias corrections.  FusedAdam must leave
    those parameters and moments untouched while they get nothing and then match torch step for step (also
    through allreduce_step, its data-parallel entry, at world size 1)."""
    a, b, opt_a, opt_b, gen = _adam_pair()
    for k in range(7):
        ws = [torch.randn(p.shape, generator=gen).to(DEV) * (10.0 ** -(k % 3)) for p in a]
        with_net = k >= 4
        _adam_backward(a, ws, with_net)
        _adam_backward(b, ws, with_net)
        if k % 2:
            opt_a.allreduce_step(zero_grad=True)
        else:
            opt_a.step(zero_grad=True)
        opt_b.step()
        opt_b.zero_grad(set_to_none=True)
        for i, (pa, pb) in enumerate(zip(a, b)):
            st = opt_b.state.get(pb)
            assert opt_a.steps[i] == (int(st["step"]) if st else 0), (k, i)
            assert float((pa - pb).abs().max()) <= 1e-6 * max(1.0, float(pb.abs().max())), (k, i)
            if st:
                ma, va = opt_a.moments(pa)
                # torch's foreach kernels may contract to FMA: moments agree to float rounding (rel 1e-6)
                assert float((ma - st["exp_avg"]).abs().max()) <= 1e-6 * float(st["exp_avg"].abs().max())
                assert float((va - st["exp_avg_sq"]).abs().max()) <= 1e-6 * float(st["exp_avg_sq"].abs().max())
        if not with_net:
            for pa in a[3:]:
                assert all(float(m.abs().max()) == 0.0 for m in opt_a.moments(pa))
    assert opt_a.steps == [7, 7, 7, 3, 3, 3]


def test_checkpoint_roundtrip_multi_parameter_group(tmp_path):
    """gsd_amd.io.capture / restore with the offset network's multi-parameter group (nonzero moments, a step
    count of its own -- it got gradients in 2 of 5 steps): every entry comes back by (group name, position in
    group) with its own step, the state_dict loads into torch.optim.Adam, and the restored FusedAdam and that
    torch Adam then take the same next step."""
    from gsd_amd import DeformableGaussians
    from gsd_amd.io import capture, restore
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    lrs = [0.00016, 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]

    def model(seed):
        torch.manual_seed(seed)
        pc = DeformableGaussians(make_gaussians(599, 64, 48, seed=seed, device=DEV), sh_degree=3)
        net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3)).to(DEV)
        ps = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
        groups = ([{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(ps, lrs, names)] +
                  [{"params": list(net.parameters()), "lr": 8e-4, "name": "offset_model"}])
        return ps, net, FusedAdam(groups, lr=0.0, eps=1e-15), pc

    def backward(ps, net, ws, x, with_net):
        loss = sum((p * w).sum() for p, w in zip(ps, ws))
        if with_net:
            loss = loss + net(x).square().sum()
        loss.backward()

    ps, net, opt, pc = model(1)
    gen = torch.Generator().manual_seed(2)
    x = torch.randn(5, 8, generator=gen).to(DEV)
    for k in range(5):
        backward(ps, net, [torch.randn(p.shape, generator=gen).to(DEV) for p in ps], x, k >= 3)
        opt.step(zero_grad=True)
    path = str(tmp_path / "chkpnt.pth")
    torch.save(capture(pc, opt, None, 1.0), path)
    args = torch.load(path, weights_only=True)
    assert [float(args[10]["state"][i]["step"]) for i in range(10)] == [5.0] * 6 + [2.0] * 4
    ps2, net2, opt2, pc2 = model(9)
    net2.load_state_dict(net.state_dict())   # the reference saves the network itself separately
    restore(args, pc2, opt2)
    assert opt2.steps == opt.steps == [5] * 6 + [2] * 4
    for p, q in zip(ps + list(net.parameters()), ps2 + list(net2.parameters())):
        assert torch.equal(p.detach(), q.detach())
        for m1, m2 in zip(opt.moments(p), opt2.moments(q)):
            assert torch.equal(m1, m2) and float(m1.abs().max()) > 0
    # the reference's optimizer built the same way takes the checkpoint and the same next step
    ref_ps = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    ref_net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3)).to(DEV)
    ref_net.load_state_dict(net.state_dict())
    ref = torch.optim.Adam([{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(ref_ps, lrs, names)] +
                           [{"params": list(ref_net.parameters()), "lr": 8e-4, "name": "offset_model"}],
                           lr=0.0, eps=1e-15)
    ref.load_state_dict(args[10])
    ws = [torch.randn(p.shape, generator=gen).to(DEV) for p in ps]
    backward(ps2, net2, ws, x, True)
    backward(ref_ps, ref_net, ws, x, True)
    opt2.step(zero_grad=True)
    ref.step()
    for p, q in zip(ps2 + list(net2.parameters()), ref_ps + list(ref_net.parameters())):
        assert float((p - q).abs().max()) <= 1e-6 * max(1.0, float(q.abs().max()))


def test_densify_and_prune_matches_reference():
    """gsd_amd.densify (fused statistics kernel + FusedAdam slab surgery) vs the line-by-line restatement of
    scene/gaussian_model.py's densification on torch.optim.Adam (oracle/densify_ref.py): statistics after three
    views, then densify_and_prune (clone + split with the same torch.normal draws + prune), reset_opacity and
    one more optimizer step -- same point count, parameters, moments and statistics."""
    from gsd_amd import DeformableGaussians
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    from oracle.densify_ref import RefGaussians
    P = 4000
    prm = make_gaussians(P, 320, 240, seed=21, device=DEV)
    lrs = [0.00016, 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]
    pc = DeformableGaussians(prm, sh_degree=3)
    ps = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
    opt = FusedAdam([{"params": [p], "lr": lr, "name": n} for p, lr, n in
                     zip(ps, lrs, ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"])], lr=0.0, eps=1e-15)
    dens = GaussianDensifier(pc, opt)
    ref = RefGaussians(*(p.detach() for p in ps), lrs=lrs)
    gen = torch.Generator().manual_seed(3)
    extent = float(torch.exp(prm.scaling).max(dim=1).values.median()) / 0.01  # ~half the points split, half clone

    def both_step():
        gs = [torch.randn(p.shape, generator=gen).to(DEV) * 1e-3 for p in ps]
        for p, g in zip(ps, gs):
            p.grad.copy_(g)
        for p, g in zip(ref.params(), gs):
            p.grad = g.clone()
        opt.step()
        ref.optimizer.step()

    def compare(tag):
        assert pc._xyz.shape == ref._xyz.shape, tag
        for a, b in zip(ps, ref.params()):
            assert float((a.detach() - b.detach()).abs().max()) <= 1e-5, tag
        for a, b in zip(ps, ref.params()):
            m, v = opt.moments(a)
            st = ref.optimizer.state[b]
            assert float((m - st["exp_avg"]).abs().max()) <= 1e-6, tag
            assert float((v - st["exp_avg_sq"]).abs().max()) <= 1e-9, tag
        for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
            assert float((getattr(dens, n) - getattr(ref, n)).abs().max()) <= 1e-6, (tag, n)

    both_step()
    for _ in range(3):
        vg = torch.randn(P, 3, generator=gen).to(DEV) * 2e-4
        radii = torch.randint(0, 30, (P,), generator=gen, dtype=torch.int32).to(DEV)
        holder = torch.zeros(P, 3, device=DEV, requires_grad=True)
        holder.grad = vg
        dens.add_densification_stats(holder, radii)
        ref.add_stats(vg, radii)
    compare("stats")
    torch.cuda.manual_seed(11)
    dens.densify_and_prune(2e-4, 0.05, extent, 20)
    torch.cuda.manual_seed(11)
    ref.densify_and_prune(2e-4, 0.05, extent, 20)
    assert pc._xyz.shape[0] != P  # something was cloned / split / pruned
    compare("densify_and_prune")
    dens.reset_opacity()
    ref.reset_opacity()
    compare("reset_opacity")
    ps[:] = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
    both_step()
    compare("step after surgery")


def test_checkpoint_capture_restore_roundtrip(tmp_path):
    """gsd_amd.io.capture / restore (gaussian_model.py:686-730): the tuple survives torch.save /
    torch.load(weights_only=True), restores parameters, statistics and Adam moments into a fresh model, and
    its optimizer state_dict loads into a torch.optim.Adam built with the reference's groups."""
    from gsd_amd import DeformableGaussians
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.io import capture, restore
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    lrs = [0.00016, 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]

    def model(seed):
        pc = DeformableGaussians(make_gaussians(999, 64, 48, seed=seed, device=DEV), sh_degree=3)
        ps = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
        opt = FusedAdam([{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(ps, lrs, names)], eps=1e-15)
        return pc, ps, opt, GaussianDensifier(pc, opt)

    pc, ps, opt, dens = model(1)
    gen = torch.Generator().manual_seed(2)
    for _ in range(2):
        for p in ps:
            p.grad.copy_(torch.randn(p.shape, generator=gen).to(DEV))
        opt.step()
    dens.max_radii2D.fill_(3.0)
    path = str(tmp_path / "chkpnt_2.pth")
    torch.save((capture(pc, opt, dens, 1.5), 2), path)
    model_args, it = torch.load(path, weights_only=True)
    assert it == 2 and len(model_args) == 12
    pc2, ps2, opt2, dens2 = model(9)
    assert restore(model_args, pc2, opt2, dens2) == 1.5
    for a, b in zip(ps, ps2):
        assert torch.equal(a.detach(), b.detach())
        for x, y in zip(opt.moments(a), opt2.moments(b)):
            assert torch.equal(x, y)
    assert opt2.step_count == 2 and torch.equal(dens2.max_radii2D, dens.max_radii2D)
    ref_ps = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    ref = torch.optim.Adam([{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(ref_ps, lrs, names)],
                           lr=0.0, eps=1e-15)
    ref.load_state_dict(model_args[10])
    assert torch.equal(ref.state[ref_ps[2]]["exp_avg"], opt.moments(ps[2])[0])


def test_render_with_deformation_mlp():
    """render() with the reference's deformation network as the offset producer (past its 3000-iteration
    zero phase): the fused preamble + split-SH rasterizer and the reference-literal preamble give the same
    image and the same gradients for the network's weights and the Gaussians."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    from gsd_amd.scene import make_gaussians
    torch.manual_seed(0)
    net = DirectTemporalNeRF().to(DEV)
    with torch.no_grad():
        for h in (net._time_out, net._time_out_scale, net._time_out_rot, net._time_out_shs):
            h.weight.mul_(0.01)  # small offsets, like a trained network
    params = make_gaussians(8000, 256, 192, seed=5, device=DEV)
    cam = synthetic_camera(256, 192).to(DEV)
    res = []
    for fused in (True, False):
        net.zero_grad(set_to_none=True)
        pc = DeformableGaussians(params, sh_degree=3, offset_model=net)
        pc.fused_preamble = fused
        out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV), iteration=5000)
        (out["render"] * torch.linspace(0, 1, 256, device=DEV)).sum().backward()
        res.append((out["render"].detach(), [p.grad.clone() for p in pc.parameters()],
                    [p.grad.clone() for p in net.parameters()]))
    assert (res[0][0] - res[1][0]).abs().max() <= 1e-5
    for a, b in zip(res[0][1] + res[0][2], res[1][1] + res[1][2]):
        assert rel_l2(a, b) <= 1e-4


@pytest.mark.parametrize("P,dup", [(2, False), (5, False), (3000, False), (5000, True)])
def test_knn_init_matches_bruteforce(P, dup):
    """gsd_knn (simple-knn's Morton-box 3-NN, distCUDA2) bit-exact against the brute-force float32 restatement
    (oracle/knn_ref.py), several boxes of 1024, duplicated points, fewer than 4 points; create_from_pcd."""
    from gsd_amd.init import create_from_pcd, dist_cuda2
    from oracle.knn_ref import mean_dist2
    gen = torch.Generator().manual_seed(P)
    pts = torch.randn(P, 3, generator=gen) * torch.tensor([3.0, 1.0, 0.5]) + 2.0
    if dup:
        pts[100:200] = pts[0:100]
    got = dist_cuda2(pts.to(DEV)).cpu().numpy()
    ref = mean_dist2(pts.numpy())
    assert np.array_equal(got, ref) or (np.isinf(ref).any() and np.array_equal(np.isinf(got), np.isinf(ref)))
    if P >= 4:
        g = create_from_pcd(pts.to(DEV), torch.rand(P, 3, generator=gen).to(DEV))
        assert g.features_dc.shape == (P, 1, 3) and g.features_rest.shape == (P, 15, 3)
        assert torch.allclose(g.scaling[:, 0].cpu(), torch.log(torch.sqrt(torch.clamp_min(torch.from_numpy(ref),
                                                                                            1e-7))))


def test_coefficient_major_sh_layout_same_gradients():
    """FusedAdam(coef_major=True) stores the SH parameters coefficient-major (permuted slab views, gsd_sh_split
    strides): render + backward + one step give the same parameters as the default contiguous layout."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    params = make_gaussians(20_000, 320, 240, seed=8, device=DEV)
    cam = synthetic_camera(320, 240).to(DEV)
    outs = []
    for cm in (False, True):
        pc = DeformableGaussians(params, sh_degree=3)
        opt = FusedAdam([{"params": [p], "lr": 1e-3} for p in pc.parameters()], lr=0.0, eps=1e-15, coef_major=cm)
        assert pc._features_rest.is_contiguous() == (not cm)
        for _ in range(2):
            out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV))
            (out["render"] * torch.linspace(0, 1, 320, device=DEV)).sum().backward()
            opt.step(zero_grad=True)
        outs.append([p.detach().clone() for p in pc.parameters()])
    for a, b in zip(*outs):
        assert rel_l2(a, b) <= 1e-5


def _fused_step_run(fused, net=None, steps=3, P=20_000, W=320, H=240, iteration=0):
    """render + loss + backward + Adam for `steps` steps, with the step fused into the backward
    (FusedAdam.step_in_backward) or as the separate pass (allreduce_step) -> parameters, moments, steps."""
    from gsd_amd import DeformableGaussians, default_pipe, l1_ssim_loss, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    params = make_gaussians(P, W, H, seed=8, device=DEV)
    cam = synthetic_camera(W, H).to(DEV)
    pc = DeformableGaussians(params, sh_degree=3, offset_model=net)
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    lrs = [0.00016, 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]
    ps = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
    groups = [{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(ps, lrs, names)]
    if net is not None:
        groups.append({"params": list(net.parameters()), "lr": 1e-4, "name": "offset_model"})
    opt = FusedAdam(groups, lr=0.0, eps=1e-15)
    gt = torch.rand(3, H, W, generator=torch.Generator().manual_seed(3)).to(DEV)
    for _ in range(steps):
        out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV), iteration=iteration)
        loss = l1_ssim_loss(out["render"], gt, 0.2)
        if fused:
            with opt.step_in_backward():
                loss.backward()
        else:
            loss.backward()
            opt.allreduce_step(zero_grad=True)
    return ([p.detach().clone() for p in opt._params], [m.clone() for p in opt._params for m in opt.moments(p)],
            list(opt.steps), opt)


def test_step_in_backward_equals_backward_then_step():
    """FusedAdam.step_in_backward (Adam fused into the preprocess backward for the SH pieces and the raw
    parameters: gsd_adam_epilogue) gives the parameters and moments of backward() + allreduce_step() -- the same
    per-element arithmetic, up to the float-atomic order of the rasterizer's gradient sums -- and the same step
    counts; no separate Adam launch remains."""
    from gsd_amd._native import kernel_times
    kernel_times(enable=True, reset=True)
    a_p, a_m, a_s, opt = _fused_step_run(True)
    kt = kernel_times(enable=False, reset=True)
    assert "adam" not in kt and opt.flat.fused == set()
    b_p, b_m, b_s, _ = _fused_step_run(False)
    assert a_s == b_s == [3] * 6
    for x, y in zip(a_p + a_m, b_p + b_m):
        assert rel_l2(x, y) <= 1e-5
        assert float((x - y).abs().max()) <= 1e-5 * max(1.0, float(y.abs().max()))


def test_step_in_backward_with_offset_network():
    """With the deformation network live (iteration past 3000): the SH pieces are fused (the offset's gradient
    still flows to the network), the raw parameters take the separate pass (the activation preamble path),
    the network is stepped on leaving the block -- all equal to backward() + step."""
    from gsd_amd.deform_mlp import DirectTemporalNeRF
    res = []
    for fused in (True, False, False, False):   # one fused run, three unfused runs for the noise figure
        torch.manual_seed(0)
        net = DirectTemporalNeRF().to(DEV)
        with torch.no_grad():
            for h in (net._time_out, net._time_out_scale, net._time_out_rot, net._time_out_shs):
                h.weight.mul_(0.01)
        res.append(_fused_step_run(fused, net=net, steps=2, P=6000, W=192, H=128, iteration=5000))
    assert res[0][2] == res[1][2]
    # Bars: the Gaussians' parameters and moments 1e-4 (the rasterizer's float-atomic order, ~1e-6 relative per
    # gradient, is all that differs).  The network's gradients are sums over the 6,000 Gaussians that mostly cancel
    # (layer-0 weight gradients ~1e-9 from terms ~1e-6), which amplifies that same noise by up to ~1e3.  So each
    # tensor's bar is measured: 20x the largest rel L2 between the three unfused runs (the same float-atomic order
    # noise, with no fusion in it), with the Gaussians' 1e-4 as the floor.
    n_params = len(res[0][0])
    flat = [r[0] + r[1] for r in res]
    for k in range(len(flat[0])):
        noise = max(rel_l2(flat[i][k], flat[j][k]) for i, j in ((1, 2), (1, 3), (2, 3)))
        bar = max(1e-4, 20.0 * noise)
        err = rel_l2(flat[0][k], flat[1][k])
        assert err <= bar, (k, "moment" if k >= n_params else "param", err, noise)


def test_step_in_backward_rejects_second_producer():
    """A second gradient for a parameter the block already stepped (a regulariser on _scaling: autograd sums its
    gradient with the rasterizer's before the parameter's AccumulateGrad, after the rasterizer has run) would be
    lost: it raises instead, whichever of the two was built first -- autograd's saved-tensor version check (the
    fused kernel bumps the parameters' versions) or the FlatGrads guard; outside the block the loss trains."""
    from gsd_amd import DeformableGaussians, default_pipe, render
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    cam = synthetic_camera(128, 96).to(DEV)
    for reg_first in (True, False):
        pc = DeformableGaussians(make_gaussians(3000, 128, 96, seed=2, device=DEV), sh_degree=3)
        opt = FusedAdam([{"params": [p], "lr": 1e-3} for p in pc.parameters()], lr=0.0, eps=1e-15)
        reg = 1e-3 * pc._scaling.square().sum() if reg_first else None
        out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV))
        loss = out["render"].sum() + (reg if reg_first else 1e-3 * pc._scaling.square().sum())
        with pytest.raises(RuntimeError, match="second gradient|modified by an inplace operation"):
            with opt.step_in_backward():
                loss.backward()
        assert opt.flat.epilogue is None and not opt.flat.fused
        out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV))
        (out["render"].sum() + 1e-3 * pc._scaling.square().sum()).backward()
        opt.allreduce_step(zero_grad=True)
        assert all(bool(torch.isfinite(p).all()) for p in pc.parameters())


def test_fused_adam_addend_matches_torch_adam():
    """FlatGrads.add_after_reduce (a gradient term already summed over the ranks: the exchanged views' mean term,
    gsd_sh_grad_views_ex d_means): FusedAdam steps on grad + addend inside its pass (gsd_adam_step_ex), for
    parameters whose slab range starts on and off a quad boundary, against torch.optim.Adam on the sum."""
    from gsd_amd.optim import FusedAdam
    gen = torch.Generator().manual_seed(9)
    shapes = [(333, 3), (250, 1), (101, 4)]   # the second and third start off a quad boundary of the slab
    init = [torch.randn(*s, generator=gen) for s in shapes]
    a = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    b = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    opt_a = FusedAdam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(a)], lr=0.0, eps=1e-15)
    opt_b = torch.optim.Adam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(b)], lr=0.0, eps=1e-15,
                             foreach=True)
    for k in range(2):
        gs = [torch.randn(*s, generator=gen) for s in shapes]
        adds = [torch.randn(*s, generator=gen) * 0.5 for s in shapes]
        for p, g in zip(a, gs):
            p.grad.copy_(g.to(DEV))
        for i in (0, 2):                       # two of the three take an addend
            opt_a.flat.add_after_reduce(a[i], adds[i].to(DEV).contiguous())
        for i, (p, g) in enumerate(zip(b, gs)):
            p.grad = (g + adds[i]).to(DEV) if i in (0, 2) else g.to(DEV)
        opt_a.step(zero_grad=True)
        opt_b.step()
    for pa, pb in zip(a, b):
        assert float((pa - pb).abs().max()) <= 1e-6
    assert opt_a.flat.addends == {}


@pytest.mark.parametrize("P", [1, 37, 100_003, 1_000_000])
def test_offset_norm_matches_torch(P):
    """train.py:329 torch.norm(means3D_offset, dim=-1).mean() (the expression itself is the reference) against
    gsd_offset_norm: value rel 1e-5 (deterministic fixed-order sum vs torch's reduction order), gradient rel L2
    1e-6, zero rows giving a zero gradient as torch's norm backward does."""
    from gsd_amd.loss import offset_norm
    gen = torch.Generator().manual_seed(P)
    x = torch.randn(P, 3, generator=gen) * 0.05
    x[::7] = 0.0                                                          # zero offsets (norm 0)
    a = x.clone().to(DEV).requires_grad_(True)
    b = x.clone().to(DEV).requires_grad_(True)
    got = offset_norm(a)
    ref = torch.norm(b, dim=-1).mean()
    assert abs(float(got) - float(ref)) <= 1e-5 * max(float(ref), 1e-30)
    (3.0 * got).backward()
    (3.0 * ref).backward()
    assert rel_l2(a.grad, b.grad) <= 1e-6
    assert float(a.grad[::7].abs().max()) == 0.0
    assert float(offset_norm(a.detach(), 2.0)) == pytest.approx(2.0 * float(got), rel=1e-6)


def test_training_loss_with_offset_regulariser():
    """The reference's loss of train.py:323-332 and :529 -- (1 - l) (L1 + 0.1 mean||offset||) + l (1 - SSIM) --
    against its literal torch expression over the loss restatement; the gradient reaches both the image and the
    offsets.  An undeformed render's offset (an expanded zero row, no gradient) adds exactly 0."""
    from gsd_amd.loss import l1_ssim_loss, training_loss
    from oracle import loss_ref
    gen = torch.Generator().manual_seed(31)
    gt = torch.rand(3, 60, 80, generator=gen).to(DEV)
    base = (gt + 0.1 * torch.randn(3, 60, 80, generator=gen).to(DEV)).clamp(0, 1)
    off0 = (torch.randn(5000, 3, generator=gen) * 0.02).to(DEV)
    x1, o1 = base.clone().requires_grad_(True), off0.clone().requires_grad_(True)
    x2, o2 = base.clone().requires_grad_(True), off0.clone().requires_grad_(True)
    got = training_loss(x1, gt, o1, 0.2)
    Ll1 = loss_ref.l1_loss(x2, gt) + 0.1 * torch.norm(o2, dim=-1).mean()
    ref = (1.0 - 0.2) * Ll1 + 0.2 * (1.0 - loss_ref.ssim(x2, gt))
    assert abs(float(got) - float(ref)) <= 1e-5 * abs(float(ref))
    got.backward()
    ref.backward()
    assert rel_l2(x1.grad, x2.grad) <= 1e-4 and rel_l2(o1.grad, o2.grad) <= 1e-6
    zero = torch.zeros(1, 3, device=DEV).expand(5000, 3)
    assert float(training_loss(base, gt, zero)) == float(l1_ssim_loss(base, gt))


def test_fused_adam_follows_expon_lr_schedule():
    """update_learning_rate (scene/gaussian_model.py:875-886) rewriting the xyz and offset_model groups every step,
    on FusedAdam and on torch.optim.Adam: same parameters after 6 steps (1e-6), through both the plain step and
    the data-parallel entry at world size 1."""
    from gsd_amd.schedule import get_expon_lr_func, update_learning_rate
    a, b, opt_a, opt_b, gen = _adam_pair(seed=17)
    opt_a.param_groups[0]["name"] = opt_b.param_groups[0]["name"] = "xyz"
    xyz = get_expon_lr_func(0.00016, 0.0000016, max_steps=10)
    off = get_expon_lr_func(8e-4, 1.6e-6, max_steps=10)
    for k in range(6):
        for opt in (opt_a, opt_b):
            update_learning_rate(opt, 2 * k, xyz, off)
        assert opt_a.param_groups[0]["lr"] == xyz(2 * k) and opt_a.param_groups[3]["lr"] == off(2 * k)
        ws = [torch.randn(p.shape, generator=gen).to(DEV) for p in a]
        _adam_backward(a, ws, True)
        _adam_backward(b, ws, True)
        opt_a.allreduce_step(zero_grad=True) if k % 2 else opt_a.step(zero_grad=True)
        opt_b.step()
        opt_b.zero_grad(set_to_none=True)
    for pa, pb in zip(a, b):
        assert float((pa - pb).abs().max()) <= 1e-6 * max(1.0, float(pb.abs().max()))


def test_zero_grad_set_to_none_skips_parameters_without_grad():
    """optimizer.zero_grad(set_to_none=True) (train.py:683) then a backward that reaches only the Gaussian groups:
    torch.optim.Adam skips the network's grad-None parameters (no move, no step count, moments kept); FusedAdam
    must do the same.  zero_grad(set_to_none=False) zeroes the gradients that exist (stepped with zeros next) and
    leaves grad-None parameters without one."""
    a, b, opt_a, opt_b, gen = _adam_pair(seed=23)
    for k in range(4):
        ws = [torch.randn(p.shape, generator=gen).to(DEV) for p in a]
        with_net = k == 0
        _adam_backward(a, ws, with_net)
        _adam_backward(b, ws, with_net)
        opt_a.step()
        opt_b.step()
        opt_a.zero_grad(set_to_none=(k != 1))
        opt_b.zero_grad(set_to_none=(k != 1))
        for i, (pa, pb) in enumerate(zip(a, b)):
            st = opt_b.state.get(pb)
            assert opt_a.steps[i] == (int(st["step"]) if st else 0), (k, i)
            assert float((pa - pb).abs().max()) <= 1e-6 * max(1.0, float(pb.abs().max())), (k, i)
    # the network got a gradient at k = 0 only: set_to_none=False after k = 1 zeroes existing gradients and leaves
    # its grad None (torch), so k = 2 skips it as well
    assert opt_a.steps[3:] == [1, 1, 1] and opt_a.steps[:3] == [4, 4, 4]


def test_densify_and_prune_carries_the_se3_twist():
    """SE(3) mode: the per-Gaussian twist is trained (its own optimizer group) and must follow the densification
    surgery like the other per-Gaussian attributes -- clones and split children inherit their parent's twist with
    zero moments, pruned points drop it -- so the next SE(3) render sees a twist of the new length.  The twist is
    set to a copy of attributes the reference's surgery already carries (rotation, f_dc), so the rows can be
    checked exactly; its moment rows must be zero exactly where the rotation's are."""
    from gsd_amd import DeformableGaussians, l1_ssim_loss, render, default_pipe
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import make_gaussians
    P, W, H = 4000, 320, 240
    prm = make_gaussians(P, W, H, seed=22, se3="random", device=DEV)
    with torch.no_grad():
        prm.twist.copy_(torch.cat([prm.rotation, prm.features_dc[:, 0, :2]], 1))
    pc = DeformableGaussians(prm, sh_degree=3, deform="se3")
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "twist"]
    opt = FusedAdam([{"params": [p], "lr": 1e-3, "name": n} for p, n in zip(pc.parameters(), names)], lr=0.0,
                    eps=1e-15)
    dens = GaussianDensifier(pc, opt)
    gen = torch.Generator().manual_seed(4)
    for p in pc.parameters():   # one step with the same gradient rows for rotation and twist: equal moments
        p.grad.copy_(torch.randn(p.shape, generator=gen).to(DEV) * 1e-3)
    with torch.no_grad():
        pc._twist.grad.copy_(torch.cat([pc._rotation.grad, pc._features_dc.grad[:, 0, :2]], 1))
    opt.step(zero_grad=True)
    vg = torch.randn(P, 3, generator=gen).to(DEV) * 2e-4
    holder = torch.zeros(P, 3, device=DEV, requires_grad=True)
    holder.grad = vg
    dens.add_densification_stats(holder, torch.randint(1, 30, (P,), generator=gen, dtype=torch.int32).to(DEV))
    extent = float(torch.exp(pc._scaling).max(dim=1).values.median()) / 0.01
    dens.densify_and_prune(2e-4, 0.05, extent, 20)
    Pn = pc._xyz.shape[0]
    assert Pn != P and pc._twist.shape == (Pn, 6)
    assert torch.equal(pc._twist[:, :4], pc._rotation) and torch.equal(pc._twist[:, 4:], pc._features_dc[:, 0, :2])
    mt, vt = opt.moments(pc._twist)
    mr, vr = opt.moments(pc._rotation)
    assert torch.equal(mt[:, :4], mr) and torch.equal(vt[:, :4], vr)
    assert int((mr.abs().sum(1) == 0).sum()) > 0          # new points with zero moments exist
    cam = synthetic_camera(W, H).to(DEV)
    out = render(cam, pc, default_pipe(), torch.zeros(3, device=DEV))
    l1_ssim_loss(out["render"], torch.zeros_like(out["render"])).backward()
    assert pc._twist.grad.shape == (Pn, 6) and torch.isfinite(pc._twist.grad).all()


def test_densify_and_prune_matches_reference_gaussian_model_fixture(monkeypatch):
    """gsd_amd.densify + FusedAdam on the GPU against the reference's own GaussianModel + torch.optim.Adam run
    (tests/golden/densify.npz, gaussian_model.py:1027-1257 and train.py:613-616): two Adam steps, three views of
    statistics, densify_and_prune with the reference's split samples, reset_opacity and one more step -- the same
    point count, and parameters / moments / statistics within the FusedAdam-vs-torch bars of
    test_densify_and_prune_matches_reference."""
    from test_oracle_golden import _densify_fixture_run
    from conftest import golden
    from gsd_amd import DeformableGaussians
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.optim import FusedAdam
    from gsd_amd.scene import GaussianParams
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]

    class M:
        pass

    def make(init, lrs, pd):
        m = M()
        t = [torch.from_numpy(v).to(DEV) for v in init]
        prm = GaussianParams(xyz=t[0], features_dc=t[1], features_rest=t[2], opacity=t[3], scaling=t[4],
                             rotation=t[5])
        m.pc = DeformableGaussians(prm, sh_degree=3)
        ps = [m.pc._xyz, m.pc._features_dc, m.pc._features_rest, m.pc._opacity, m.pc._scaling, m.pc._rotation]
        m.opt = FusedAdam([{"params": [p], "lr": lr, "name": n} for p, lr, n in zip(ps, lrs, names)], lr=0.0,
                          eps=1e-15)
        m.dens = GaussianDensifier(m.pc, m.opt, percent_dense=pd)
        return m

    def params(m):
        return [m.pc._xyz, m.pc._features_dc, m.pc._features_rest, m.pc._opacity, m.pc._scaling, m.pc._rotation]

    def step(m, gs):
        for p, gr in zip(params(m), gs):
            p.grad.copy_(torch.from_numpy(gr).to(DEV))
        m.opt.step()

    def stats(m, vg, radii):
        holder = torch.zeros(vg.shape, device=DEV, requires_grad=True)
        holder.grad = torch.from_numpy(vg).to(DEV)
        m.dens.add_densification_stats(holder, torch.from_numpy(radii).to(DEV))

    def densify(m, max_grad, min_op, extent, mss, samples):
        monkeypatch.setattr(torch, "normal", lambda mean, std: torch.from_numpy(samples).to(mean.device, mean.dtype))
        m.dens.densify_and_prune(max_grad, min_op, extent, mss)
        monkeypatch.undo()

    def snapshot(m):
        out = {}
        for n, p in zip(names, params(m)):
            out[n] = p.detach().cpu().numpy()
            mo, v = m.opt.moments(p)
            out[n + ":exp_avg"], out[n + ":exp_avg_sq"] = mo.cpu().numpy(), v.cpu().numpy()
        for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
            out["stat:" + n] = getattr(m.dens, n).cpu().numpy().reshape(-1, *getattr(m.dens, n).shape[1:])
        return out

    _densify_fixture_run(golden("densify.npz"), make, step, stats, densify, lambda m: m.dens.reset_opacity(),
                         snapshot, dict(param=1e-5, m=1e-6, v=1e-9, stat=1e-6))


def _train_run(fused_step, steps=4, P=30_000, W=320, H=240, densify_at=None):
    """`steps` training steps (render + 0.8 L1 + 0.2 (1 - SSIM) + backward + Adam + densification statistics) of
    one view through the drop-in API (render, training_loss, FusedAdam.step_in_backward, GaussianDensifier) or
    through FusedTrainStep -> parameters, moments, statistics, the last image and loss."""
    from bench import make_optimizer
    from gsd_amd import DeformableGaussians, default_pipe, render, training_loss
    from gsd_amd.camera import synthetic_camera
    from gsd_amd.densify import GaussianDensifier
    from gsd_amd.scene import make_gaussians
    from gsd_amd.train_step import FusedTrainStep
    torch.manual_seed(123)   # densify_and_prune's split samples come from the global generators
    pc = DeformableGaussians(make_gaussians(P, W, H, seed=9).to(DEV), sh_degree=3)
    cam = synthetic_camera(W, H).to(DEV)
    bg = torch.zeros(3, device=DEV)
    gt = torch.rand(3, H, W, generator=torch.Generator().manual_seed(4)).to(DEV)
    opt = make_optimizer(pc)
    dens = GaussianDensifier(pc, opt)
    seed = torch.ones((), device=DEV)
    fs = FusedTrainStep(pc, opt, cam, gt, bg, 0.2, densifier=dens) if fused_step else None
    img = loss = None
    for i in range(steps):
        if fs is not None:
            out = fs()
            img, loss = out["render"].clone(), fs.loss()
        else:
            out = render(cam, pc, default_pipe(), bg)
            lo = training_loss(out["render"], gt, out["means3D_offset"], 0.2)
            with opt.step_in_backward():
                lo.backward(seed)
            dens.add_densification_stats(out["viewspace_points"], out["radii"])
            img, loss = out["render"].detach().clone(), float(lo.detach())
        if densify_at is not None and i == densify_at:
            dens.densify_and_prune(0.0002, 0.005, 10.0, None)
    stats = [dens.xyz_gradient_accum, dens.xyz_gradient_accum_3vec, dens.denom, dens.max_radii2D]
    return ([p.detach().clone() for p in opt._params], [opt.exp_avg.clone(), opt.exp_avg_sq.clone()],
            [s.clone() for s in stats], list(opt.steps), img, loss)


@pytest.mark.parametrize("densify_at", [None, 1])
def test_fused_train_step_equals_dropin_step(densify_at):
    """FusedTrainStep (one gsd_train_step call per step) against the drop-in API's step: the same parameters,
    Adam moments, step counts and densification statistics after several steps (the float-atomic order of the
    rasterizer's gradient sums is all that differs, rel L2 1e-5), the same image and loss on the last step; with
    a densify_and_prune in between (new slabs: the fused step rebuilds its structures)."""
    a = _train_run(True, densify_at=densify_at)
    b = _train_run(False, densify_at=densify_at)
    assert a[3] == b[3]
    for x, y in zip(a[0] + a[1] + a[2], b[0] + b[1] + b[2]):
        assert x.shape == y.shape
        assert rel_l2(x, y) <= 1e-5, rel_l2(x, y)
    # the last image: both runs' parameters differ by the gradient sums' float-atomic order (above), which the
    # compositing can amplify at a pixel to ~1e-5 (1.4e-5 measured after a densification)
    assert float((a[4] - b[4]).abs().max()) <= 1e-4
    assert abs(a[5] - b[5]) <= 1e-5 * max(1.0, abs(b[5]))


def test_fused_train_step_grows_its_binning_buffer():
    """A short binning buffer (a guess of 1 instance) is grown and the step redone without a state change: the
    result equals the drop-in path's."""
    from gsd_amd import train_step
    orig = train_step.FusedTrainStep._build

    def tiny(self):
        self._k_guess = 1
        orig(self)
    train_step.FusedTrainStep._build = tiny
    try:
        a = _train_run(True, steps=2)
    finally:
        train_step.FusedTrainStep._build = orig
    b = _train_run(False, steps=2)
    for x, y in zip(a[0] + a[1], b[0] + b[1]):
        assert rel_l2(x, y) <= 1e-5
