"""Generate the golden fixtures in tests/golden/ from the reference's own Python modules.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):   python tests/golden/make_golden.py

The reference modules are imported by file path, no bytecode written:
  scene/rigid_body.py     exp_se3 (+ the twist normalisation of gaussian_model.py:161-165)
  utils/sh_utils.py       eval_sh
  utils/graphics_utils.py getWorld2View2, getProjectionMatrix
  utils/general_utils.py  build_scaling_rotation, strip_symmetric (their hard-coded
                          device="cuda" is redirected to the CPU for this run)
  utils/loss_utils.py     l1_loss, ssim
  utils/general_utils.py  get_expon_lr_func (the training loop's learning-rate schedule)
  scene/gaussian_model.py DirectTemporalNeRF (forward + autograd), GaussianModel's densification statistics,
                          densify_and_prune and reset_opacity on its torch.optim.Adam ("model" section).  Its
                          imports plyfile, simple_knn._C and FrEIA are absent here: they are replaced by
                          placeholder modules whose every attribute raises when used, which shows the executed
                          code never touches them; the package imports utils.* / scene.rigid_body are the
                          reference's own files loaded by path; device="cuda" allocations land on the CPU.
Outputs are plain .npz arrays (inputs and expected outputs; no pickles).  Arguments name the sections to
write (default: all): se3 sh camera cov3d loss lr model.
"""
from __future__ import annotations

import importlib.util
import math
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cpu_torch_proxy():
    """A torch namespace whose zeros(..., device='cuda') lands on the CPU."""
    proxy = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})

    def zeros(*a, **kw):
        kw.pop("device", None)
        return torch.zeros(*a, **kw)

    proxy.zeros = zeros
    return proxy


class _Absent:
    """Stand-in for an attribute of a dependency absent here: any use raises."""

    def __init__(self, name):
        object.__setattr__(self, "_name", name)

    def __getattr__(self, k):
        raise RuntimeError(f"{self._name}.{k}: the executed reference code must not use {self._name}")

    def __call__(self, *a, **kw):
        raise RuntimeError(f"{self._name} called: the executed reference code must not use it")


def _absent_module(name):
    m = types.ModuleType(name)
    m.__path__ = []
    m.__getattr__ = lambda k: _Absent(f"{name}.{k}")
    return m


class _Normal:
    """torch.normal(mean=, std=) for the reference's split (gaussian_model.py:1140), drawn from a seeded CPU
    generator and recorded, so the fixture carries the exact samples the reference used."""

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.draws = []

    def __call__(self, mean, std):
        s = mean + std * torch.randn(mean.shape, generator=self.g, dtype=mean.dtype)
        self.draws.append(s.detach().clone())
        return s


def load_gaussian_model(genu, rb, shu, gu):
    """scene/gaussian_model.py by path, its package imports bound to the reference files already loaded."""
    saved = dict(sys.modules)
    utils_pkg, scene_pkg = types.ModuleType("utils"), types.ModuleType("scene")
    utils_pkg.__path__, scene_pkg.__path__ = [], []
    sysu = load("ref_system_utils", "utils/system_utils.py")
    sys.modules.update({"utils": utils_pkg, "utils.general_utils": genu, "utils.system_utils": sysu,
                        "utils.sh_utils": shu, "utils.graphics_utils": gu, "scene": scene_pkg,
                        "scene.rigid_body": rb})
    for name in ("plyfile", "simple_knn", "simple_knn._C", "FrEIA", "FrEIA.framework", "FrEIA.modules"):
        sys.modules[name] = _absent_module(name)
    try:
        gm = load("ref_gaussian_model", "scene/gaussian_model.py")
    finally:
        for k in list(sys.modules):
            if k not in saved:
                del sys.modules[k]
    return gm


def model_fixtures(genu, rb, shu, gu, lu):
    """DirectTemporalNeRF, the densification on GaussianModel + torch.optim.Adam, and the SSIM gradient."""
    gm = load_gaussian_model(genu, rb, shu, gu)
    proxy = cpu_torch_proxy()
    gm.torch = proxy

    # ---- DirectTemporalNeRF (gaussian_model.py:242-316): weights from a seeded init, 64 points, one time
    torch.manual_seed(77)
    net = gm.DirectTemporalNeRF()
    g = torch.Generator().manual_seed(78)
    x = torch.randn(64, 3, generator=g) * 0.7
    t = torch.full((64, 1), 0.375)
    xr = x.clone().requires_grad_(True)
    outs = net(xr, t, 5000)
    ws = [torch.randn(o.shape, generator=g) for o in outs]
    loss = sum((o * w).sum() for o, w in zip(outs, ws))
    names = [n for n, _ in net.named_parameters()]
    grads = torch.autograd.grad(loss, [xr] + [p for _, p in net.named_parameters()])
    zero = net(x, t, 2000)
    out = {"x": x.numpy(), "t": t.numpy(), "iteration": np.int64(5000), "names": np.array(names)}
    for n, p in net.named_parameters():
        out["w:" + n] = p.detach().numpy()
    for k, o in zip(("dx", "dscale", "drot", "dshs"), outs):
        out["out:" + k] = o.detach().numpy()
        out["zero2000:" + k] = zero[("dx", "dscale", "drot", "dshs").index(k)].detach().numpy()
    for k, w in zip(("dx", "dscale", "drot", "dshs"), ws):
        out["upstream:" + k] = w.numpy()
    out["grad:x"] = grads[0].numpy()
    for n, gr in zip(names, grads[1:]):
        out["grad:" + n] = gr.numpy()
    np.savez(os.path.join(OUT, "mlp.npz"), **out)

    # ---- densification (gaussian_model.py:1027-1257, train.py:610-618) on the reference's own GaussianModel
    torch.manual_seed(79)
    g = torch.Generator().manual_seed(80)
    P = 400
    model = gm.GaussianModel(3)
    xyz = torch.randn(P, 3, generator=g)
    fdc = torch.randn(P, 1, 3, generator=g) * 0.5
    frest = torch.randn(P, 15, 3, generator=g) * 0.1
    opac = torch.randn(P, 1, generator=g) * 2.0
    scal = torch.log(torch.rand(P, 3, generator=g) * 0.09 + 0.01)
    rot = torch.randn(P, 4, generator=g)
    nn = torch.nn
    model._xyz, model._features_dc, model._features_rest = (nn.Parameter(v.clone().requires_grad_(True))
                                                            for v in (xyz, fdc, frest))
    model._opacity, model._scaling, model._rotation = (nn.Parameter(v.clone().requires_grad_(True))
                                                       for v in (opac, scal, rot))
    model.max_radii2D = torch.zeros(P)
    targs = types.SimpleNamespace(percent_dense=0.01, position_lr_init=0.00016, position_lr_final=0.0000016,
                                  position_lr_delay_mult=0.01, position_lr_max_steps=30_000, feature_lr=0.0025,
                                  opacity_lr=0.05, scaling_lr=0.005, rotation_lr=0.001)
    model.spatial_lr_scale = 5.0
    model.training_setup(targs)
    groups = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    params = lambda: [model._xyz, model._features_dc, model._features_rest, model._opacity, model._scaling,  # noqa
                      model._rotation]
    out = {"P": np.int64(P), "percent_dense": np.float64(0.01), "spatial_lr_scale": np.float64(5.0),
           "lrs": np.array([gr["lr"] for gr in model.optimizer.param_groups if gr["name"] in groups]),
           "group_names": np.array(groups)}
    for n, v in zip(groups, (xyz, fdc, frest, opac, scal, rot)):
        out["init:" + n] = v.numpy()
    steps = []
    for k in range(2):   # two Adam steps on seeded gradients: non-trivial moments before the surgery
        gs = [torch.randn(p.shape, generator=g) * 1e-2 for p in params()]
        for p, gr in zip(params(), gs):
            p.grad = gr.clone()
        model.optimizer.step()
        model.optimizer.zero_grad()
        steps.append(gs)
    for k, gs in enumerate(steps):
        for n, gr in zip(groups, gs):
            out[f"step{k}:" + n] = gr.numpy()
    # three views of statistics (train.py:613-616 + add_densification_stats)
    for k in range(3):
        vg = torch.randn(P, 3, generator=g) * 2e-4
        radii = torch.randint(0, 30, (P,), generator=g, dtype=torch.int32)
        vis = radii > 0
        model.max_radii2D[vis] = torch.max(model.max_radii2D[vis], radii[vis])
        holder = torch.zeros(P, 3, requires_grad=True)
        holder.grad = vg
        model.add_densification_stats(holder, vis)
        out[f"view{k}:grad"] = vg.numpy()
        out[f"view{k}:radii"] = radii.numpy()
    for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
        out["stats:" + n] = getattr(model, n).numpy()
    extent = float(torch.exp(scal).max(dim=1).values.median()) / 0.01
    normal = _Normal(81)
    proxy.normal = normal
    model.densify_and_prune(2e-4, 0.05, extent, 20)
    out.update({"extent": np.float64(extent), "max_grad": np.float64(2e-4), "min_opacity": np.float64(0.05),
                "max_screen_size": np.float64(20), "split_samples": normal.draws[0].detach().numpy()})

    def snapshot(tag):
        for n, p in zip(groups, params()):
            out[f"{tag}:{n}"] = p.detach().numpy().copy()
            st = model.optimizer.state[p]
            out[f"{tag}:{n}:exp_avg"] = st["exp_avg"].numpy().copy()
            out[f"{tag}:{n}:exp_avg_sq"] = st["exp_avg_sq"].numpy().copy()
        for n in ("xyz_gradient_accum", "xyz_gradient_accum_3vec", "denom", "max_radii2D"):
            out[f"{tag}:stat:{n}"] = getattr(model, n).numpy().copy()
    snapshot("densified")
    model.reset_opacity()
    snapshot("reset")
    gs = [torch.randn(p.shape, generator=g) * 1e-2 for p in params()]
    for p, gr in zip(params(), gs):
        p.grad = gr.clone()
    model.optimizer.step()
    for n, gr in zip(groups, gs):
        out["after:grad:" + n] = gr.numpy()
    snapshot("after")
    np.savez(os.path.join(OUT, "densify.npz"), **out)

    # ---- the loss gradient (autograd of utils/loss_utils.py, train.py:529) on loss.npz's images
    lf = np.load(os.path.join(OUT, "loss.npz"))
    im1 = torch.from_numpy(lf["img1"]).requires_grad_(True)
    im2 = torch.from_numpy(lf["img2"])
    (ds,) = torch.autograd.grad(lu.ssim(im1, im2), [im1])
    loss = (1.0 - 0.2) * lu.l1_loss(im1, im2) + 0.2 * (1.0 - lu.ssim(im1, im2))
    (dl,) = torch.autograd.grad(loss, [im1])
    np.savez(os.path.join(OUT, "loss_grad.npz"), img1=lf["img1"], img2=lf["img2"], dssim_dimg1=ds.numpy(),
             loss=loss.detach().numpy(), dloss_dimg1=dl.numpy())


def lr_schedule(genu):
    """get_expon_lr_func at the reference's own arguments (gaussian_model.py:857-864 with
    arguments/__init__.py:74-77) and with a delay, over steps that cover both clips and a negative step."""
    steps = np.array([-1, 0, 1, 2, 10, 99, 100, 500, 1000, 2999, 3000, 7000, 15000, 29999, 30000, 39999, 40000,
                      40001, 100000], dtype=np.int64)
    cases = {"xyz": dict(lr_init=0.00016, lr_final=0.0000016, lr_delay_mult=0.01, max_steps=40_000),
             "offset": dict(lr_init=8e-4, lr_final=1.6e-6, max_steps=40_000),
             "delay": dict(lr_init=0.01, lr_final=1e-4, lr_delay_steps=500, lr_delay_mult=0.01, max_steps=30_000),
             "zero": dict(lr_init=0.0, lr_final=0.0, max_steps=100)}
    out = {"steps": steps}
    for name, kw in cases.items():
        f = genu.get_expon_lr_func(**kw)
        out[name] = np.array([float(f(int(s))) for s in steps], dtype=np.float64)
        for k, v in kw.items():
            out[f"{name}_{k}"] = np.float64(v)
    np.savez(os.path.join(OUT, "lr.npz"), **out)


def main():
    only = set(sys.argv[1:])
    rb = load("ref_rigid_body", "scene/rigid_body.py")
    shu = load("ref_sh_utils", "utils/sh_utils.py")
    gu = load("ref_graphics_utils", "utils/graphics_utils.py")
    genu = load("ref_general_utils", "utils/general_utils.py")
    genu.torch = cpu_torch_proxy()
    lu = load("ref_loss_utils", "utils/loss_utils.py")
    if only and only <= {"lr", "model"}:   # these sections draw nothing from the shared generator: alone
        if "lr" in only:
            lr_schedule(genu)
        if "model" in only:
            model_fixtures(genu, rb, shu, gu, lu)
        print("wrote", sorted(only))
        return
    g = torch.Generator().manual_seed(1234)

    # ---- SE(3): exp_se3 on normalised twists (gaussian_model.py:161-165), float64
    n = 64
    w = torch.randn(n, 3, generator=g, dtype=torch.float64) * 0.3
    v = torch.randn(n, 3, generator=g, dtype=torch.float64) * 0.2
    thetas = [1e-8, 1e-6, 1e-4, 1e-2, 0.5, 1.0, 2.0, math.pi - 1e-3]
    for i, t in enumerate(thetas):
        w[i] = w[i] / torch.linalg.norm(w[i]) * t
    theta = torch.linalg.norm(w, dim=-1)
    S = torch.cat([w / theta[:, None], v / theta[:, None]], dim=-1)
    T = rb.exp_se3(S, theta)
    x = torch.randn(n, 3, generator=g, dtype=torch.float64) * 2.0
    moved = rb.from_homogenous((T @ rb.to_homogenous(x)[..., None])[..., 0])
    # the reference's behaviour at a zero twist: NaN
    wz = torch.zeros(1, 3, dtype=torch.float64)
    thz = torch.linalg.norm(wz, dim=-1)
    Tz = rb.exp_se3(torch.cat([wz / thz[:, None], wz / thz[:, None]], -1), thz)
    np.savez(os.path.join(OUT, "se3.npz"), twist=torch.cat([w, v], 1).numpy(), means=x.numpy(), T=T.numpy(),
             moved=moved.numpy(), zero_twist_T=Tz.numpy())

    # ---- SH evaluation, degrees 0..3 (float32, as the renderer calls it)
    sh_out = {}
    for deg in range(4):
        sh = torch.randn(32, 3, 16, generator=g)
        d = torch.nn.functional.normalize(torch.randn(32, 3, generator=g), dim=1)
        sh_out[f"sh{deg}"] = sh.numpy()
        sh_out[f"dirs{deg}"] = d.numpy()
        sh_out[f"out{deg}"] = shu.eval_sh(deg, sh, d).numpy()
    np.savez(os.path.join(OUT, "sh.npz"), **sh_out)

    # ---- camera matrices exactly as scene/cameras.py:55-58 (minus .cuda())
    cams = {}
    for k, (yaw, tx, fovy, W, H) in enumerate([(0.0, (0, 0, 0), 60.0, 400, 400), (2.0, (0.1, -0.2, 0.5), 60.0, 1920,
                                                                                     1080), (14.0, (1, 2, 3), 45.0,
                                                                                             800, 600)]):
        a = math.radians(yaw)
        R = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        Tv = np.array(tx, dtype=np.float64)
        fy = math.radians(fovy)
        fx = 2 * math.atan(math.tan(fy / 2) * W / H)
        wv = torch.tensor(gu.getWorld2View2(R, Tv, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        pm = gu.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fx, fovY=fy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pm.unsqueeze(0)).squeeze(0)
        cc = wv.inverse()[3, :3]
        cams.update({f"R{k}": R, f"T{k}": Tv, f"fovx{k}": fx, f"fovy{k}": fy, f"W{k}": W, f"H{k}": H,
                     f"view{k}": wv.numpy(), f"proj{k}": pm.numpy(), f"full{k}": full.numpy(), f"campos{k}": cc.numpy()})
    np.savez(os.path.join(OUT, "camera.npz"), **cams)

    # ---- 3D covariance, Python path (gaussian_model.py:634-638 via general_utils)
    s = torch.exp(torch.randn(64, 3, generator=g) * 0.5 - 3.0)
    q = torch.nn.functional.normalize(torch.randn(64, 4, generator=g), dim=1)
    L = genu.build_scaling_rotation(1.0 * s, q)
    cov = genu.strip_symmetric(L @ L.transpose(1, 2))
    np.savez(os.path.join(OUT, "cov3d.npz"), scales=s.numpy(), rotations=q.numpy(), cov=cov.numpy())

    # ---- losses of the training step (next row)
    im1 = torch.rand(3, 40, 48, generator=g)
    im2 = torch.rand(3, 40, 48, generator=g)
    np.savez(os.path.join(OUT, "loss.npz"), img1=im1.numpy(), img2=im2.numpy(),
             l1=lu.l1_loss(im1, im2).numpy(), ssim=lu.ssim(im1, im2).numpy())
    lr_schedule(genu)
    model_fixtures(genu, rb, shu, gu, lu)
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
