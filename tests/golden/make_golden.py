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
Outputs are plain .npz arrays (inputs and expected outputs; no pickles).  Arguments name the sections to
write (default: all): se3 sh camera cov3d loss lr.
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
    if only == {"lr"}:   # the later sections draw nothing from the generator: write them alone
        lr_schedule(genu)
        print("wrote lr.npz")
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
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
