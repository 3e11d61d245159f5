"""On-disk formats: the reference's PLY point cloud and checkpoint tuple.

- ``save_ply`` / ``load_ply`` follow scene/gaussian_model.py:891-929 and :965-1003: one binary little-endian
  ``vertex`` element of float32 properties in the order ``x y z nx ny nz f_dc_0..2 f_rest_0..44 opacity
  scale_0..2 rot_0..3``; the SH are stored channel-major (``features.transpose(1, 2).flatten(1)``). The
  reference uses the ``plyfile`` package, which is not installed here, so the format is written and parsed
  with numpy (ascii and both binary byte orders are read; any numeric property type).
- ``capture`` / ``restore`` produce and consume the tuple of ``GaussianModel.capture`` (:686-700) --
  (active_sh_degree, xyz, f_dc, f_rest, scaling, rotation, opacity, max_radii2D, xyz_gradient_accum, denom,
  optimizer state_dict, spatial_lr_scale) -- with the optimizer state in torch.optim.Adam's state_dict
  layout, matched to groups by ``name``, so checkpoints move between this framework and the reference.
  Load them with ``torch.load(path, weights_only=True)``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .scene import GaussianParams

_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def attribute_names(n_dc: int = 3, n_rest: int = 45, n_scale: int = 3, n_rot: int = 4):
    """construct_list_of_attributes (gaussian_model.py:891-903)."""
    return (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(n_dc)] +
            [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"] + [f"scale_{i}" for i in range(n_scale)] +
            [f"rot_{i}" for i in range(n_rot)])


def write_ply(path: str, columns: dict):
    """Write one float32 ``vertex`` element (binary little endian, plyfile's default layout)."""
    names = list(columns)
    n = len(next(iter(columns.values())))
    arr = np.empty(n, dtype=[(k, "<f4") for k in names])
    for k in names:
        arr[k] = np.asarray(columns[k], dtype=np.float32)
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    header += [f"property float {k}" for k in names] + ["end_header"]
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(arr.tobytes())


def read_ply(path: str) -> dict:
    """-> {property name: numpy array} of the ``vertex`` element (scalar properties only)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements, cur = None, [], None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii", "replace").split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                cur = {"name": tok[1], "count": int(tok[2]), "props": []}
                elements.append(cur)
            elif tok[0] == "property":
                if tok[1] == "list":
                    raise ValueError(f"{path}: list properties are not supported")
                cur["props"].append((tok[2], _PLY_TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        out = None
        for el in elements:
            if fmt == "ascii":
                rows = [f.readline().split() for _ in range(el["count"])]
                data = {name: np.array([r[i] for r in rows], dtype=t) for i, (name, t) in enumerate(el["props"])}
            else:
                order = "<" if fmt == "binary_little_endian" else ">"
                dt = np.dtype([(name, order + t) for name, t in el["props"]])
                raw = np.frombuffer(f.read(dt.itemsize * el["count"]), dtype=dt, count=el["count"])
                data = {name: raw[name].copy() for name, _ in el["props"]}
            if el["name"] == "vertex":
                out = data
                break
    if out is None:
        raise ValueError(f"{path}: no vertex element")
    return out


def save_ply(path: str, pc) -> None:
    """GaussianModel.save_ply (gaussian_model.py:905-922) for a DeformableGaussians (the raw parameters)."""
    xyz = pc._xyz.detach().cpu().numpy()
    f_dc = pc._features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    f_rest = pc._features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    opac = pc._opacity.detach().cpu().numpy()
    scale = pc._scaling.detach().cpu().numpy()
    rot = pc._rotation.detach().cpu().numpy()
    attrs = np.concatenate((xyz, np.zeros_like(xyz), f_dc, f_rest, opac, scale, rot), axis=1)
    names = attribute_names(f_dc.shape[1], f_rest.shape[1], scale.shape[1], rot.shape[1])
    write_ply(path, {k: attrs[:, i] for i, k in enumerate(names)})


def save_ply_t(path: str, pc, xyz, opacities, rotation) -> None:
    """GaussianModel.save_ply_t (gaussian_model.py:932-958), what render(..., save_ply=True) writes per frame
    (gaussian_renderer/__init__.py:165-167): the DEFORMED means and rotations and the ACTIVATED opacities that
    render() handed the rasterizer, with the raw SH pieces and raw scaling of ``pc``; zero normals; the attribute
    order of ``attribute_names``."""
    xyz = xyz.detach().cpu().numpy()
    f_dc = pc._features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    f_rest = pc._features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    opac = opacities.detach().cpu().numpy()
    scale = pc._scaling.detach().cpu().numpy()
    rot = rotation.detach().cpu().numpy()   # None (compute_cov3D_python) fails here, as upstream
    attrs = np.concatenate((xyz, np.zeros_like(xyz), f_dc, f_rest, opac, scale, rot), axis=1)
    names = attribute_names(f_dc.shape[1], f_rest.shape[1], scale.shape[1], rot.shape[1])
    write_ply(path, {k: attrs[:, i] for i, k in enumerate(names)})


def load_ply(path: str, max_sh_degree: int = 3) -> GaussianParams:
    """GaussianModel.load_ply (gaussian_model.py:965-1003) -> raw parameters (CPU float32 tensors)."""
    v = read_ply(path)
    xyz = np.stack((v["x"], v["y"], v["z"]), axis=1)
    opac = np.asarray(v["opacity"])[..., None]
    f_dc = np.zeros((xyz.shape[0], 3, 1))
    for c in range(3):
        f_dc[:, c, 0] = v[f"f_dc_{c}"]
    extra = sorted((k for k in v if k.startswith("f_rest_")), key=lambda k: int(k.split("_")[-1]))
    if len(extra) != 3 * (max_sh_degree + 1) ** 2 - 3:
        raise ValueError(f"{path}: {len(extra)} f_rest properties, expected {3 * (max_sh_degree + 1) ** 2 - 3}")
    f_rest = np.stack([v[k] for k in extra], axis=1).reshape(xyz.shape[0], 3, (max_sh_degree + 1) ** 2 - 1)
    sc = sorted((k for k in v if k.startswith("scale_")), key=lambda k: int(k.split("_")[-1]))
    ro = sorted((k for k in v if k.startswith("rot")), key=lambda k: int(k.split("_")[-1]))
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32)  # noqa: E731
    return GaussianParams(xyz=t(xyz), features_dc=t(f_dc).transpose(1, 2).contiguous(),
                          features_rest=t(f_rest).transpose(1, 2).contiguous(), opacity=t(opac),
                          scaling=t(np.stack([v[k] for k in sc], axis=1)),
                          rotation=t(np.stack([v[k] for k in ro], axis=1)), twist=None)


_ORDER = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


_ADAM_DEFAULTS = dict(torch.optim.Adam([torch.zeros(1, requires_grad=True)]).defaults)


def _adam_state_dict(optimizer):
    """torch.optim.Adam.state_dict() layout for a FusedAdam (global indices in group order; a parameter that
    never got a gradient has no state entry, as in torch, and every entry carries its own step)."""
    state, groups, idx = {}, [], 0
    steps = dict(zip((id(p) for p in optimizer._params), optimizer.steps))
    for g in optimizer.param_groups:
        ids = []
        for p in g["params"]:
            if steps[id(p)] > 0:
                m, v = optimizer.moments(p)
                state[idx] = {"step": torch.tensor(float(steps[id(p)])), "exp_avg": m.detach().clone(),
                              "exp_avg_sq": v.detach().clone()}
            ids.append(idx)
            idx += 1
        # torch.optim.Adam's own group keys (weight_decay, amsgrad, ...) at their defaults, so the state_dict
        # loads into it and steps there
        groups.append(_ADAM_DEFAULTS | {k: val for k, val in g.items() if k != "params"} | {"params": ids})
    return {"state": state, "param_groups": groups}


def capture(pc, optimizer, densifier=None, spatial_lr_scale: float = 1.0):
    """GaussianModel.capture (gaussian_model.py:686-700)."""
    P, dev = pc._xyz.shape[0], pc._xyz.device
    max_r = densifier.max_radii2D if densifier is not None else torch.zeros(P, device=dev)
    accum = densifier.xyz_gradient_accum if densifier is not None else torch.zeros(P, 1, device=dev)
    denom = densifier.denom if densifier is not None else torch.zeros(P, 1, device=dev)
    return (pc.active_sh_degree, pc._xyz.detach(), pc._features_dc.detach(), pc._features_rest.detach(),
            pc._scaling.detach(), pc._rotation.detach(), pc._opacity.detach(), max_r, accum, denom,
            _adam_state_dict(optimizer), spatial_lr_scale)


def restore(model_args, pc, optimizer, densifier=None):
    """GaussianModel.restore (gaussian_model.py:702-730): parameters, statistics and the Adam moments of the
    groups whose names match (a reference checkpoint may carry extra groups, e.g. its offset network)."""
    (active, xyz, f_dc, f_rest, scaling, rotation, opacity, max_r, accum, denom, opt_dict, spatial) = model_args
    pc.active_sh_degree = int(active)
    data = {"xyz": xyz, "f_dc": f_dc, "f_rest": f_rest, "opacity": opacity, "scaling": scaling,
            "rotation": rotation}
    # the checkpoint's state per (group name, position in group) -- a multi-parameter group such as the
    # reference's offset network keeps every entry -- with groups lacking a name matched by their index
    saved = {}
    for gi, g in enumerate(opt_dict["param_groups"]):
        for pos, idx in enumerate(g["params"]):
            saved[(g.get("name", gi), pos)] = opt_dict["state"].get(idx)
    news, ms, vs, steps = [], [], [], []
    gauss = {id(p): n for p, n in zip([pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling,
                                       pc._rotation], _ORDER)}
    for gi, g in enumerate(optimizer.param_groups):
        for pos, p in enumerate(g["params"]):
            n = gauss.get(id(p))
            d = data[n].to(p.device) if n is not None else p.detach()
            st = saved.get((n, 0)) if n is not None else saved.get((g.get("name", gi), pos))
            if st is not None and st.get("exp_avg") is not None and st["exp_avg"].shape == d.shape:
                ms.append(st["exp_avg"].to(p.device))
                vs.append(st["exp_avg_sq"].to(p.device))
                steps.append(int(float(st.get("step", 0))))
            else:
                ms.append(torch.zeros_like(d))
                vs.append(torch.zeros_like(d))
                steps.append(0)
            news.append(d)
    optimizer.rebuild(news, ms, vs)
    optimizer.steps = steps
    if densifier is not None:
        densifier.max_radii2D = max_r.to(pc._xyz.device)
        densifier.xyz_gradient_accum = accum.to(pc._xyz.device)
        densifier.denom = denom.to(pc._xyz.device)
        densifier.xyz_gradient_accum_3vec = torch.zeros((pc._xyz.shape[0], 3), device=pc._xyz.device)
    return spatial
