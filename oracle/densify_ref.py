"""Test infrastructure only (tests/ may import this; the product path never does).

Torch restatement of the reference's densification (scene/gaussian_model.py:960-1257, train.py:613-616)
on plain nn.Parameters trained by torch.optim.Adam, following the reference's statements line by line
(boolean-mask statistics updates, clone / split / prune with the optimizer-state surgery of
replace_tensor_to_optimizer / _prune_optimizer / cat_tensors_to_optimizer).  The only changes: the
device comes from the tensors (the reference hard-codes "cuda") and the model is a small container
instead of GaussianModel (whose module needs plyfile / FrEIA / simple_knn, absent here).
"""
from __future__ import annotations

import torch
import torch.nn as nn


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


def build_rotation(r):
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device)
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - r * z)
    R[:, 0, 2] = 2 * (x * z + r * y)
    R[:, 1, 0] = 2 * (x * y + r * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - r * x)
    R[:, 2, 0] = 2 * (x * z - r * y)
    R[:, 2, 1] = 2 * (y * z + r * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class RefGaussians:
    def __init__(self, xyz, f_dc, f_rest, opacity, scaling, rotation, lrs, percent_dense=0.01):
        mk = lambda t: nn.Parameter(t.clone().requires_grad_(True))  # noqa: E731
        self._xyz, self._features_dc, self._features_rest = mk(xyz), mk(f_dc), mk(f_rest)
        self._opacity, self._scaling, self._rotation = mk(opacity), mk(scaling), mk(rotation)
        self.percent_dense = percent_dense
        dev = xyz.device
        P = xyz.shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.xyz_gradient_accum_3vec = torch.zeros((P, 3), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)
        names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
        params = [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]
        self.optimizer = torch.optim.Adam([{"params": [p], "lr": lr, "name": n} for p, lr, n in
                                           zip(params, lrs, names)], lr=0.0, eps=1e-15, foreach=True)

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    def params(self):
        return [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]

    # train.py:613-616 + gaussian_model.py:1252-1257
    def add_stats(self, viewspace_grad, radii):
        visibility_filter = radii > 0
        self.max_radii2D[visibility_filter] = torch.max(self.max_radii2D[visibility_filter],
                                                        radii[visibility_filter].float())
        self.xyz_gradient_accum_3vec[visibility_filter] += viewspace_grad[visibility_filter]
        self.xyz_gradient_accum[visibility_filter] += torch.norm(viewspace_grad[visibility_filter, :2], dim=-1,
                                                                 keepdim=True)
        self.denom[visibility_filter] += 1

    def replace_tensor_to_optimizer(self, tensor, name):
        out = {}
        for group in self.optimizer.param_groups:
            if group["name"] == name:
                stored_state = self.optimizer.state.get(group["params"][0], None)
                stored_state["exp_avg"] = torch.zeros_like(tensor)
                stored_state["exp_avg_sq"] = torch.zeros_like(tensor)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(tensor.requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored_state
                out[group["name"]] = group["params"][0]
        return out

    def _prune_optimizer(self, mask):
        out = {}
        for group in self.optimizer.param_groups:
            stored_state = self.optimizer.state.get(group["params"][0], None)
            if stored_state is not None:
                stored_state["exp_avg"] = stored_state["exp_avg"][mask]
                stored_state["exp_avg_sq"] = stored_state["exp_avg_sq"][mask]
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter((group["params"][0][mask].requires_grad_(True)))
                self.optimizer.state[group["params"][0]] = stored_state
            else:
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def _assign(self, t):
        self._xyz, self._features_dc, self._features_rest = t["xyz"], t["f_dc"], t["f_rest"]
        self._opacity, self._scaling, self._rotation = t["opacity"], t["scaling"], t["rotation"]

    def prune_points(self, mask):
        valid = ~mask
        self._assign(self._prune_optimizer(valid))
        self.xyz_gradient_accum = self.xyz_gradient_accum[valid]
        self.xyz_gradient_accum_3vec = self.xyz_gradient_accum_3vec[valid]
        self.denom = self.denom[valid]
        self.max_radii2D = self.max_radii2D[valid]

    def cat_tensors_to_optimizer(self, tensors_dict):
        out = {}
        for group in self.optimizer.param_groups:
            ext = tensors_dict[group["name"]]
            stored_state = self.optimizer.state.get(group["params"][0], None)
            if stored_state is not None:
                stored_state["exp_avg"] = torch.cat((stored_state["exp_avg"], torch.zeros_like(ext)), dim=0)
                stored_state["exp_avg_sq"] = torch.cat((stored_state["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored_state
            else:
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def densification_postfix(self, new_xyz, new_f_dc, new_f_rest, new_opacities, new_scaling, new_rotation):
        d = {"xyz": new_xyz, "f_dc": new_f_dc, "f_rest": new_f_rest, "opacity": new_opacities,
             "scaling": new_scaling, "rotation": new_rotation}
        self._assign(self.cat_tensors_to_optimizer(d))
        P, dev = self._xyz.shape[0], self._xyz.device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.xyz_gradient_accum_3vec = torch.zeros((P, 3), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P), device=dev)

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2):
        n_init_points = self._xyz.shape[0]
        padded_grad = torch.zeros((n_init_points), device=self._xyz.device)
        padded_grad[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded_grad >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values > self.percent_dense * scene_extent)
        stds = self.get_scaling[sel].repeat(N, 1)
        means = torch.zeros((stds.size(0), 3), device=self._xyz.device)
        samples = torch.normal(mean=means, std=stds)
        rots = build_rotation(self._rotation[sel]).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self._xyz[sel].repeat(N, 1)
        new_scaling = torch.log(self.get_scaling[sel].repeat(N, 1) / (0.8 * N))
        new_rotation = self._rotation[sel].repeat(N, 1)
        new_f_dc = self._features_dc[sel].repeat(N, 1, 1)
        new_f_rest = self._features_rest[sel].repeat(N, 1, 1)
        new_opacity = self._opacity[sel].repeat(N, 1)
        self.densification_postfix(new_xyz, new_f_dc, new_f_rest, new_opacity, new_scaling, new_rotation)
        prune_filter = torch.cat((sel, torch.zeros(N * sel.sum(), device=sel.device, dtype=bool)))
        self.prune_points(prune_filter)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        sel = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values <= self.percent_dense * scene_extent)
        self.densification_postfix(self._xyz[sel], self._features_dc[sel], self._features_rest[sel],
                                   self._opacity[sel], self._scaling[sel], self._rotation[sel])

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent)
        prune_mask = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_points_vs = self.max_radii2D > max_screen_size
            big_points_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune_mask = torch.logical_or(torch.logical_or(prune_mask, big_points_vs), big_points_ws)
        self.prune_points(prune_mask)

    def reset_opacity(self):
        opacities_new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        self._opacity = self.replace_tensor_to_optimizer(opacities_new, "opacity")["opacity"]
