"""Densification and pruning (cfg 5 runs it every 100 views).

Mirrors scene/gaussian_model.py:960-1257 and its call site train.py:610-648 for a ``DeformableGaussians``
trained by ``gsd_amd.optim.FusedAdam``:

- ``add_densification_stats`` / the max-radii update (train.py:613-616, :1252-1257) run as one fused HIP
  pass (``gsd_densify_stats``) instead of ~8 boolean-mask torch kernels per view.
- ``densify_and_clone`` (:1186-1200), ``densify_and_split`` (:1129-1152), ``prune_points`` (:1064-1079),
  ``densify_and_prune`` (:1219-1233) and ``reset_opacity`` (:960-963) keep the reference's selection rules,
  sampling (``torch.normal`` around the parent with its scale, rotated), ordering and optimizer-state
  semantics: new points get zero moments, pruned points drop theirs, a replaced tensor gets zero moments.
  They run every ``densification_interval`` (100) views, so they stay torch ops on the GPU; the flat
  parameter / moment / gradient slabs are rebuilt once per call (``FusedAdam.rebuild``).
- A per-Gaussian SE(3) twist (``DeformableGaussians._twist``, the SE(3) mode's trained parameter) is a
  per-Gaussian attribute like the rotation: clones and split children inherit their parent's twist with zero
  moments, pruned points drop it (the reference has no per-Gaussian twist -- its twists come from the network).
- Data parallel (one view per rank, replicated Gaussians): every rank accumulates the statistics of its own
  views; ``densify_and_prune`` first combines them across ranks (``sync_stats``: sums of the counts and
  gradient norms, max of the radii -- what one process accumulating every view holds), and the split's normal
  samples are drawn on rank 0 and broadcast, so every rank selects, samples and prunes identically and the
  replicated parameters (and P) stay the same on every rank.
"""
from __future__ import annotations

import torch

from . import _native
from ._C import _ptr, _stream
from .parallel import broadcast_, dp_active, view_stats_allreduce
from .renderer import build_rotation, inverse_sigmoid

_NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


class GaussianDensifier:
    def __init__(self, pc, optimizer, percent_dense: float = 0.01):
        self.pc = pc
        self.opt = optimizer
        self.percent_dense = percent_dense
        self._reset_stats()

    # ---- statistics (one fused kernel per view) ----
    def _reset_stats(self):
        P, dev = self.pc._xyz.shape[0], self.pc._xyz.device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.xyz_gradient_accum_3vec = torch.zeros((P, 3), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)

    def add_densification_stats(self, viewspace_point_tensor, radii):
        """train.py:613-616: max_radii2D / gradient accumulators for the Gaussians with radii > 0
        (``visibility_filter``); ``viewspace_point_tensor`` is render()'s ``viewspace_points``."""
        g = viewspace_point_tensor.grad
        if g is None:
            raise RuntimeError("add_densification_stats: viewspace_points has no gradient (call backward first)")
        lib = _native.load()
        P = int(radii.shape[0])
        g = g.contiguous()
        r = radii.to(torch.int32).contiguous()
        with torch.cuda.device(g.device):
            _native.check(lib.gsd_densify_stats(P, _ptr(g), _ptr(r), _ptr(self.xyz_gradient_accum),
                                                _ptr(self.xyz_gradient_accum_3vec), _ptr(self.denom),
                                                _ptr(self.max_radii2D), _stream(g.device)))

    def sync_stats(self):
        """Combine the per-rank statistics (no-op on one rank): afterwards every rank holds the statistics of
        all ranks' views."""
        if dp_active():
            view_stats_allreduce(self.denom, self.xyz_gradient_accum, self.max_radii2D,
                                 self.xyz_gradient_accum_3vec)

    # ---- optimizer-state surgery ----
    def _params(self):
        pc = self.pc
        ps = [pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation]
        return ps + ([pc._twist] if getattr(pc, "_twist", None) is not None else [])

    def _names(self):
        return _NAMES + (("twist",) if getattr(self.pc, "_twist", None) is not None else ())

    def _apply(self, fn):
        """fn(name, data, exp_avg, exp_avg_sq) -> (data, exp_avg, exp_avg_sq) for every Gaussian attribute;
        any other optimizer parameter (e.g. a twist or an offset network) must not change shape."""
        datas, ms, vs = [], [], []
        gauss = {id(p): n for p, n in zip(self._params(), self._names())}
        for g in self.opt.param_groups:
            for p in g["params"]:
                m, v = self.opt.moments(p)
                if id(p) in gauss:
                    d, m, v = fn(gauss[id(p)], p.detach(), m, v)
                else:
                    d = p.detach()
                datas.append(d)
                ms.append(m)
                vs.append(v)
        self.opt.rebuild(datas, ms, vs)

    def densification_postfix(self, new):
        """:1107-1127 -- append points (zero moments) and reset the statistics."""
        self._apply(lambda n, d, m, v: (torch.cat((d, new[n]), 0), torch.cat((m, torch.zeros_like(new[n])), 0),
                                        torch.cat((v, torch.zeros_like(new[n])), 0)))
        self._reset_stats()

    def prune_points(self, mask):
        """:1064-1079 -- drop the points where ``mask`` is True (with their moments and statistics)."""
        keep = ~mask
        self._apply(lambda n, d, m, v: (d[keep], m[keep], v[keep]))
        self.xyz_gradient_accum = self.xyz_gradient_accum[keep]
        self.xyz_gradient_accum_3vec = self.xyz_gradient_accum_3vec[keep]
        self.denom = self.denom[keep]
        self.max_radii2D = self.max_radii2D[keep]

    # ---- the reference's operations ----
    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        pc = self.pc
        sel = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(pc.get_scaling, dim=1).values <= self.percent_dense * scene_extent)
        new = {"xyz": pc._xyz[sel], "f_dc": pc._features_dc[sel], "f_rest": pc._features_rest[sel],
               "opacity": pc._opacity[sel], "scaling": pc._scaling[sel], "rotation": pc._rotation[sel]}
        if "twist" in self._names():
            new["twist"] = pc._twist[sel]
        self.densification_postfix({k: v.detach() for k, v in new.items()})

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2):
        pc = self.pc
        n_init = pc._xyz.shape[0]
        padded = torch.zeros((n_init), device=pc._xyz.device)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(pc.get_scaling, dim=1).values > self.percent_dense * scene_extent)
        with torch.no_grad():
            stds = pc.get_scaling[sel].repeat(N, 1)
            means = torch.zeros((stds.size(0), 3), device=pc._xyz.device)
            samples = broadcast_(torch.normal(mean=means, std=stds))   # rank 0's draw on every rank
            rots = build_rotation(pc._rotation[sel]).repeat(N, 1, 1)
            new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + pc._xyz[sel].repeat(N, 1),
                   "scaling": torch.log(pc.get_scaling[sel].repeat(N, 1) / (0.8 * N)),
                   "rotation": pc._rotation[sel].repeat(N, 1), "f_dc": pc._features_dc[sel].repeat(N, 1, 1),
                   "f_rest": pc._features_rest[sel].repeat(N, 1, 1), "opacity": pc._opacity[sel].repeat(N, 1)}
            if "twist" in self._names():
                new["twist"] = pc._twist[sel].repeat(N, 1)
        self.densification_postfix(new)
        prune = torch.cat((sel, torch.zeros(N * int(sel.sum()), device=sel.device, dtype=torch.bool)))
        self.prune_points(prune)

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, N=2):
        """:1219-1233 (after combining the ranks' statistics) as ONE optimizer-state surgery: the reference runs
        clone (append), split (append, then drop the split originals) and the prune as four tensor rebuilds; the
        result is assembled here directly -- [surviving originals | clones | split children], pruned -- with the
        same selections, the same torch.normal draw and the same order, so the points, parameters and moments
        are the reference's (tests/test_gpu_train.py::test_densify_and_prune_matches_reference).  Clone and split
        select from the original points only (the split's padded gradients are zero for the clones), and the
        statistics are reset by the reference's densification_postfix before its final prune, so the screen-size
        test (max_radii2D) never fires there; it is kept as the reference writes it.
        2M Gaussians: one rebuild instead of four."""
        self.sync_stats()
        grads = self.xyz_gradient_accum / self.denom
        grads = torch.where(grads.isnan(), 0.0, grads)   # grads[grads.isnan()] = 0.0, without a mask index
        pc = self.pc
        with torch.no_grad():
            scal = pc.get_scaling
            smax = scal.max(dim=1).values
            clone = torch.logical_and(torch.norm(grads, dim=-1) >= max_grad, smax <= self.percent_dense * extent)
            split = torch.logical_and(grads.squeeze(-1) >= max_grad, smax > self.percent_dense * extent)
            # each selection as ascending indices, once: a boolean-mask index runs nonzero and waits for its count
            # on the host, and the ~50 of them over the parameters and moments took half of the call (2M Gaussians:
            # 9.4 ms); index_select with these is the same gather, in the same order
            split_i, clone_i, keep_i = split.nonzero().squeeze(1), clone.nonzero().squeeze(1), (~split).nonzero().squeeze(1)
            # densify_and_split's draw (after the clones, which draw nothing): rank 0's samples on every rank
            scal_s = scal.index_select(0, split_i)
            stds = scal_s.repeat(N, 1)
            samples = broadcast_(torch.normal(mean=torch.zeros((stds.size(0), 3), device=stds.device), std=stds))
            rots = build_rotation(pc._rotation.index_select(0, split_i)).repeat(N, 1, 1)
            src = dict(zip(self._names(), (p.detach() for p in self._params())))
            children = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1)
                        + src["xyz"].index_select(0, split_i).repeat(N, 1),
                        "scaling": torch.log(scal_s.repeat(N, 1) / (0.8 * N))}

            def kids(n, d):
                return children[n] if n in children else d.index_select(0, split_i).repeat(N, *([1] * (d.dim() - 1)))

            def assemble(n, d):
                return torch.cat((d.index_select(0, keep_i), d.index_select(0, clone_i), kids(n, d)), 0)

            opac = assemble("opacity", src["opacity"])
            prune = (pc.opacity_activation(opac) < min_opacity).squeeze(-1)
            if max_screen_size:
                P_new = opac.shape[0]   # the statistics were reset before this test: max_radii2D is all zero
                big_vs = torch.zeros(P_new, dtype=torch.bool, device=opac.device) > max_screen_size
                big_ws = pc.scaling_activation(assemble("scaling", src["scaling"])).max(dim=1).values > 0.1 * extent
                prune = torch.logical_or(torch.logical_or(prune, big_vs), big_ws)
            live_i = (~prune).nonzero().squeeze(1)
            # cat(d[keep], d[clone], kids)[live] as one gather from d and one from the children: the surviving rows
            # of the [keep | clone] part come first, in order, so their indices compose; a moment row is the old one
            # for a surviving kept point and zero for every clone and child (the reference's cat of zeros)
            nk, nkc = keep_i.numel(), keep_i.numel() + clone_i.numel()
            n_from_d = int(torch.searchsorted(live_i, torch.tensor([nkc], device=live_i.device)).item())
            n_from_keep = int(torch.searchsorted(live_i, torch.tensor([nk], device=live_i.device)).item())
            idx_d = torch.cat((keep_i, clone_i)).index_select(0, live_i[:n_from_d])
            idx_kid = live_i[n_from_d:] - nkc
            idx_m = keep_i.index_select(0, live_i[:n_from_keep])
            n_zero = live_i.numel() - n_from_keep

            def surgery(n, d, m, v):
                zm = torch.zeros((n_zero,) + tuple(d.shape[1:]), dtype=d.dtype, device=d.device)
                return (torch.cat((d.index_select(0, idx_d), kids(n, d).index_select(0, idx_kid)), 0),
                        torch.cat((m.index_select(0, idx_m), zm), 0),
                        torch.cat((v.index_select(0, idx_m), zm), 0))

        self._apply(surgery)
        self._reset_stats()

    def reset_opacity(self):
        """:960-963 -- opacities to min(sigmoid(o), 0.01), with zero moments for that group."""
        with torch.no_grad():
            new = inverse_sigmoid(torch.min(self.pc.get_opacity, torch.ones_like(self.pc.get_opacity) * 0.01))
        self._apply(lambda n, d, m, v: (new, torch.zeros_like(new), torch.zeros_like(new)) if n == "opacity"
                    else (d, m, v))
