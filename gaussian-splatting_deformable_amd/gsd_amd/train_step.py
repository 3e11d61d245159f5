"""One training step of one view as one native call (``gsd_train_step``, ABI 17).

The reference's step (train.py:138-683 for the live, offset-free path) is a Python sequence: ``render()``
(gaussian_renderer/__init__.py:20-195) -> ``0.8 L1 + 0.2 (1 - SSIM)`` (:529) -> ``loss.backward()`` ->
``optimizer.step()`` / ``zero_grad`` (:681-683) -> ``add_densification_stats`` (:613-616).  Through the drop-in
API (``gsd_amd.render`` + ``training_loss`` + ``FusedAdam.step_in_backward`` + ``GaussianDensifier``) each hop
is a Python / autograd / ctypes call that builds its argument structures again; at small views (configuration 2:
0.24 ms of kernels) the host then takes ~0.5 ms per step and the device waits for it
(profiles/round6/host_cfg2/).

``FusedTrainStep`` builds the argument structures once -- the raw parameters read in place (gsd_activation,
gsd_sh_split), their Adam step fused into the backward (gsd_adam_epilogue), the state buffers, the loss and
statistics buffers -- and each call only writes the per-step learning rates and step counts into them and makes
the one native call.  The kernels and their arguments are those of the drop-in path, so the results are the same
(tests/test_gpu_train.py pins that); the host work per step drops to one call.  It serves the configuration the
reference trains before its deformation network turns on (iteration < 3000: no offsets) and configurations 2, 4
and 5 of the bench: additive mode, no offset model, one rank.  Anything else (offsets, SE(3), the Python
covariance / SH modes, data parallel) keeps the drop-in path.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _C, _native
from ._C import _dev_mat, _ptr, _stream
from .parallel import dp_active
from .renderer import ZeroOffsets

_SLOTS = (("xyz", "_xyz"), ("scaling", "_scaling"), ("rotation", "_rotation"), ("opacity", "_opacity"),
          ("dc", "_features_dc"), ("rest", "_features_rest"))


class FusedTrainStep:
    """``step = FusedTrainStep(pc, opt, cam, gt, bg, densifier=dens)``; ``out = step()`` is one training step of
    view ``cam`` against ``gt``: render, ``(1 - lambda) L1 + lambda (1 - SSIM)``, backward, the Adam step of every
    Gaussian parameter and the densification statistics (when a densifier is given).  Returns a dict with the
    rendered image (``render``), ``radii``, ``viewspace_grad`` (dL/dmeans2D, what ``viewspace_points.grad`` holds on
    the drop-in path) and ``num_rendered``; the loss value is ``step.loss()`` (a device read, on demand).  The
    camera's matrices may change between calls (a different view of the same size); after ``densify_and_prune``
    (new parameter slabs) the structures are rebuilt on the next call."""

    def __init__(self, pc, opt, cam, gt, bg, lambda_dssim: float = 0.2, densifier=None, scaling_modifier=1.0):
        if getattr(pc, "deform", "additive") != "additive" or not isinstance(pc.offset_model, ZeroOffsets):
            raise RuntimeError("FusedTrainStep: the additive mode without an offset model only (offsets, SE(3): use "
                               "render() + training_loss + FusedAdam.step_in_backward)")
        if dp_active():
            raise RuntimeError("FusedTrainStep: one rank only (the data-parallel step exchanges gradients)")
        if getattr(opt, "coef_major", False):
            raise RuntimeError("FusedTrainStep: needs the parameter-major slabs (coef_major=False)")
        index = {id(p): i for i, p in enumerate(opt._params)}
        if any(id(getattr(pc, a)) not in index for _, a in _SLOTS):
            raise RuntimeError("FusedTrainStep: every Gaussian parameter must belong to the optimizer")
        self.pc, self.opt, self.cam, self.dens = pc, opt, cam, densifier
        self.lambda_dssim = float(lambda_dssim)
        self.scaling_modifier = float(scaling_modifier)
        self.gt = gt.detach().contiguous()
        self.bg = bg.detach().contiguous()
        self.dev = pc._xyz.device
        self._key = None
        self._k_guess = None
        self._seed = torch.ones(1, dtype=torch.float32, device=self.dev)

    # ---- structures ----
    def _state_key(self):
        ps = [getattr(self.pc, a) for _, a in _SLOTS]
        return tuple(p.data_ptr() for p in ps) + (int(self.pc._xyz.shape[0]), self.opt.exp_avg.data_ptr(),
                                                  self.opt.exp_avg_sq.data_ptr())

    def _stats(self):
        """The densifier's statistics buffers (re-read every call: its reset replaces them without a new P)."""
        a, d = self.args, self.dens
        if d is None:
            return
        if d.xyz_gradient_accum.shape[0] != self.P:
            raise RuntimeError("FusedTrainStep: the densifier's statistics do not match the Gaussians")
        a.grad_accum, a.grad_accum_3vec = d.xyz_gradient_accum.data_ptr(), d.xyz_gradient_accum_3vec.data_ptr()
        a.denom, a.max_radii2D = d.denom.data_ptr(), d.max_radii2D.data_ptr()

    def _build(self):
        lib = _native.load()
        pc, opt, dev = self.pc, self.opt, self.dev
        P = int(pc._xyz.shape[0])
        H, W = int(self.gt.shape[1]), int(self.gt.shape[2])
        byte = dict(dtype=torch.uint8, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.P, self.H, self.W = P, H, W
        self.geom = torch.empty(lib.gsd_geom_buffer_bytes(P, W, H), **byte)
        self.img = torch.empty(lib.gsd_image_buffer_bytes(W, H), **byte)
        self.scratch = torch.empty(lib.gsd_backward_scratch_bytes(P), **byte)
        self.radii = torch.empty(P, dtype=torch.int32, device=dev)
        self.color = torch.empty(3, H, W, **f32)
        self.dimg = torch.empty(3, H, W, **f32)
        self.loss3 = torch.empty(3, **f32)
        self.loss_ws = torch.empty(lib.gsd_l1_ssim_workspace_bytes(3, H, W), **byte)
        self.dmeans2D = torch.empty(P, 3, **f32)
        self.dcolors = torch.empty(P, 3, **f32)
        guess = self._k_guess if self._k_guess is not None else 4 * P
        self._bin(max(guess, 1))
        ps = {slot: getattr(pc, a) for slot, a in _SLOTS}
        if any(not p.is_contiguous() for p in ps.values()):
            raise RuntimeError("FusedTrainStep: the Gaussian parameters must be contiguous")
        # the gradient sinks are the parameters' .grad views of the optimizer's slab (stored, not added: every
        # sink below is fused, so none is written -- they are what the drop-in backward would name)
        opt.flat.invalidate()
        g = {slot: p.grad for slot, p in ps.items()}
        self.split = _native.ShSplit(dc=ps["dc"].data_ptr(), rest=ps["rest"].data_ptr(), d_dc=g["dc"].data_ptr(),
                                     d_rest=g["rest"].data_ptr(), accumulate=0)
        self.act = _native.Activation(d_xyz=g["xyz"].data_ptr(), d_scaling=g["scaling"].data_ptr(),
                                      d_rotation=g["rotation"].data_ptr(), d_opacity=g["opacity"].data_ptr(),
                                      accumulate=0)
        g0 = opt.param_groups[0]
        self.epi = _native.AdamEpilogue(beta1=float(g0["betas"][0]), beta2=float(g0["betas"][1]),
                                        eps=float(g0["eps"]))
        index = {id(p): i for i, p in enumerate(opt._params)}
        self._sinks = []
        for slot, p in ps.items():
            i = index[id(p)]
            a = opt._span[i][0]
            setattr(self.epi, slot, _native.AdamSink(param=p.data_ptr(), exp_avg=opt.exp_avg.data_ptr() + 4 * a,
                                                     exp_avg_sq=opt.exp_avg_sq.data_ptr() + 4 * a))
            self._sinks.append((slot, i))
        self.args = _native.TrainStepArgs(
            geom_buffer=self.geom.data_ptr(), image_buffer=self.img.data_ptr(), radii=self.radii.data_ptr(),
            out_color=self.color.data_ptr(), gt=self.gt.data_ptr(), lambda_dssim=self.lambda_dssim,
            loss_out3=self.loss3.data_ptr(), loss_workspace=self.loss_ws.data_ptr(), dL_dimg=self.dimg.data_ptr(),
            grad_seed=self._seed.data_ptr(), dL_dmeans2D=self.dmeans2D.data_ptr(),
            dL_dcolors=self.dcolors.data_ptr(), scratch=self.scratch.data_ptr())
        self.args.binning_buffer, self.args.binning_bytes = self.binning.data_ptr(), self.binning.numel()
        r = self.args.raster
        r.P, r.D, r.M, r.width, r.height = P, int(pc.active_sh_degree), 1 + int(ps["rest"].shape[1]), W, H
        r.scale_modifier = self.scaling_modifier
        r.background, r.means3D = self.bg.data_ptr(), ps["xyz"].data_ptr()
        r.opacities, r.scales, r.rotations = ps["opacity"].data_ptr(), ps["scaling"].data_ptr(), \
            ps["rotation"].data_ptr()
        r.sh_split, r.activation, r.adam = ctypes.addressof(self.split), ctypes.addressof(self.act), \
            ctypes.addressof(self.epi)
        r.grad_scratch = self.scratch.data_ptr()
        self._params = list(ps.values())
        self._key = self._state_key()

    def _bin(self, k):
        lib = _native.load()
        self.binning = torch.empty(lib.gsd_binning_buffer_bytes(k + k // 4), dtype=torch.uint8, device=self.dev)

    def _camera(self):
        cam, r = self.cam, self.args.raster
        r.alpha_mode = _C._ALPHA_MODE[0]
        r.tan_fovx = math.tan(cam.FoVx * 0.5)
        r.tan_fovy = math.tan(cam.FoVy * 0.5)
        # held for the call: the contiguous (cached) copies of the camera's matrices
        self._mats = (_dev_mat(cam.world_view_transform, "viewmatrix", self.dev),
                      _dev_mat(cam.full_proj_transform, "projmatrix", self.dev),
                      _dev_mat(cam.camera_center, "campos", self.dev))
        r.viewmatrix, r.projmatrix, r.campos = (t.data_ptr() for t in self._mats)

    # ---- the step ----
    def __call__(self):
        if self._key != self._state_key():
            self._build()
        self._stats()
        self._camera()
        opt, lib = self.opt, _native.load()
        steps = opt.steps
        for slot, i in self._sinks:   # torch.optim.Adam: this step's count and the group's current lr
            s = getattr(self.epi, slot)
            s.lr = float(opt.param_groups[opt._gidx[i]]["lr"])
            s.step = steps[i] + 1
        K = ctypes.c_int64(0)
        stream = _stream(self.dev)
        rc = lib.gsd_train_step(ctypes.byref(self.args), ctypes.byref(K), stream)
        if rc == _native.GSD_NEED_BINNING:   # nothing was modified: grow the binning buffer, step again
            self._bin(int(K.value))
            self.args.binning_buffer, self.args.binning_bytes = self.binning.data_ptr(), self.binning.numel()
            rc = lib.gsd_train_step(ctypes.byref(self.args), ctypes.byref(K), stream)
        _native.check(rc)
        for _, i in self._sinks:
            steps[i] += 1
        opt._bump(i for _, i in self._sinks)   # in-place updates through raw pointers: advance the versions
        self._k_guess = int(K.value)
        _C.last_forward.update(P=self.P, W=self.W, H=self.H, num_rendered=self._k_guess)
        return {"render": self.color, "radii": self.radii, "viewspace_grad": self.dmeans2D,
                "num_rendered": self._k_guess}

    def loss(self) -> float:
        """The last step's loss value ((1 - lambda) L1 + lambda (1 - SSIM)); reads the device."""
        return float(self.loss3[0].item())
