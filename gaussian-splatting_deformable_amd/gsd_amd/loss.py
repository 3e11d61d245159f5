"""Training loss of one view, fused in HIP (gsd_loss.hip via gsd_l1_ssim).

Mirrors ``utils/loss_utils.py``: ``l1_loss`` (:17-18), ``ssim`` (:33-63: 11x11 Gaussian window,
sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2, mean over the map) and the combination of
``train.py:529``: ``(1 - lambda_dssim) * L1 + lambda_dssim * (1 - SSIM)`` with lambda_dssim = 0.2
(``arguments/__init__.py:83``), plus the offset-norm regulariser of ``train.py:329-332``
(``Ll1 = Ll1 + 0.1 * torch.norm(means3D_offset, dim=-1).mean()``, before the mix): ``training_loss``.  The forward computes the value and keeps the SSIM window adjoints; the
backward (gsd_l1_ssim_backward) turns them into d loss / d image, scaled by autograd's incoming gradient.  Images are (C,H,W) (or (1,C,H,W)) float32 on a HIP
device.  No CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native
from ._C import _dev_f32, _ptr, _stream


def _check(img: torch.Tensor, gt: torch.Tensor):
    if img.dim() == 4 and img.size(0) == 1:
        img, gt = img[0], gt[0]
    if img.dim() != 3 or img.shape != gt.shape:
        raise RuntimeError(f"l1_ssim: expected two (C,H,W) images of the same shape, got {tuple(img.shape)} and "
                           f"{tuple(gt.shape)}")
    dev = img.device
    if dev.type != "cuda":
        raise RuntimeError("l1_ssim: images must be HIP device tensors (there is no CPU implementation)")
    return _dev_f32(img.detach(), "image", dev), _dev_f32(gt.detach(), "gt", dev)


def _run(img: torch.Tensor, gt: torch.Tensor, lambda_dssim: float):
    """Forward: {loss, L1, SSIM} (device) and the workspace holding the window adjoints the backward reads."""
    lib = _native.load()
    x, y = _check(img, gt)
    dev = x.device
    C, H, W = (int(s) for s in x.shape)
    ws = torch.empty(lib.gsd_l1_ssim_workspace_bytes(C, H, W), dtype=torch.uint8, device=dev)
    out3 = torch.empty(3, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _native.check(lib.gsd_l1_ssim(C, H, W, _ptr(x), _ptr(y), ctypes.c_float(lambda_dssim), _ptr(out3), None,
                                      _ptr(ws), _stream(dev)))
    return out3, x, y, ws


class _L1Ssim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, gt, lambda_dssim, which):
        out3, x, y, ws = _run(img, gt, lambda_dssim)
        ctx.shape = img.shape
        ctx.lambda_dssim = lambda_dssim
        ctx.sign = -1.0 if which == 2 else 1.0  # ssim() returns SSIM = 1 - loss(lambda = 1)
        ctx.save_for_backward(x, y, ws)
        return out3[which]

    @staticmethod
    def backward(ctx, g):
        # the incoming gradient scales d loss / d img inside the kernel (no separate multiply)
        x, y, ws = ctx.saved_tensors
        lib = _native.load()
        dev = x.device
        C, H, W = (int(s) for s in x.shape)
        gs = _dev_f32(g.reshape(1), "grad", dev)
        dimg = torch.empty_like(x)
        with torch.cuda.device(dev):
            _native.check(lib.gsd_l1_ssim_backward(C, H, W, _ptr(x), _ptr(y), ctypes.c_float(ctx.lambda_dssim),
                                                   _ptr(gs), ctypes.c_float(ctx.sign), _ptr(dimg), _ptr(ws),
                                                   _stream(dev)))
        return dimg.view(ctx.shape), None, None, None


def l1_ssim_loss(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float = 0.2) -> torch.Tensor:
    """(1 - lambda) * l1_loss + lambda * (1 - ssim)  (train.py:529), differentiable w.r.t. ``image``."""
    return _L1Ssim.apply(image, gt, float(lambda_dssim), 0)


def l1_loss(network_output: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """utils/loss_utils.py:17-18 (fused kernel with lambda = 0)."""
    return _L1Ssim.apply(network_output, gt, 0.0, 1)


def ssim(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 11, size_average: bool = True) -> torch.Tensor:
    """utils/loss_utils.py:33-41 (window 11, size_average only), differentiable w.r.t. ``img1``."""
    if window_size != 11 or not size_average:
        raise NotImplementedError("ssim: only the reference's defaults (window_size=11, size_average=True)")
    return _L1Ssim.apply(img1, img2, 1.0, 2)


class _OffsetNormMean(torch.autograd.Function):
    """weight * mean_g ||offset_g||_2 (train.py:329: torch.norm(means3D_offset, dim=-1).mean()), gsd_offset_norm;
    the weight is folded into the kernels' scale (no separate multiply)."""

    @staticmethod
    def forward(ctx, offset, weight):
        lib = _native.load()
        dev = offset.device
        x = _dev_f32(offset.detach(), "means3D_offset", dev)
        P = int(x.shape[0])
        out = torch.empty((), dtype=torch.float32, device=dev)
        ws = torch.empty(lib.gsd_offset_norm_workspace_bytes(P), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            _native.check(lib.gsd_offset_norm(P, _ptr(x), ctypes.c_float(weight / P), _ptr(out), _ptr(ws),
                                              _stream(dev)))
        ctx.save_for_backward(x)
        ctx.shape = offset.shape
        ctx.weight = weight
        return out

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        lib = _native.load()
        dev = x.device
        P = int(x.shape[0])
        gs = _dev_f32(g.reshape(1), "grad", dev)
        d = torch.empty_like(x)
        with torch.cuda.device(dev):
            _native.check(lib.gsd_offset_norm_backward(P, _ptr(x), _ptr(gs), ctypes.c_float(ctx.weight / P),
                                                       _ptr(d), _stream(dev)))
        return d.view(ctx.shape), None


def offset_norm(means3D_offset: torch.Tensor, weight: float = 1.0) -> torch.Tensor:
    """train.py:329 ``torch.norm(means3D_offset, dim=-1).mean()`` (times ``weight``) for (P,3) offsets on a HIP device.  An offset
    that carries no gradient and is all zeros by construction (render()'s expanded zero row when nothing deforms
    the means) contributes exactly 0 and is not read."""
    off = means3D_offset
    if off.dim() != 2 or off.shape[-1] != 3:
        raise RuntimeError(f"offset_norm: expected (P,3) offsets, got {tuple(off.shape)}")
    if off.device.type != "cuda":
        raise RuntimeError("offset_norm: offsets must be HIP device tensors (there is no CPU implementation)")
    if off.shape[0] == 0:
        raise RuntimeError("offset_norm: the mean over zero Gaussians is undefined")
    if not off.requires_grad and off.stride(0) == 0:
        return off.new_zeros(())
    return _OffsetNormMean.apply(off, float(weight))


def training_loss(image: torch.Tensor, gt: torch.Tensor, means3D_offset: torch.Tensor | None = None,
                  lambda_dssim: float = 0.2, offset_weight: float = 0.1) -> torch.Tensor:
    """The reference's training loss (train.py:323-332 and :529):
    (1 - lambda) * (L1 + offset_weight * mean ||means3D_offset||) + lambda * (1 - SSIM), evaluated as the fused
    l1_ssim_loss plus (1 - lambda) * offset_weight * offset_norm (the same value up to float rounding)."""
    loss = l1_ssim_loss(image, gt, lambda_dssim)
    if means3D_offset is None or offset_weight == 0.0:
        return loss
    off = means3D_offset
    if not off.requires_grad and off.stride(0) == 0:
        return loss   # the zero offset of an undeformed render: the term is exactly 0
    return loss + offset_norm(off, (1.0 - lambda_dssim) * offset_weight)
