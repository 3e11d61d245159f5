"""gsd_amd -- MI355X-native deformable Gaussian-splatting rasterizer.

Hot path: SE(3) deform -> EWA preprocess + SH -> tile binning
-> front-to-back compositing -> full backward, as hand-written gfx950 HIP
kernels behind the C-ABI of include/gsd_raster.h.  Public surface mirrors the
reference: ``GaussianRasterizationSettings``, ``GaussianRasterizer``,
``rasterize_gaussians`` (diff_gaussian_rasterization) and ``render``
(gaussian_renderer).
"""
from .rasterizer import GaussianRasterizationSettings, GaussianRasterizer, rasterize_gaussians  # noqa: F401
from .deform import se3_deform  # noqa: F401
from .renderer import render, DeformableGaussians, default_pipe  # noqa: F401
from .loss import l1_ssim_loss, l1_loss, ssim, offset_norm, training_loss  # noqa: F401
from . import _C, _native, camera, scene, parallel  # noqa: F401

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "se3_deform", "render",
           "DeformableGaussians", "default_pipe", "l1_ssim_loss", "l1_loss", "ssim",
           "offset_norm", "training_loss"]
