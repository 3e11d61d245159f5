"""Drop-in module name of the reference rasterizer
(submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py):
``from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer``
works unchanged with gaussian-splatting_deformable_amd/ on sys.path."""
from gsd_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: F401
                                _RasterizeGaussians, cpu_deep_copy_tuple, rasterize_gaussians)
from gsd_amd import _C  # noqa: F401
