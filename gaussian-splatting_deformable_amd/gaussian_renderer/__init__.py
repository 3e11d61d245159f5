"""Drop-in module name of the reference's gaussian_renderer (render(), :20-195)."""
from gsd_amd.renderer import render  # noqa: F401
