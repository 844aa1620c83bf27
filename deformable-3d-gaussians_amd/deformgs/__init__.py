"""deformgs — MI355X-native deformable-Gaussian training path (host side).

The hot path (fused deformation MLP + differentiable tile rasterizer) runs in libdgs_hip.so
(hand-written HIP for gfx950, C ABI in include/dgs.h); this package mirrors the reference's
Python surface: DeformNetwork(Baseline), DeformModel(Baseline), GaussianModel, render().
"""
from . import _lib  # noqa: F401
