"""Deterministic weight / projection generators shared by make_golden.py and the tests.

numpy's PCG64 stream is bit-stable across numpy versions, so the golden fixtures store no
weights: both sides regenerate them here. Bounds follow nn.Linear's default init
(U(-1/sqrt(fan_in), 1/sqrt(fan_in)), torch/nn/modules/linear.py reset_parameters), which is
what the reference network uses (utils/time_utils.py:74-100).
"""
import numpy as np


def mlp_weights(shapes, seed):
    """shapes: ordered dict name -> shape (state_dict order). Returns name -> float32 array."""
    rng = np.random.default_rng(seed)
    out = {}
    fan_in = None
    for name, shp in shapes.items():
        if name.endswith(".weight"):
            fan_in = shp[1]
        bound = 1.0 / np.sqrt(fan_in)
        out[name] = rng.uniform(-bound, bound, size=shp).astype(np.float32)
    return out


def proj_mats(shape, seed):
    """Two +-1 projection matrices (8 x rows, 8 x cols) for checking a large gradient by sketch."""
    rng = np.random.default_rng(seed + shape[0] * 7919 + shape[1])
    r1 = rng.choice([-1.0, 1.0], size=(8, shape[0]))
    r2 = rng.choice([-1.0, 1.0], size=(8, shape[1]))
    return r1, r2
