"""Synthetic "synth-100k" workload used by bench.py, smoke() and the tests.

Distribution (seeded numpy default_rng, then torch.manual_seed for the MLP weights):
  xyz ~ U[-1.3, 1.3]^3                   (scene/dataset_readers.py:286-290, D-NeRF random init)
  _scaling = log(0.02) + 0.1 N(0,1)      _rotation ~ N(0,1)^4 (raw, normalised by the getter)
  _opacity = logit(U[0.05, 0.95])        f_dc ~ N(0, 0.5), f_rest ~ N(0, 0.05), active_sh_degree 3
Camera: D-NeRF camera_angle_x = 0.6911112, radius 4.0311, looking at the origin.
"""
import math

import numpy as np
import torch

from .cameras import orbit_camera

DNERF_FOV = 0.6911112070083618
DNERF_RADIUS = 4.0311


def synth_gaussians(N, seed=0, device="cuda", sh_degree=3):
    rng = np.random.default_rng(seed)
    xyz = rng.uniform(-1.3, 1.3, (N, 3))
    scaling = math.log(0.02) + 0.1 * rng.standard_normal((N, 3))
    rot = rng.standard_normal((N, 4))
    op = rng.uniform(0.05, 0.95, (N, 1))
    opacity = np.log(op / (1 - op))
    M = (sh_degree + 1) ** 2
    f_dc = 0.5 * rng.standard_normal((N, 1, 3))
    f_rest = 0.05 * rng.standard_normal((N, M - 1, 3))

    def t(a):
        return torch.tensor(a, dtype=torch.float32, device=device)

    return dict(xyz=t(xyz), scaling=t(scaling), rotation=t(rot), opacity=t(opacity),
                features_dc=t(f_dc), features_rest=t(f_rest))


def synth_camera(width, height, index=0, fid=0.0, device="cuda", az=None, el=None):
    """Camera `index` of a ring of views around the origin (rank r renders view r); `az` / `el`
    (radians) place it explicitly instead."""
    if az is None:
        az = 2.0 * math.pi * (index % 16) / 16.0
    if el is None:
        el = 0.25 * math.sin(0.7 * index)
    return orbit_camera(az, el, DNERF_RADIUS, DNERF_FOV, width, height, fid=fid, data_device=device)
