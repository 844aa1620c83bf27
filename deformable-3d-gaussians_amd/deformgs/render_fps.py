"""Inference FPS loop of render_baseline.render_set (render_baseline.py:57-74): per view, deform.step
+ render() between two device synchronisations, FPS = 1 / mean(t[skip:]). No image I/O (the
reference's first loop, which writes PNGs, is not timed there either)."""
import time

import numpy as np
import torch

from .renderer import render


@torch.no_grad()
def measure_fps(views, gaussians, pipeline, background, deform, is_6dof=False, skip=5, repeat=1):
    t_list = []
    for _ in range(repeat):
        for view in views:
            xyz = gaussians.get_xyz
            time_input = view.fid.unsqueeze(0).expand(xyz.shape[0], -1)
            torch.cuda.synchronize()
            t0 = time.time()
            d_xyz, d_rotation, d_scaling = deform.step(xyz.detach(), time_input)
            render(view, gaussians, pipeline, background, d_xyz, d_rotation, d_scaling, is_6dof)
            torch.cuda.synchronize()
            t_list.append(time.time() - t0)
    t = np.array(t_list[skip:])
    return 1.0 / t.mean(), len(t)
