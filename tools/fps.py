#!/usr/bin/env python3
"""Render FPS (deform + raster forward, render_baseline.py:57-74 timing) on synthetic scenes sized like
the README's D-NeRF table (README.md:150-159, 400x400): hell 15 733, bouncing 55 622, trex 78 624
Gaussians; plus synth-100k at 800x800. Random-init deformation heads at 1/100 scale (steady state)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))

import torch  # noqa: E402


def main():
    from deformgs.arguments import PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.render_fps import measure_fps
    from deformgs.synthetic import synth_camera, synth_gaussians
    dev = torch.device("cuda", 0)
    out = {}
    for name, n, res in [("hell", 15733, 400), ("bouncing", 55622, 400), ("trex", 78624, 400), ("synth-100k", 100000, 800)]:
        g = synth_gaussians(n, seed=0, device=dev)
        gm = GaussianModel(3)
        gm.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
        torch.manual_seed(0)
        deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
        with torch.no_grad():
            for head in (deform.deform.gaussian_warp, deform.deform.gaussian_rotation, deform.deform.gaussian_scaling):
                head.weight.mul_(0.01)
                head.bias.mul_(0.01)
        views = [synth_camera(res, res, index=k, fid=k / 20.0, device=dev) for k in range(20)]
        fps, nt = measure_fps(views, gm, PipelineParams(), torch.zeros(3, device=dev), deform, repeat=3)
        out[name] = {"gaussians": n, "res": res, "fps": round(fps, 1), "timed_views": nt}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
