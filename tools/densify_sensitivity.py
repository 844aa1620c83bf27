#!/usr/bin/env python3
"""R8 sensitivity check: the fork's densification statistic is computed from
means2D_densify, whose CUDA semantics are not visible (un-vendored filter-norm branch). This build
defines it as the per-pixel |dL/dmean2D| summed per axis (AbsGS-style); the upstream 3DGS statistic
is |sum of dL/dmean2D| (means2D). The fork raised the threshold from 3DGS's 0.0002 to 0.0007.

Runs the fused training step on a synthetic scene (no densification, so N is fixed), accumulates both
statistics exactly as add_densification_stats does (norm of the first two components over visible
iterations, divided by the visible count), and prints, per threshold, the fraction of Gaussians each
definition would densify. If the fork's 0.0007 on the AbsGS statistic selects a fraction close to
3DGS's 0.0002 on the plain one, the higher threshold is consistent with this reading.

python3 tools/densify_sensitivity.py [--n 55000 --res 800 --iters 300]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=55_000)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.train import SyntheticScene, build_viewpoint_stack
    from deformgs.train_step import optimizer_step, train_step
    import random
    dev = torch.device("cuda", 0)
    scene = SyntheticScene(a.n, a.res, a.res, device=dev)
    g = scene.init_gaussians(GaussianModel(3))
    g.active_sh_degree = 3
    opt = OptimizationParams()
    g.training_setup(opt)
    torch.manual_seed(0)
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    deform.train_setting(opt)
    bg = torch.zeros(3, device=dev)
    N = g.get_xyz.shape[0]
    acc = {"plain": torch.zeros(N, device=dev), "absgs": torch.zeros(N, device=dev)}
    denom = torch.zeros(N, device=dev)
    rng = random.Random(0)
    stack = []
    for it in range(a.iters):
        if not stack:
            stack = build_viewpoint_stack(scene.getTrainCameras(), 30)
        cam = stack.pop(rng.randint(0, len(stack) - 1))
        warm = it >= a.iters // 3  # the first third static, as the reference's warm-up
        loss, pkg, _ = train_step(g, deform, cam, cam.original_image, PipelineParams(), bg, warm=warm)
        with torch.no_grad():
            vis = pkg["visibility_filter"]
            acc["plain"] += torch.where(vis, pkg["viewspace_points"].grad[:, :2].norm(dim=-1), 0.0)
            acc["absgs"] += torch.where(vis, pkg["viewspace_points_densify"].grad[:, :2].norm(dim=-1), 0.0)
            denom += vis.float()
        optimizer_step(g, deform, 3000 + it)
    out = {"n": N, "iters": a.iters, "res": a.res, "selected_fraction": {}}
    for k, v in acc.items():
        mean = torch.where(denom > 0, v / denom.clamp_min(1), 0.0)
        out["selected_fraction"][k] = {str(t): float((mean >= t).float().mean()) for t in (0.0002, 0.0004, 0.0007, 0.001)}
        out[k + "_median"] = float(mean[denom > 0].median())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
