#!/usr/bin/env python3
"""Host-side cost of the bench's training step by Python function (cProfile over 30 unsynchronised
steps, deferred pair count as in bench.py). The wait for the pair count sits inside the raster
backward's ctypes call; everything else is host issue time."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import forward_backward, optimizer_step
    dev = torch.device("cuda", 0)
    N, R = 100_000, 800
    g = synth_gaussians(N, seed=0, device=dev)
    gaussians = GaussianModel(3)
    gaussians.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    opt = OptimizationParams()
    gaussians.training_setup(opt)
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    with torch.no_grad():
        for head in (deform.deform.gaussian_warp, deform.deform.gaussian_rotation, deform.deform.gaussian_scaling):
            head.weight.mul_(0.01)
            head.bias.mul_(0.01)
    deform.train_setting(opt)
    pipe = PipelineParams()
    bg = torch.zeros(3, device=dev)
    cam = synth_camera(R, R, index=0, fid=0.5, device=dev)
    gt = torch.rand((3, R, R), device=dev)

    def steps(k):
        for it in range(k):
            forward_backward(gaussians, deform, cam, gt, pipe, bg, deferred_count=True)
            optimizer_step(gaussians, deform, 3000 + it)
    steps(5)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    steps(30)
    torch.cuda.synchronize()
    pr.disable()
    out = io.StringIO()
    st = pstats.Stats(pr, stream=out)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(30)
    print(out.getvalue())


if __name__ == "__main__":
    main()
