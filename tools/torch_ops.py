#!/usr/bin/env python3
"""Which torch (non-HIP-library) kernels run per training step, and from which op: the bench step
under torch.profiler, printing each aten op that launched device work in one step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.renderer import render
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import forward_backward, optimizer_step
    dev = torch.device("cuda", 0)
    N, R = 100_000, 800
    g = synth_gaussians(N, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    opt = OptimizationParams()
    gs.training_setup(opt)
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    deform.train_setting(opt)
    pipe = PipelineParams()
    bg = torch.zeros(3, device=dev)
    cam = synth_camera(R, R, index=0, fid=0.3, device=dev)
    with torch.no_grad():
        d = deform.step(gs.get_xyz.detach(), cam.fid.unsqueeze(0).expand(N, -1))
        gt = render(cam, gs, pipe, bg, d[0], d[1], d[2])["render"].clone()
    for it in range(3):
        forward_backward(gs, deform, cam, gt, pipe, bg)
        optimizer_step(gs, deform, 3000 + it)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        forward_backward(gs, deform, cam, gt, pipe, bg)
        optimizer_step(gs, deform, 3010)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))


if __name__ == "__main__":
    main()
