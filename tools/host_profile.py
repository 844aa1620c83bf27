#!/usr/bin/env python3
"""Host-side cost of one bench step: wall time of each phase with the GPU kept busy-free
(synchronize around every phase, so each number is CPU issue time + that phase's GPU time), and a
torch.profiler table of CPU self time per op over a few unsynchronised steps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import forward_backward, optimizer_step
    from deformgs.renderer import render
    from deformgs.loss import l1_ssim_loss
    from deformgs.adam import step_all
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
    for _ in range(5):
        forward_backward(gaussians, deform, cam, gt, pipe, bg)
        optimizer_step(gaussians, deform, 3000)
    torch.cuda.synchronize()

    phases = {}

    def tick(name, t0):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        phases.setdefault(name, []).append((t1 - t0) * 1e3)
        return t1

    for _ in range(10):
        t = time.perf_counter()
        xyz = gaussians.get_xyz.detach()
        ti = cam.fid.unsqueeze(0).expand(N, -1)
        d = deform.step(xyz, ti)
        t = tick("deform_fwd", t)
        pkg = render(cam, gaussians, pipe, bg, *d)
        t = tick("render_fwd", t)
        loss, _, _ = l1_ssim_loss(pkg["render"], gt, 0.2)
        t = tick("loss_fwd", t)
        loss.backward()
        t = tick("backward", t)
        step_all(gaussians.optimizer, deform.optimizer)
        gaussians.optimizer.zero_grad(set_to_none=True)
        deform.optimizer.zero_grad()
        t = tick("adam+zero", t)
    print("phase wall (ms, synchronised, median of 10):")
    for k, v in phases.items():
        v.sort()
        print(f"  {k:12s} {v[len(v) // 2]:8.3f}")

    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(5):
            forward_backward(gaussians, deform, cam, gt, pipe, bg)
            optimizer_step(gaussians, deform, 3000)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=45, max_name_column_width=60))


if __name__ == "__main__":
    main()
