#!/usr/bin/env python3
"""Run-to-run determinism stress: the MLP forward / backward and the rasterizer forward (rect and sort
binning) repeated many times on fixed inputs, every result compared bitwise with the first."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    from deformgs import _lib
    from deformgs.deform_network import DeformNetworkBaseline
    from deformgs.arguments import PipelineParams
    from deformgs.gaussian_model import GaussianModel
    from deformgs.renderer import render
    from deformgs.synthetic import synth_camera, synth_gaussians
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = DeformNetworkBaseline(is_blender=True).to(dev)
    N = 100_000
    x = torch.rand(N, 3, device=dev) * 2.6 - 1.3
    t = torch.full((1, 1), 0.3, device=dev).expand(N, -1)
    ref = None
    bad = 0
    for i in range(reps):
        out = net.raw(x, t)
        (out * 0.5).sum().backward()
        g = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
        for p in net.parameters():
            p.grad = None
        cur = (out.detach().clone(), g.clone())
        if ref is None:
            ref = cur
        elif not (torch.equal(cur[0], ref[0]) and torch.equal(cur[1], ref[1])):
            bad += 1
            print("MLP mismatch at", i, (cur[0] - ref[0]).abs().max().item(), (cur[1] - ref[1]).abs().max().item())
    print("MLP reps", reps, "mismatches", bad)
    gd = synth_gaussians(N, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(gd["xyz"], gd["features_dc"], gd["features_rest"], gd["scaling"], gd["rotation"], gd["opacity"])
    cam = synth_camera(800, 800, index=1, fid=0.3, device=dev)
    bg = torch.zeros(3, device=dev)
    for mode in (0, 1):
        lib.dgs_debug_set_binning(mode)
        ref, bad = None, 0
        with torch.no_grad():
            for i in range(reps):
                img = render(cam, gs, PipelineParams(), bg, 0.0, 0.0, 0.0)["render"].clone()
                if ref is None:
                    ref = img
                elif not torch.equal(img, ref):
                    bad += 1
                    d = (img - ref).abs()
                    print("raster mode", mode, "mismatch at", i, d.max().item(), int((d > 0).sum()))
        print("raster mode", mode, "reps", reps, "mismatches", bad)
    lib.dgs_debug_set_binning(0)


if __name__ == "__main__":
    main()
