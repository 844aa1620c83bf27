#!/usr/bin/env python3
"""Renders synth-100k (800x800) forward + backward and saves image, radii and gradients to an .npz:
python3 tools/sort_check.py OUT.npz. Run once with DGS_HIPCUB_SORT=1 and once without to check that
the build's radix sort (radix.hip) bins exactly as hipcub::DeviceRadixSort (bitwise-equal results
up to the order of float atomics in the blend backward, so gradients are compared to tolerance)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from deformgs.arguments import PipelineParams
    from deformgs.gaussian_model import GaussianModel
    from deformgs.renderer import render
    from deformgs.synthetic import synth_camera, synth_gaussians
    dev = torch.device("cuda", 0)
    N, R = 100_000, 800
    g = synth_gaussians(N, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    out = {}
    for k in range(3):
        cam = synth_camera(R, R, index=k, fid=0.3, device=dev)
        pk = render(cam, gs, PipelineParams(), torch.zeros(3, device=dev), 0.0, 0.0, 0.0)
        img = pk["render"]
        (img * torch.linspace(0, 1, img.numel(), device=dev).view_as(img)).sum().backward()
        out[f"img{k}"] = img.detach().cpu().numpy()
        out[f"radii{k}"] = pk["radii"].cpu().numpy()
        out[f"gxyz{k}"] = gs._xyz.grad.cpu().numpy()
        gs._xyz.grad = None
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
