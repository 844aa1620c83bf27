#!/usr/bin/env python3
"""Sort-binning renders at many speculative pair capacities (the tile sort then runs over `cap`
items, padding sorting last) compared bitwise with the render at the exact capacity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from deformgs import _lib
    from deformgs.arguments import PipelineParams
    from deformgs.gaussian_model import GaussianModel
    from deformgs.renderer import render
    from deformgs.synthetic import synth_camera, synth_gaussians
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    bad = 0
    for N, R in ((6000, 160), (100_000, 800)):
        gd = synth_gaussians(N, seed=0, device=dev)
        gs = GaussianModel(3)
        gs.from_tensors(gd["xyz"], gd["features_dc"], gd["features_rest"], gd["scaling"], gd["rotation"], gd["opacity"])
        cam = synth_camera(R, R * 4 // 5, index=2, fid=0.3, device=dev)
        bg = torch.zeros(3, device=dev)
        for mode in (1, 0):
            lib.dgs_debug_set_binning(mode)
            lib.dgs_debug_set_pair_cap(0, 1)  # synchronous exact count for nr
            pk = render(cam, gs, PipelineParams(), bg, 0.0, 0.0, 0.0)
            nr = int(pk["render"].grad_fn.num_rendered)
            del pk
            with torch.no_grad():
                lib.dgs_debug_set_pair_cap(0, 1)  # force the exact (redo) path: reference image
                ref = render(cam, gs, PipelineParams(), bg, 0.0, 0.0, 0.0)["render"].clone()
                caps = list(range(1, 4000, 37)) + [nr + k for k in range(0, 70000, 997)]
                for cap in caps:
                    lib.dgs_debug_set_pair_cap(0, cap)
                    img = render(cam, gs, PipelineParams(), bg, 0.0, 0.0, 0.0)["render"]
                    if not torch.equal(img, ref):
                        bad += 1
                        d = (img - ref).abs()
                        print("N", N, "mode", mode, "cap", cap, "nr", nr, "max", d.max().item(), "px", int((d > 0).sum()))
            print("N", N, "mode", mode, "nr", nr, "caps", len(caps))
    lib.dgs_debug_set_binning(0)
    print("mismatches", bad)


if __name__ == "__main__":
    main()
