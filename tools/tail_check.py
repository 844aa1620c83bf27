#!/usr/bin/env python3
"""Outputs and parameter gradients of the fused deformation MLP at sizes whose last block round is
split into 16-point tail blocks (mlp_split.hip block_split) -> npz; run once with DGS_MLP_NO_TAIL=1
and once without and compare bitwise: python3 tools/tail_check.py out.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from deformgs.deform_network import DeformNetworkBaseline
    dev = torch.device("cuda", 0)
    res = {}
    for N, uniform in ((100_000, True), (20_000, False), (65_600, True)):
        torch.manual_seed(0)
        net = DeformNetworkBaseline(is_blender=True).to(dev)
        x = torch.rand(N, 3, device=dev) * 2.6 - 1.3
        t = torch.full((1, 1), 0.3, device=dev).expand(N, 1) if uniform else torch.rand(N, 1, device=dev)
        out = net(x, t)
        w = [torch.linspace(-1, 1, o.numel(), device=dev).reshape(o.shape) for o in out]
        sum((o * wi).sum() for o, wi in zip(out, w)).backward()
        for i, o in enumerate(out):
            res[f"N{N}_out{i}"] = o.detach().cpu().numpy()
        for k, p in net.named_parameters():
            res[f"N{N}_{k}"] = p.grad.cpu().numpy()
    np.savez(sys.argv[1], **res)


if __name__ == "__main__":
    main()
