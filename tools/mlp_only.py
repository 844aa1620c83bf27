#!/usr/bin/env python3
"""Runs only the fused deformation MLP (pack, forward, backward, dW) at the bench size, for
counter collection: rocprofv3 --pmc ... -- python3 tools/mlp_only.py [--iters K] [--n N]."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--n", type=int, default=100_000)
    a = ap.parse_args()
    from deformgs.deform_network import DeformNetworkBaseline
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = DeformNetworkBaseline(is_blender=True).to(dev)
    x = torch.rand(a.n, 3, device=dev) * 2 - 1
    t = torch.full((a.n, 1), 0.3, device=dev)  # one frame time, as in training
    for _ in range(a.iters):
        d_xyz, d_rot, d_s = net(x, t)
        (d_xyz.sum() + d_rot.square().sum() + d_s.abs().sum()).backward()
    torch.cuda.synchronize()
    print("ok", a.n, a.iters)


if __name__ == "__main__":
    main()
