#!/usr/bin/env python3
"""Bitwise comparison of two builds of libdgs_hip.so on the fused MLP (a kernel restructuring that
keeps every output tile's summation order must reproduce the previous build's bits).
  python3 tools/lib_bitwise.py dump OUT.npz      (with DGS_LIB=... selecting the build)
  python3 tools/lib_bitwise.py cmp A.npz B.npz
The dump runs DeformNetworkBaseline forward + backward (blender and non-blender; frame-uniform t and
per-point t; ragged N) and stores the outputs and every parameter gradient."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))


def dump(path):
    import torch
    from deformgs.deform_network import DeformNetworkBaseline
    dev = torch.device("cuda", 0)
    out = {}
    for blender in (True, False):
        for N in (100_000, 4099, 70001, 17):
            for uniform in (True, False):
                torch.manual_seed(N + 7 * blender)
                net = DeformNetworkBaseline(is_blender=blender).to(dev)
                x = torch.rand(N, 3, device=dev) * 2.6 - 1.3
                t = torch.full((1, 1), 0.3, device=dev).expand(N, -1) if uniform else torch.rand(N, 1, device=dev)
                d_xyz, d_rot, d_s = net(x, t)
                (d_xyz.square().sum() + d_rot.sum() + d_s.abs().sum()).backward()
                key = f"{'bl' if blender else 'nb'}_{N}_{'u' if uniform else 'p'}"
                for name, v in (("d_xyz", d_xyz), ("d_rot", d_rot), ("d_s", d_s)):
                    out[f"{key}/{name}"] = v.detach().cpu().numpy()
                for name, p in net.named_parameters():
                    out[f"{key}/g_{name}"] = p.grad.detach().cpu().numpy()
    np.savez(path, **out)
    print(f"dumped {len(out)} arrays to {path}")


def cmp(pa, pb):
    a, b = np.load(pa), np.load(pb)
    assert sorted(a.files) == sorted(b.files), "different keys"
    bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
    print(f"{len(a.files)} arrays, {len(bad)} differ bitwise")
    for k in bad[:20]:
        d = np.abs(a[k].astype(np.float64) - b[k]).max()
        print(f"  {k}: max|d| {d:.3g} (max|a| {np.abs(a[k]).max():.3g})")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
