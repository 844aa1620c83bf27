"""Per-parameter gradient error of the fused MLP against the golden fixtures (diagnostic: which dW
jobs / layers are off). usage: python tools/golden_grad_report.py [variant ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deformable-3d-gaussians_amd"))
from test_gpu_mlp import _net  # noqa: E402

G = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
for name in sys.argv[1:] or ["blender", "nonblender"]:
    f = np.load(f"{G}/mlp_{name}.npz")
    net, _ = _net(name, int(f["seed_w"]))
    x = torch.from_numpy(f["x"]).cuda()
    t = torch.from_numpy(f["t"]).cuda()
    d_xyz, d_rot, d_scale = net(x, t)
    loss = (d_xyz * torch.from_numpy(f["g_xyz"]).cuda()).sum()
    if torch.is_tensor(d_rot):
        loss = loss + (d_rot * torch.from_numpy(f["g_rot"]).cuda()).sum() + (
            d_scale * torch.from_numpy(f["g_scale"]).cuda()).sum()
    loss.backward()
    print(f"== {name} N={x.shape[0]}")
    for k, p in net.named_parameters():
        if "grad." + k not in f:
            continue
        g = p.grad.cpu().numpy().astype(np.float64)
        ref = f["grad." + k]
        e = np.abs(g - ref)
        m = max(np.abs(ref).max(), 1e-12)
        bad = np.argwhere(e > 1e-4 * m + 1e-7)
        print(f"{k:32s} {tuple(ref.shape)} rel {e.max() / m:.2e} bad {len(bad)}"
              + (f" rows {sorted(set(bad[:, 0].tolist()))[:12]}" + (f" cols {sorted(set(bad[:, 1].tolist()))[:12]}" if bad.shape[1] > 1 else "") if len(bad) else ""))
