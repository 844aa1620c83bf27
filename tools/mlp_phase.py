#!/usr/bin/env python3
"""Per-phase cycle breakdown of the split-bf16 MLP forward from the DGS_MLP_PROFILE build
(tools/build_diag.sh prof=-DDGS_MLP_PROFILE; run with DGS_LIB=.../libdgs_prof.so):
stamps 0 start, 1 inputs staged, 4+2L / 5+2L after layer L's GEMM / epilogue, 20 heads, 21 end."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from deformgs import _lib
    from deformgs.deform_network import DeformNetworkBaseline
    lib = _lib.load()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    dev = torch.device("cuda", 0)
    nb = (N + 63) // 64
    prof = torch.zeros(nb * 64, dtype=torch.int64, device=dev)
    lib.dgs_mlps_set_prof.argtypes = [ctypes.c_void_p]
    lib.dgs_mlps_set_prof(ctypes.c_void_p(prof.data_ptr()))
    torch.manual_seed(0)
    net = DeformNetworkBaseline(is_blender=True).to(dev)
    x = torch.rand(N, 3, device=dev) * 2.6 - 1.3
    t = torch.full((1, 1), 0.3, device=dev).expand(N, -1)  # one frame time: the folded training path
    for _ in range(3):
        out = net(x, t)
        (out[0].sum() + out[1].sum() + out[2].sum()).backward()
    torch.cuda.synchronize()
    p = prof.view(nb, 64).cpu().numpy().astype(np.float64)
    p = p[(p[:, 0] > 0) & (p[:, 21] > 0)]  # persistent k_fwd: one row per workgroup (its last block)
    nb = len(p)
    names = {0: "start", 1: "inputs"}
    for L in range(8):
        names[4 + 2 * L] = f"L{L} gemm"
        names[5 + 2 * L] = f"L{L} epi"
    names[20] = "heads"
    names[21] = "out"
    order = [0, 1] + [k for L in range(8) for k in (4 + 2 * L, 5 + 2 * L)] + [20, 21]
    tot = p[:, 21] - p[:, 0]
    print(f"blocks {nb}, mean block cycles {tot.mean():.0f}")
    for a, b in zip(order[:-1], order[1:]):
        d = p[:, b] - p[:, a]
        print(f"  {names[b]:10s} {d.mean():9.0f} cyc  ({100 * d.mean() / tot.mean():5.1f}%)")
    # layer 3 detail: every wave's GEMM end, then wave 0 through the epilogue
    L3 = p[:, 9]
    wend = np.stack([p[:, 22 + w] - L3 for w in range(16)], 1)
    print("L3 per-wave GEMM end (mean over blocks):", " ".join(f"{v:.0f}" for v in wend.mean(0)))
    print(f"L3 slowest wave GEMM end {wend.max(1).mean():.0f}, fastest {wend.min(1).mean():.0f}")
    for nm, a_, b_ in (("barrier1", 10, 56), ("bias/relu/mask/saved", 56, 54), ("split+LDS", 54, 55), ("barrier2", 55, 11)):
        print(f"  L3 {nm:22s} {(p[:, b_] - p[:, a_]).mean():8.0f} cyc")
    clk = (p[:, 61] - p[:, 0]) / np.maximum(p[:, 60] - p[:, 60].min() + 1, 1)
    start = p[:, 0] - p[:, 0].min()
    end = p[:, 21] - p[:, 0].min()
    print(f"kernel span {end.max():.0f} cyc; blocks start spread {np.percentile(start, [0, 50, 100])}")


if __name__ == "__main__":
    main()
