#!/usr/bin/env python3
"""Per-wave phase timeline of k_fwd8 (8 waves) from the DGS_MLP_PROFILE build (tools/build_diag.sh
prof=-DDGS_MLP_PROFILE [-DDGS_PROF_LAYER=L]; run with DGS_LIB=.../libdgs_prof.so): the first block of
every workgroup stamps 0 start, 1 inputs staged, 20 end of the trunk, and for layer DGS_PROF_LAYER per
wave w: 24+w GEMM start, 32+w GEMM end, 40+w epilogue statistics done (before the WAR wait), 48+w WAR
wait done, 56+w LDS image written + signalled. Prints medians over workgroups, cycles relative to the
layer's first GEMM start."""
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
    t = torch.full((1, 1), 0.3, device=dev).expand(N, -1)
    for _ in range(3):
        prof.zero_()
        out = net(x, t)
        torch.cuda.synchronize()
    P = prof.view(nb, 64).cpu().numpy().astype(np.int64)
    wg = P[(P[:, 0] > 0) & (P[:, 24:32].min(1) > 0) & (P[:, 56:64].min(1) > 0)]
    print(f"workgroups stamped: {len(wg)}")
    ref = wg[:, 24:32].min(1, keepdims=True)
    rel = lambda k: np.median(wg[:, k:k + 8] - ref, axis=0)  # noqa: E731
    names = [("gemm start", 24), ("gemm end", 32), ("stats done", 40), ("WAR done", 48), ("signalled", 56)]
    print("wave " + " ".join(f"{w:>7d}" for w in range(8)))
    for n, k in names:
        print(f"{n:10s} " + " ".join(f"{v:7.0f}" for v in rel(k)))
    g = np.median(wg[:, 32:40] - wg[:, 24:32], axis=0)
    e1 = np.median(wg[:, 40:48] - wg[:, 32:40], axis=0)
    war = np.median(wg[:, 48:56] - wg[:, 40:48], axis=0)
    e2 = np.median(wg[:, 56:64] - wg[:, 48:56], axis=0)
    print("gemm dur   " + " ".join(f"{v:7.0f}" for v in g))
    print("stats dur  " + " ".join(f"{v:7.0f}" for v in e1))
    print("WAR wait   " + " ".join(f"{v:7.0f}" for v in war))
    print("write+sig  " + " ".join(f"{v:7.0f}" for v in e2))
    print(f"block: inputs {np.median(wg[:, 1] - wg[:, 0]):.0f}, trunk {np.median(wg[:, 20] - wg[:, 1]):.0f} cycles")


if __name__ == "__main__":
    main()
