#!/usr/bin/env python3
"""Diagnostic: per-layer error of the saved hidden activations / relu masks of the fused MLP
(split-bf16 and exact-fp32) against the float64 oracle."""
import sys
import numpy as np
import torch
sys.path[:0] = ["tests", "tests/golden", "deformable-3d-gaussians_amd", "."]
from oracle import mlp_ref  # noqa: E402
from test_gpu_mlp import _net, VARIANTS  # noqa: E402

S_ROWS = [0, 256, 512, 768, 1120, 1376, 1632, 1888]
name, N = (sys.argv[1], int(sys.argv[2])) if len(sys.argv) > 2 else ("nonblender", 4099)
bl, d6, fork = VARIANTS[name]
rng = np.random.default_rng(N)
x = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
t = np.full((N, 1), 0.37, np.float32)
for exact in (False, True):
    net, w = _net(name, 77, exact)
    out, c = mlp_ref.forward(w, x, t, bl, d6)
    res = net(torch.from_numpy(x).cuda(), torch.from_numpy(t).cuda())
    packed, saved = res[0].grad_fn.saved_tensors if hasattr(res[0].grad_fn, "saved_tensors") else (None, None)
    if saved is None:  # d_xyz is a slice of the kernel output: walk to the fused node
        fn = res[0].grad_fn
        while fn is not None and not hasattr(fn, "saved_tensors"):
            fn = fn.next_functions[0][0]
        packed, saved = fn.saved_tensors
    Ns = (N + (31 if exact else 63)) // (32 if exact else 64) * (32 if exact else 64)
    sv = saved[: 2144 * Ns].view(2144, Ns).cpu().numpy()[:, :N]
    for L in range(8):
        ref = np.maximum(c["z"][L], 0).T  # (256, N)
        got = sv[S_ROWS[L]:S_ROWS[L] + 256]
        err = np.abs(got - ref)
        flips = int(((got > 0) != (ref > 0)).sum())
        i = np.unravel_index(err.argmax(), err.shape)
        print(("exact" if exact else "split"), "H%d" % L, "max err %.2e at (unit %d, point %d) ref %.4e got %.4e; relu flips %d" % (
            err.max(), i[0], i[1], ref[i], got[i], flips), flush=True)
