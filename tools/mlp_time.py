#!/usr/bin/env python3
"""Times the fused deformation MLP alone (forward, backward dX, dW) at the bench size with the
library's own HIP-event kernel timers, for the split-bf16 and the exact-fp32 arithmetic:
python3 tools/mlp_time.py [--n N] [--iters K]."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--n", type=int, default=100_000)
    a = ap.parse_args()
    from deformgs import _lib
    from deformgs.deform_network import DeformNetworkBaseline
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    res = {}
    for exact in (False, True):
        torch.manual_seed(0)
        net = DeformNetworkBaseline(is_blender=True, exact_fp32=exact).to(dev)
        x = torch.rand(a.n, 3, device=dev) * 2.6 - 1.3
        t = torch.full((1, 1), 0.3, device=dev).expand(a.n, -1)  # one frame time (training path)
        for it in range(a.iters + 2):
            if it == 2:
                torch.cuda.synchronize()
                lib.dgs_timing_reset()
                lib.dgs_timing_select(b"")
                lib.dgs_timing_enable(1)
            d_xyz, d_rot, d_s = net(x, t)
            (d_xyz.sum() + d_rot.square().sum() + d_s.abs().sum()).backward()
        torch.cuda.synchronize()
        lib.dgs_timing_enable(0)
        r = {}
        for k in ("mlp_fwd", "mlp_bwd", "mlp_dw", "mlp_dw_reduce", "mlp_tgrad"):
            n = _lib.I(0)
            ms = lib.dgs_timing_query(k.encode(), n)
            r[k] = ms / max(n.value, 1)
        r["total"] = sum(r.values())
        lib.dgs_timing_reset()
        lib.dgs_timing_enable(1)
        with torch.no_grad():  # inference: no saved activations, per-point timenet
            for _ in range(a.iters):
                net(x, t)
        torch.cuda.synchronize()
        lib.dgs_timing_enable(0)
        n = _lib.I(0)
        r["fwd_nosave"] = lib.dgs_timing_query(b"mlp_fwd", n) / max(n.value, 1)
        res["exact" if exact else "split"] = r
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
