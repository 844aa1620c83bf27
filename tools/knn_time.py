#!/usr/bin/env python3
"""Times dgs_knn_dist2 (distCUDA2 replacement, exact LDS-tiled all-pairs 3-NN) at init sizes:
python3 tools/knn_time.py [sizes...]  -> one JSON line (ms per call, median of 3 after a warm-up)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))

import torch  # noqa: E402


def main():
    from deformgs.gaussian_model import distCUDA2
    sizes = [int(s) for s in sys.argv[1:]] or [100_000, 300_000, 1_000_000]
    out = {}
    for n in sizes:
        pts = (torch.rand(n, 3, device="cuda", generator=torch.Generator(device="cuda").manual_seed(n)) * 2.6 - 1.3)
        distCUDA2(pts)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            distCUDA2(pts)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        out[str(n)] = sorted(ts)[1]
        print(n, out[str(n)], "ms", flush=True)
    print(json.dumps({"knn_dist2_ms": out}), flush=True)


if __name__ == "__main__":
    main()
