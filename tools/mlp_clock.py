#!/usr/bin/env python3
"""In-kernel clock of the split-bf16 MLP kernels (MI355X_MICROARCH.md 'DVFS give-back' item 6): runs
the deformation MLP forward + backward at the bench size back to back for --seconds, then reads the
per-workgroup shader-clock / real-time stamps of the last k_fwd, k_bwd and k_dws launches. Needs a
diagnostic library built with -DDGS_CLOCK_STAMPS (tools/build_diag.sh clk=-DDGS_CLOCK_STAMPS) in DGS_LIB.

MFMA-dense kernels run below the 2.4 GHz the bf16 peak is quoted at; `mfma_frac_at_clock` rescales a
kernel's fraction of the nominal split ceiling to the clock it actually held.
python3 tools/mlp_clock.py [--n 100000] [--seconds 3]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

NOMINAL_GHZ = 2.4
CLK_BLOCKS = 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    from deformgs import _lib
    from deformgs.deform_network import DeformNetworkBaseline
    lib = _lib.load()
    fn = lib.dgs_debug_clock
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong)]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = DeformNetworkBaseline(is_blender=True).to(dev)
    x = torch.rand(a.n, 3, device=dev) * 2.6 - 1.3
    t = torch.full((1, 1), 0.3, device=dev).expand(a.n, -1)
    lib.dgs_timing_reset()
    lib.dgs_timing_select(b"")
    lib.dgs_timing_enable(1)
    t0 = time.time()
    iters = 0
    while time.time() - t0 < a.seconds:
        for _ in range(10):
            d_xyz, d_rot, d_s = net(x, t)
            (d_xyz.sum() + d_rot.square().sum() + d_s.abs().sum()).backward()
        torch.cuda.synchronize()
        iters += 10
    lib.dgs_timing_enable(0)
    out = {"n": a.n, "iters": iters}
    buf = (ctypes.c_ulonglong * (6 * CLK_BLOCKS))()
    for k, name, tname in ((0, "k_fwd", "mlp_fwd"), (1, "k_bwd", "mlp_bwd"), (2, "k_dws", "mlp_dw")):
        assert fn(k, CLK_BLOCKS, buf) == 0
        raw = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 6)
        # the last launch's workgroups: real-time start within 10 ms of the latest start
        ok = (raw[:, 3] > raw[:, 2]) & (raw[:, 2] + 1_000_000 > raw[:, 2].max())
        if not ok.any():  # the kernel wrote no stamps (k_fwd8, the default training forward, has none)
            out[name] = "no stamps"
            continue
        v = raw[ok].astype(np.float64)
        cyc, tick = v[:, 1] - v[:, 0], v[:, 3] - v[:, 2]
        ghz = cyc / tick * 0.1
        n = _lib.I(0)
        ms = lib.dgs_timing_query(tname.encode(), n) / max(n.value, 1)
        span = (v[:, 3].max() - v[:, 2].min()) / 100.0
        # CU key: XCC id, SE / SH / CU fields of HW_ID (bits 8..15)
        hw = raw[ok][:, 4]
        cu = ((hw >> np.uint64(32)) << np.uint64(8)) | ((hw >> np.uint64(8)) & np.uint64(0xFF))
        keys, inv = np.unique(cu, return_inverse=True)
        busy = np.bincount(inv, weights=tick) / 100.0
        nblk = np.bincount(inv)
        start0 = v[:, 2].min()
        first = np.array([v[inv == c, 2].min() for c in range(len(keys))]) - start0
        last = np.array([v[inv == c, 3].max() for c in range(len(keys))]) - start0
        out[name] = {"blocks": int(len(v)), "ghz_median": float(np.median(ghz)),
                     "kernel_ms": ms, "span_us": span, "clock_frac_of_nominal": float(np.median(ghz)) / NOMINAL_GHZ,
                     "block_us_pct": [float(np.percentile(tick, q)) / 100.0 for q in (0, 10, 50, 90, 100)],
                     "cus": int(len(keys)), "blocks_per_cu": np.bincount(nblk).tolist(),
                     "cu_busy_us_pct": [float(np.percentile(busy, q)) for q in (0, 10, 50, 90, 100)],
                     "cu_first_start_us_pct": [float(np.percentile(first, q)) / 100.0 for q in (0, 50, 100)],
                     "cu_last_end_us_pct": [float(np.percentile(last, q)) / 100.0 for q in (0, 50, 100)],
                     "busy_frac": float(busy.sum() / (len(keys) * span))}
        if k == 2:  # per workgroup, in launch order (jobs own contiguous block ranges)
            order = np.argsort(np.nonzero(ok)[0])
            out[name]["block_us"] = [round(float(u) / 100.0, 1) for u in tick[order]]
        xcc = (hw >> np.uint64(32)).astype(np.int64)
        out[name]["per_xcc"] = {int(x): {"blocks": int((xcc == x).sum()), "block_us_median": float(np.median(tick[xcc == x])) / 100.0,
                                         "ghz_median": float(np.median(ghz[xcc == x])),
                                         "last_end_us": float(v[xcc == x, 3].max() - start0) / 100.0}
                                for x in np.unique(xcc)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
