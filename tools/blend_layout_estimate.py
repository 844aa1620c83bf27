#!/usr/bin/env python3
"""Work estimate for the blend backward's parallelisation, on the bench scene
(synth-100k, 800x800, camera 0) from the CPU oracle's forward (oracle/raster_ref.c).

Counts, per 16x16 tile, the list positions the backward must replay (todo = the tile's largest
last-contributor position + 1) and every (pixel, Gaussian) pair that takes part (power <= 0,
alpha >= 1/255, position below the pixel's own last contributor), then prices two layouts:
  pixel-parallel (k_blend_bwd2): per 128-pixel half-tile wave and Gaussian, the full path when any
    of its 128 pixels takes part, the skip path otherwise;
  per-Gaussian (Taming-3DGS style): lanes own 64 consecutive list positions, the tile's 256 pixels
    stream through them in a 64-deep lane pipeline (256 + 63 steps per bucket), no skipping.
Test infrastructure (reads the oracle; never on the product path)."""
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "deformable-3d-gaussians_amd"), ROOT, os.path.join(ROOT, "tests")]
from helpers import oracle_run, scene  # noqa: E402

N, H, W = 100_000, 800, 800
inputs, rs, _ = scene(N, H, W, cam_index=0)
o, _ = oracle_run(inputs, rs, None, None)
geo = o.geometry()
xy, co, dep = geo["xy"], geo["conic_opacity"], geo["depth"]
_, ncon = o.pixel_state()
radii = o.radii
gx = gy = 50
idx = np.nonzero(radii > 0)[0]
f = np.float32
px, py, r = xy[idx, 0], xy[idx, 1], radii[idx].astype(f)
x0 = np.minimum(gx, np.maximum(0, np.trunc((px - r) / f(16)))).astype(int)
y0 = np.minimum(gy, np.maximum(0, np.trunc((py - r) / f(16)))).astype(int)
x1 = np.minimum(gx, np.maximum(0, np.trunc((px + r + f(15)) / f(16)))).astype(int)
y1 = np.minimum(gy, np.maximum(0, np.trunc((py + r + f(15)) / f(16)))).astype(int)
order = idx[np.argsort(dep[idx], kind="stable")]
rect = {g: (a, b, c, d) for g, a, b, c, d in zip(idx, x0, y0, x1, y1)}
lists = [[] for _ in range(gx * gy)]
for g in order:
    a, b, c, d = rect[g]
    for ty in range(b, d):
        for tx in range(a, c):
            lists[ty * gx + tx].append(g)
print("pairs", sum(len(L) for L in lists), "oracle num_rendered", o.num_rendered)
t0 = time.time()
tot_todo = buckets = act_wg = skip_wg = act_pairs = 0
todos = []
for t in range(gx * gy):
    L = lists[t]
    if not L:
        continue
    tx, ty = t % gx, t // gx
    nc = ncon[ty * 16:ty * 16 + 16, tx * 16:tx * 16 + 16]
    todo = int(nc.max())
    tot_todo += todo
    buckets += math.ceil(todo / 64)
    todos.append(todo)
    if todo == 0:
        continue
    g = np.array(L[:todo])
    pxs = (tx * 16 + np.arange(16)).astype(f)
    pys = (ty * 16 + np.arange(16)).astype(f)
    dx = xy[g, 0][:, None, None] - pxs[None, None, :]
    dy = xy[g, 1][:, None, None] - pys[None, :, None]
    c = co[g]
    power = -0.5 * (c[:, 0, None, None] * dx * dx + c[:, 2, None, None] * dy * dy) - c[:, 1, None, None] * dx * dy
    alpha = np.minimum(0.99, c[:, 3, None, None] * np.exp(power))
    act = (power <= 0) & (alpha >= 1 / 255) & (np.arange(todo)[:, None, None] < nc[None])
    act_pairs += int(act.sum())
    for h in range(2):  # the two 16x8 half-tile waves of k_blend_bwd2
        a = act[:, 8 * h:8 * h + 8, :].reshape(todo, -1).any(1)
        act_wg += int(a.sum())
        skip_wg += int((~a).sum())
todos = np.array(todos)
print(f"({time.time() - t0:.1f} s)")
print(f"list positions replayed (sum of todo) {tot_todo}; todo per tile mean {todos.mean():.1f}, p90 "
      f"{np.percentile(todos, 90):.0f}, max {todos.max()}")
print(f"(pixel, Gaussian) pairs taking part {act_pairs}")
pp_full, pp_skip = 166, 47  # k_blend_bwd2 wave-instructions per (wave, Gaussian): full / skip path
pp = act_wg * pp_full + skip_wg * pp_skip
print(f"pixel-parallel: (wave, Gaussian) full path {act_wg}, skipped {skip_wg} (full {act_wg / (act_wg + skip_wg):.3f}); "
      f"pixel slots in full-path waves {act_wg * 128} ({act_pairs / (act_wg * 128):.2f} used); "
      f"~{pp / 1e6:.0f} M wave-instructions")
lane_steps = buckets * (256 + 63) * 64
pg_instr = 60  # per (lane, step): the same per-pair arithmetic unpacked, no reduction, 4 lane shifts
print(f"per-Gaussian: {buckets} buckets x 319 steps x 64 lanes = {lane_steps / 1e6:.0f} M lane-steps "
      f"({act_pairs / lane_steps:.2f} used); ~{lane_steps * pg_instr / 64 / 1e6:.0f} M wave-instructions "
      f"at {pg_instr} per step")
