"""CPU address audit of the deterministic blend backward (raster.hip): the index
expressions of k_tile_sort<true> (the position map `pre`), k_blend_bwd2<DEPTH, true> (per-pair slot
writes: zeros past the replayed prefix, zeros for tile-culled entries, the reduced sums of the replayed
ones) and k_rect_gather (the per-Gaussian slot reads of rect_walk), replayed on real tile lists, against
the buffer det_layout lays out for the forward's pair capacity:

  * every `pre` and slot index written lies inside the buffer (< det_cap) and inside its tile's clipped
    range [min(start, cap), min(end, cap));
  * every `vals` read lies inside the placed list (< cap);
  * every slot the gather reads (index-order positions < cap) is written by the backward exactly once,
    so no stale word from an earlier step enters a sum.

The lists come from the oracle's own preprocess (radii, pixel centres, view depths) through the
rasterizer's tile rectangle (helpers._rect, the C expression), in index order with the per-tile stable
depth sort (the default) or in global depth order (DGS_TILE_SORT=0: slot = list position). Capacities:
exact, forced overflow (the deferred count's clipped ranges), speculative headroom. The replayed prefix
(todo_total, the tile's max last contributor) is swept over 0, 1, the whole list and random values,
and entries are culled at random. `mutate` drops one write the kernels make (e.g. k_tile_sort's
len == 1 position), which the audit must then report: the round-5 r5dd illegal access (an intermediate
build of the rework) is consistent with exactly such a missing `pre` write."""
import numpy as np


def tile_lists(radii, pxy, depth, H, W, rect):
    """(ranges (T, 2), vals (P,)) in index order per tile, and each Gaussian's depth key."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    live = radii > 0
    x0, y0, x1, y1 = rect(pxy[:, 0], pxy[:, 1], radii, gx, gy)
    tiles, gids = [], []
    for g in np.nonzero(live)[0]:
        if x1[g] <= x0[g] or y1[g] <= y0[g]:
            continue
        ys, xs = np.meshgrid(np.arange(y0[g], y1[g]), np.arange(x0[g], x1[g]), indexing="ij")
        t = (ys * gx + xs).ravel()
        tiles.append(t)
        gids.append(np.full(t.shape, g, np.int64))
    T = gx * gy
    if not tiles:
        return np.zeros((T, 2), np.int64), np.zeros(0, np.int64), T
    tiles = np.concatenate(tiles)
    gids = np.concatenate(gids)
    o = np.lexsort((gids, tiles))  # tile-major, index order within a tile
    tiles, gids = tiles[o], gids[o]
    cnt = np.bincount(tiles, minlength=T)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    return np.stack([start, start + cnt], 1), gids, T


def audit(ranges, vals, dkey, cap, tsort=True, rng=None, mutate=None, todo_mode="random"):
    """Replays the index expressions; returns a list of violations (empty = clean)."""
    rng = rng or np.random.default_rng(0)
    bad = []
    det_cap = max(cap, 1)             # det_layout(c, cap): slots and position map for the forward's cap
    slot_writes = np.zeros(det_cap, np.int64)
    pre = np.full(det_cap, -1, np.int64)  # -1: never written (stale)
    placed = min(cap, len(vals))      # k_rect_place: pos < cap
    # k_tile_sort<true>: a = min(rg.x, cap), b = min(rg.y, cap)
    if tsort:
        for t, (x, y) in enumerate(ranges):
            a, b = min(x, cap), min(y, cap)
            n = b - a
            if n == 1 and mutate != "no_len1_pre":
                pre[a] = 0                                   # if (PRE && len == 1 && tid == 0) pre[a] = 0u
            if n <= 1:
                continue
            keys = dkey[vals[a:b]]
            order = np.argsort(keys, kind="stable")          # sorted position p <- index-order position q
            if np.all(order == np.arange(n)) and mutate == "no_sorted_pre":
                continue                                     # (the early return without its pre writes)
            for p in range(n):
                idx = a + p
                if idx >= det_cap:
                    bad.append(("pre write out of bounds", t, idx))
                else:
                    pre[idx] = order[p]
    for t, (x, y) in enumerate(ranges):
        rx, ry = min(x, cap), min(y, cap)                    # range.x / range.y clipped to cap
        n = ry - rx
        if todo_mode == "all":
            todo = n
        elif todo_mode == "zero":
            todo = 0
        else:
            todo = int(rng.integers(0, n + 1)) if n else 0
        def slot_of(lp):
            if lp >= det_cap:
                bad.append(("pre read out of bounds", t, lp))
                return None
            if not tsort:
                return lp
            q = pre[lp]
            if q < 0:
                bad.append(("stale pre word read", t, lp))
                return None
            return rx + q
        def write(lp):
            s = slot_of(lp)
            if s is None:
                return
            if not (rx <= s < ry) or s >= det_cap:
                bad.append(("slot write out of range", t, int(s)))
                return
            slot_writes[s] += 1
        for lp in range(rx + todo, ry):                      # zeros past the replayed prefix
            write(lp)
        end = rx + todo
        culled = rng.random(todo) < 0.2
        for prog in range(todo):                             # vals[end - prog - 1]; culled: zeros, kept: sums
            lp = end - prog - 1
            if not (rx <= lp < placed):
                bad.append(("vals read out of range", t, lp))
            if mutate == "skip_culled" and culled[prog]:
                continue
            write(lp)
    # k_rect_gather: rect_walk's positions in the placement order, read if pos < cap
    for pos in range(min(len(vals), cap)):
        if slot_writes[pos] != 1:
            bad.append(("gather reads a slot written %d times" % slot_writes[pos], -1, pos))
    return bad
