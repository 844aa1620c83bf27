"""CPU address audit of the deterministic blend backward's per-pair slots (tools/det_index_audit.py,
VERDICT r5 #4): on the bench lists (synth-100k at 800^2), ragged big-Gaussian lists longer than
k_tile_sort's 1024-entry LDS path, a forced overflow (clipped ranges), speculative headroom, both
binning orders (per-tile depth sort / global depth order), replayed prefixes from none to all. The
audit must also catch a dropped write (the kind of bug consistent with round 5's r5dd fault)."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
from helpers import _rect, oracle_run, scene

sys.path.insert(0, os.path.join(ROOT, "tools"))
import det_index_audit as dia  # noqa: E402


def _lists(N, H, W, cam, boost, seed):
    inputs, rs, _ = scene(N, H, W, cam_index=cam, scale_boost=boost, seed=seed)
    o, _ = oracle_run(inputs, rs)
    raw = o.preprocess_raw()
    radii = np.ceil(raw["radf"]).astype(np.int64) * (raw["radf"] > 0)
    dkey = raw["vz"].astype(np.float32).view(np.uint32).astype(np.int64)
    ranges, vals, T = dia.tile_lists(radii, raw["pxy"], raw["vz"], H, W, _rect)
    return ranges, vals, dkey, o.num_rendered


CASES = [("bench-100k", 100_000, 800, 800, 0, 0.0, 0), ("config1", 5000, 256, 256, 0, 0.0, 13),
         ("sparse", 300, 256, 256, 0, 0.0, 13),
         ("ragged-big", 2000, 61, 83, 3, 1.0, 13), ("long-lists", 3000, 128, 128, 1, 2.5, 5)]


@pytest.mark.parametrize("name,N,H,W,cam,boost,seed", CASES, ids=[c[0] for c in CASES])
def test_deterministic_slots_in_bounds_and_covered(name, N, H, W, cam, boost, seed):
    ranges, vals, dkey, nr = _lists(N, H, W, cam, boost, seed)
    P = len(vals)
    assert P == nr, (P, nr)  # the emulated lists are the oracle's own pair count
    lens = ranges[:, 1] - ranges[:, 0]
    if name == "long-lists":
        assert lens.max() > 1024  # k_tile_sort's long-list path
    rng = np.random.default_rng(1)
    caps = [P, max(1, int(0.7 * P)), P + 65536]  # exact, forced overflow, speculative headroom
    for tsort in (True, False):
        for cap in caps:
            for mode in ("zero", "all", "random"):
                bad = dia.audit(ranges, vals, dkey, cap, tsort=tsort, rng=rng, todo_mode=mode)
                assert not bad, (name, tsort, cap, mode, bad[:5])


def test_audit_catches_dropped_writes():
    ranges, vals, dkey, _ = _lists(300, 256, 256, 0, 0.0, 13)
    lens = ranges[:, 1] - ranges[:, 0]
    assert (lens == 1).any()  # single-entry tiles: a sparse scene
    for m in ("no_len1_pre", "skip_culled"):
        bad = dia.audit(ranges, vals, dkey, len(vals), tsort=True, rng=np.random.default_rng(2), mutate=m,
                        todo_mode="all")
        assert bad, m
