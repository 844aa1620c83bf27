"""The binning's own stable LSD radix sort (csrc/radix.hip, SURVEY §8 row R3: replaces the upstream
rasterizer's cub::DeviceRadixSort::SortPairs) through the dgs_debug_sort_pairs test hook, against
numpy's stable argsort on the same keys: keys and values bit-exact. Covers the onesweep scatter
(decoupled look-back over several workgroups, both tile sizes), passes in which every key carries
the same digit (the exponent byte of depths within one octave), partial last passes (end_bit not a
multiple of 8), 16-bit tile keys, ragged and tiny sizes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sort(keys, end_bit):
    from deformgs import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    kt = torch.int32 if keys.dtype == np.uint32 else torch.int16
    k0 = torch.from_numpy(keys.view(np.int32 if keys.dtype == np.uint32 else np.int16).copy()).to(dev)
    k1 = torch.empty_like(k0)
    n = keys.shape[0]
    v0 = torch.arange(n, dtype=torch.int32, device=dev)
    v1 = torch.empty_like(v0)
    assert k0.dtype == kt
    rc = lib.dgs_debug_sort_pairs(k0.data_ptr(), k1.data_ptr(), v0.data_ptr(), v1.data_ptr(), n, keys.itemsize,
                                  end_bit, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.dgs_last_error()
    torch.cuda.synchronize()
    return k0.cpu().numpy().view(keys.dtype), v0.cpu().numpy().view(np.uint32)


def _expect(keys, end_bit):
    mask = (1 << end_bit) - 1 if end_bit < 8 * keys.itemsize else (1 << (8 * keys.itemsize)) - 1
    order = np.argsort(keys.astype(np.uint64) & mask, kind="stable").astype(np.uint32)
    return keys[order], order


@pytest.mark.parametrize("n", [1, 7, 1000, 4099, 100_000, 700_003])
@pytest.mark.parametrize("kind", ["random", "one_octave_depths", "wide_depths", "constant"])
def test_sort32_matches_stable_argsort(n, kind):
    rng = np.random.default_rng(n)
    if kind == "random":
        keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    elif kind == "one_octave_depths":  # float bits of depths in [2, 4): top byte 0x40 for every key
        keys = rng.uniform(2.0, 4.0, n).astype(np.float32).view(np.uint32)
    elif kind == "wide_depths":
        keys = np.exp(rng.uniform(np.log(0.2), np.log(100.0), n)).astype(np.float32).view(np.uint32)
    else:  # every pass takes the copy path
        keys = np.full(n, 0x40490fdb, dtype=np.uint32)
    # duplicates so stability matters
    keys[rng.integers(0, n, n // 3)] = keys[rng.integers(0, n, n // 3)]
    k, v = _sort(keys, 32)
    ek, ev = _expect(keys, 32)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)


@pytest.mark.parametrize("end_bit", [12, 16])
def test_sort16_tile_keys(end_bit):
    rng = np.random.default_rng(end_bit)
    n = 300_001
    keys = rng.integers(0, 1 << end_bit, n).astype(np.uint16)
    k, v = _sort(keys, end_bit)
    ek, ev = _expect(keys, end_bit)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)


def test_sort32_partial_last_pass():
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 1 << 20, 50_000).astype(np.uint32)
    k, v = _sort(keys, 20)
    ek, ev = _expect(keys, 20)
    assert np.array_equal(k, ek) and np.array_equal(v, ev)
