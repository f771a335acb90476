"""The forward's depth sort on its own (csrc/radix.hip radix_sort over 32 bits, 4 x 8-bit LSD
passes, via the parity helper gsr_debug_depth_sort): the first half of the reference's tile|depth
key sort (rasterizer_impl.cu:306-311, cub::DeviceRadixSort::SortPairs, stable).

Cases: ties, ranges crossing powers of two, the widest range (tiny and huge floats together), one
distinct key, culled keys (0xFFFFFFFF, sorted last) mixed in or alone, digit boundaries, and sizes
around the 2,048-key chunk.  Expected order: numpy's stable argsort of the u32 keys -- exactly the
reference's stable sort over the full 32 bits.
"""
import numpy as np
import pytest
import torch

CULLED = np.uint32(0xFFFFFFFF)


def _floats(r, n, lo, hi):
    return np.exp(r.uniform(np.log(lo), np.log(hi), n)).astype(np.float32).view(np.uint32)


def _cases():
    r = np.random.default_rng(11)
    yield "bench-range", _floats(r, 300_000, 1.4, 6.6)
    yield "scene-range", _floats(r, 100_003, 0.2, 150.0)
    yield "widest", _floats(r, 50_000, 1e-37, 3e38)
    k = _floats(r, 70_000, 0.5, 4.0)
    k[r.random(70_000) < 0.3] = CULLED
    yield "culled-mix", k
    yield "ties", r.choice(_floats(r, 37, 0.3, 9.0), 200_000)
    yield "one-key", np.full(5_000, np.float32(2.0).view(np.uint32), np.uint32)
    yield "one-key+culled", np.where(r.random(4_097) < 0.5, np.float32(7.25).view(np.uint32), CULLED).astype(np.uint32)
    yield "all-culled", np.full(3_000, CULLED, np.uint32)
    yield "power-of-two-edges", np.float32([1.0, 2.0, 4.0, 0.5]).view(np.uint32)[r.integers(0, 4, 9_000)]
    # adjacent bit patterns across a digit boundary
    base = np.uint32(np.float32(3.0).view(np.uint32) & ~np.uint32(1023))
    yield "digit-boundary", (base + r.integers(1000, 1050, 20_000)).astype(np.uint32)
    for n in (1, 2, 2047, 2048, 2049, 4096 * 3 + 5):
        yield f"n={n}", _floats(r, n, 0.2, 100.0)


CASES = list(_cases())


@pytest.mark.gpu
@pytest.mark.parametrize("name,keys", CASES, ids=[c[0] for c in CASES])
def test_depth_sort_is_stable_argsort(name, keys):
    from diff_gaussian_rasterization import _C
    kt = torch.from_numpy(keys.view(np.int32).copy()).cuda()
    ids = _C.depth_sort(kt).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(ids, np.argsort(keys, kind="stable").astype(np.uint32), err_msg=name)


@pytest.mark.gpu
def test_depth_sort_full_size_and_repeat():
    """BASELINE config-2 size (1M keys, a quarter culled) and bitwise-identical repeats."""
    from diff_gaussian_rasterization import _C
    r = np.random.default_rng(5)
    keys = _floats(r, 1_000_000, 1.4, 6.6)
    keys[r.random(keys.size) < 0.25] = CULLED
    kt = torch.from_numpy(keys.view(np.int32).copy()).cuda()
    a = _C.depth_sort(kt)
    b = _C.depth_sort(kt)
    np.testing.assert_array_equal(a.cpu().numpy().view(np.uint32), np.argsort(keys, kind="stable"))
    assert torch.equal(a, b)
