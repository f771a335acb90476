"""CPU checks of the flip attribution the full-size GPU parity tests rely on
(common.flip_gaussians / check_grad_attributed)."""
import numpy as np
import pytest

import common


@pytest.fixture(scope="module")
def oracle_case():
    case = common.make_case(P=1000, H=64, W=80)
    o, _ = common.run_oracle(case, backward=False)
    return case, o


def test_flip_gaussians_is_the_pixel_walk(oracle_case):
    case, o = oracle_case
    W, H, P = case["W"], case["H"], 1000
    nc = o.get("n_contrib").astype(np.int64)
    vals, ranges = o.get("vals"), o.get("ranges")
    pix = int(np.argmax(nc))  # the longest walk
    flip = np.zeros(W * H, dtype=bool)
    flip[pix] = True
    got = common.flip_gaussians(flip, nc, nc, vals, ranges, W, H, P)
    y, x = divmod(pix, W)
    t = (y // 16) * ((W + 15) // 16) + x // 16
    want = np.zeros(P, dtype=bool)
    want[vals[ranges[t, 0]:ranges[t, 0] + nc[pix]]] = True
    assert nc[pix] > 0 and np.array_equal(got, want)
    # the larger of the two walks counts (the GPU may have walked one entry further)
    nc2 = nc.copy()
    nc2[pix] += 1
    got2 = common.flip_gaussians(flip, nc2, nc, vals, ranges, W, H, P)
    assert got2.sum() >= got.sum() and np.all(got2[got])
    assert not common.flip_gaussians(np.zeros_like(flip), nc, nc, vals, ranges, W, H, P).any()


def test_check_grad_attributed():
    rng = np.random.default_rng(0)
    ref = rng.normal(size=(100, 3)).astype(np.float32)
    affected = np.zeros(100, dtype=bool)
    affected[7] = True
    hip = ref.copy()
    hip[7, 1] += 1e-3 * np.abs(ref).max()  # inside a flipped walk: allowed
    st = common.check_grad_attributed("t", hip, ref, affected)
    assert st["attributed_rows"] == 1 and st["unattributed_rows"] == 0
    hip[9, 0] += 1e-3 * np.abs(ref).max()  # outside: must fail
    with pytest.raises(AssertionError):
        common.check_grad_attributed("t", hip, ref, affected)
    hip = ref.copy()
    hip[7, 2] += 1e-2 * np.abs(ref).max()  # inside, but beyond the attributed bound
    with pytest.raises(AssertionError):
        common.check_grad_attributed("t", hip, ref, affected)
