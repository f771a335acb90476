"""The forward's depth sort on its own (csrc/radix.hip radix_sort over 32 bits: three 9-bit LSD
passes, the third relative to the smallest key other than 0xFFFFFFFF, or four 8-bit passes when the
keys span too wide a range -- via the parity helper gsr_debug_depth_sort): the first half of the
reference's tile|depth key sort (rasterizer_impl.cu:306-311, cub::DeviceRadixSort::SortPairs, stable).

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


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [False, True])
def test_depth_sort_both_modes(wide):
    """The same keys through the three-pass sort (range fits) and the forced four-pass sort."""
    from diff_gaussian_rasterization import _C
    r = np.random.default_rng(17)
    keys = _floats(r, 250_000, 0.25, 40.0)
    keys[r.random(keys.size) < 0.1] = CULLED
    kt = torch.from_numpy(keys.view(np.int32).copy()).cuda()
    was = _C.depth_wide()
    _C.set_depth_wide(wide)
    try:
        ids = _C.depth_sort(kt).cpu().numpy().view(np.uint32)
    finally:
        _C.set_depth_wide(was)
    np.testing.assert_array_equal(ids, np.argsort(keys, kind="stable").astype(np.uint32))


def _wide_case():
    """Config 1's camera with 4,000 Gaussians whose depths span 0.3 ... 50,000 along view 0's ray (beyond
    the three-pass sort's factor of ~2^16), and the oracle on it."""
    import common
    case = common.make_case(P=4000, H=256, W=256)
    cam = case["cam"]
    g = torch.Generator().manual_seed(3)
    P = 4000
    # along the camera's view ray: depth d log-uniform in [0.3, 5e4], lateral offsets within the view
    C = torch.tensor(cam.camera_center.numpy(), dtype=torch.float64)
    fwd = -C / C.norm()
    up = torch.tensor([0.0, 1.0, 0.0], dtype=torch.float64)
    right = torch.linalg.cross(fwd, up)
    right /= right.norm()
    up2 = torch.linalg.cross(right, fwd)
    d = torch.exp(torch.rand(P, generator=g, dtype=torch.float64) * (np.log(5e4) - np.log(0.3)) + np.log(0.3))
    lat = (torch.rand(P, 2, generator=g, dtype=torch.float64) - 0.5) * 0.6 * d[:, None]
    means = C + d[:, None] * fwd + lat[:, :1] * right + lat[:, 1:] * up2
    sc = case["scene"]
    sc["means3D"] = means.float().contiguous()
    sc["scales"] = (sc["scales"] * (d[:, None].float() * 0.5)).contiguous()
    o, _ = common.run_oracle(case, nthreads=8, backward=False)
    assert o.num_rendered > 0
    return case, o


def _forward_bit_exact(case, o, tag):
    """One rasterize_gaussians forward of `case`, checked against the oracle `o`: keys / values /
    ranges / radii bit for bit, the image through check_render.  Returns the depth-sort passes it ran."""
    import common
    from diff_gaussian_rasterization import _C
    dev = torch.device("cuda:0")
    cam, sc, H, W = case["cam"], case["scene"], case["H"], case["W"]
    P = sc["means3D"].shape[0]
    e = torch.Tensor([])
    s = {k: v.to(dev) for k, v in sc.items()}
    L, color, radii, geom, binning, img, inv = _C.rasterize_gaussians(
        case["bg"].to(dev), s["means3D"], e, s["opacities"], s["scales"], s["rotations"], 1.0, e,
        cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.tanfovx, cam.tanfovy, H, W,
        s["shs"], 3, cam.camera_center.to(dev), False, False, False)
    torch.cuda.synchronize()
    passes = _C.last_depth_passes()
    assert L == o.num_rendered, tag
    np.testing.assert_array_equal(radii.cpu().numpy(), o.radii)
    keys, vals, ranges = _C.sorted_keys(geom, binning, img, P, L, W, H)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))
    common.check_render(tag, {"color": color.cpu().numpy(), "invdepth": inv.cpu().numpy()},
                        {"color": o.color, "invdepth": o.invdepth})
    return passes


@pytest.mark.gpu
def test_forward_with_too_wide_depth_range_reruns_bit_exact():
    """A forward whose visible depths span 0.3 ... 50,000 (beyond the three-pass sort's factor of
    ~2^16): the pass-1 range reduction flags it in the pinned word read with num_rendered, that call's
    depth sort re-runs in four 8-bit passes, and keys / values / ranges / radii / image match the oracle
    bit for bit (the render by check_render).  Nothing sticks (VERDICT r05 "next" #6): a narrow-range
    forward right after it runs three passes, bit-exact too, and the wide one again four."""
    import common
    from diff_gaussian_rasterization import _C
    assert not _C.depth_wide()
    case, o = _wide_case()
    narrow = common.make_case()
    on, _ = common.run_oracle(narrow, nthreads=8, backward=False)
    assert _forward_bit_exact(case, o, "wide depth range") == 4
    assert not _C.depth_wide(), "the four-pass mode must not stick"
    assert _forward_bit_exact(narrow, on, "narrow after wide") == 3
    assert _forward_bit_exact(case, o, "wide again") == 4
    assert _forward_bit_exact(narrow, on, "narrow again") == 3


@pytest.mark.gpu
def test_views_batch_reruns_only_the_wide_view():
    """gsr_forward_views over [the wide scene's view 0, a ring view that sees it narrower]: each view's
    keys, values, ranges, radii and image equal its single-view forward bit for bit, the view flagged
    wide re-ran its depth sort in four passes, and a following batch runs three passes."""
    import synthetic
    from diff_gaussian_rasterization import _C
    case, o = _wide_case()
    dev = torch.device("cuda:0")
    sc = {k: v.to(dev) for k, v in case["scene"].items()}
    P, H, W = sc["means3D"].shape[0], 256, 256
    cams = [case["cam"], synthetic.Camera(W, H, view=4)]
    e = torch.Tensor([])
    bg = case["bg"].to(dev)

    def single(c):
        out = _C.rasterize_gaussians(bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e,
                                     c.world_view_transform.to(dev), c.full_proj_transform.to(dev), c.tanfovx,
                                     c.tanfovy, H, W, sc["shs"], 3, c.camera_center.to(dev), False, False, False)
        torch.cuda.synchronize()
        return out, _C.last_depth_passes()

    ref = [single(c) for c in cams]
    assert ref[0][1] == 4
    V = len(cams)
    out = (torch.empty((V, 3, H, W), device=dev), torch.empty((V, P), dtype=torch.int32, device=dev),
           torch.empty((V, 1, H, W), device=dev))
    for rep in range(2):  # (the second batch: binning buffers pre-sized from the first)
        Ls, geoms, bins, imgs = _C.rasterize_gaussians_views(
            bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e,
            [c.world_view_transform.to(dev) for c in cams], [c.full_proj_transform.to(dev) for c in cams],
            [c.tanfovx for c in cams], [c.tanfovy for c in cams], H, W, sc["shs"], 3,
            [c.camera_center.to(dev) for c in cams], False, False, False, out=out)
        torch.cuda.synchronize()
        passes = [_C.last_depth_passes(v) for v in range(V)]
        assert passes == [r[1] for r in ref], (rep, passes, [r[1] for r in ref])
        for v in range(V):
            (L, color, radii, geom, binning, img, inv), _ = ref[v]
            assert Ls[v] == L
            assert torch.equal(out[0][v], color) and torch.equal(out[1][v], radii) and torch.equal(out[2][v], inv)
            k1, v1, r1 = _C.sorted_keys(geom, binning, img, P, L, W, H)
            k2, v2, r2 = _C.sorted_keys(geoms[v], bins[v], imgs[v], P, L, W, H)
            assert torch.equal(k1, k2) and torch.equal(v1, v2) and torch.equal(r1, r2), v
    # a batch of narrow views afterwards: three passes each
    narrow = [synthetic.Camera(W, H, view=v) for v in (0, 1)]
    nsc = {k: v.to(dev) for k, v in __import__("common").make_case()["scene"].items()}
    out2 = (torch.empty((2, 3, H, W), device=dev), torch.empty((2, 1000), dtype=torch.int32, device=dev),
            torch.empty((2, 1, H, W), device=dev))
    _C.rasterize_gaussians_views(
        bg, nsc["means3D"], e, nsc["opacities"], nsc["scales"], nsc["rotations"], 1.0, e,
        [c.world_view_transform.to(dev) for c in narrow], [c.full_proj_transform.to(dev) for c in narrow],
        [c.tanfovx for c in narrow], [c.tanfovy for c in narrow], H, W, nsc["shs"], 3,
        [c.camera_center.to(dev) for c in narrow], False, False, False, out=out2)
    torch.cuda.synchronize()
    assert [_C.last_depth_passes(v) for v in range(2)] == [3, 3]
