"""CPU tests of the oracle (no GPU): analytic backward vs torch.autograd of a dense restatement,
internal invariants of the binning, and agreement with the committed golden fixtures."""
import os

import numpy as np
import pytest
import torch

import common
import dense_ref
import oracle
import synthetic

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _small_case(P=300, H=64, W=96, seed=3):
    case = common.make_case(P=P, H=H, W=W, seed=seed)
    sc = case["scene"]
    sc["means3D"] = sc["means3D"] * 0.45
    sc["scales"] = sc["scales"] * 4.0
    # keep o*G < 0.99 so the reference's unclamped alpha gradient (backward.cu:619) is the true one
    sc["opacities"] = sc["opacities"].clamp(max=0.95)
    g = torch.Generator().manual_seed(11)
    case["colors_precomp"] = torch.rand(P, 3, generator=g)
    o, _ = common.run_oracle(case, backward=False)
    case["cov3D_precomp"] = torch.from_numpy(o.get("cov3D").copy())
    return case


def _dense_inputs(case, mode, dtype=torch.float64):
    sc = case["scene"]
    inp = {"means3D": sc["means3D"].to(dtype).requires_grad_(True),
           "opacities": sc["opacities"].to(dtype).requires_grad_(True)}
    if mode.startswith("sh"):
        inp["shs"] = sc["shs"].to(dtype).requires_grad_(True)
    else:
        inp["colors_precomp"] = case["colors_precomp"].to(dtype).requires_grad_(True)
    if mode.endswith("scales"):
        inp["scales"] = sc["scales"].to(dtype).requires_grad_(True)
        inp["rotations"] = sc["rotations"].to(dtype).requires_grad_(True)
    else:
        inp["cov3D_precomp"] = case["cov3D_precomp"].to(dtype).requires_grad_(True)
    return inp


PAIRS = {"means3D": "dL_dmeans3D", "opacities": "dL_dopacity", "shs": "dL_dsh", "colors_precomp": "dL_dcolors",
         "scales": "dL_dscales", "rotations": "dL_drotations", "cov3D_precomp": "dL_dcov3D"}


def _decisions_agree(o, out):
    """The dense restatement's own float64 decisions against the oracle's float32 ones: radii
    equal, n_contrib equal on every pixel whose decisions are not within float32 reach of a
    threshold (forward.cu:356-370)."""
    np.testing.assert_array_equal(out["radii"].numpy(), o.radii)
    nc = out["n_contrib"].numpy()
    diff = nc != o.get("n_contrib")
    tie = out["tie"].numpy()
    assert not np.any(diff & ~tie), f"n_contrib differs on {int((diff & ~tie).sum())} non-tie pixels"
    assert tie.mean() < 1e-2
    return int(diff.sum())


@pytest.mark.parametrize("mode", ["sh_scales", "colors_cov"])
@pytest.mark.parametrize("antialiasing", [False, True])
def test_oracle_backward_matches_autograd(mode, antialiasing):
    """Oracle backward vs torch.autograd of the dense float64 restatement, whose blend decisions
    (tile rects, power > 0, alpha < 1/255, the stop rule excluding the stopping Gaussian) are its
    own -- not the oracle's."""
    case = _small_case()
    o, og = common.run_oracle(case, mode, antialiasing=antialiasing)
    assert o.num_rendered > 100
    inp = _dense_inputs(case, mode)
    out = dense_ref.dense_render(inp, dense_ref.ring_cam(case["cam"]), case["H"], case["W"], 3,
                                 case["bg"].to(torch.float64), antialiasing=antialiasing)
    _decisions_agree(o, out)
    assert int((out["n_contrib"] > 0).sum()) > 500
    assert float(out["alpha_max"]) < 0.99
    # forward agreement (fp32 oracle vs fp64 dense)
    assert np.abs(out["color"].detach().numpy() - o.color).max() < 1e-4
    assert np.abs(out["invdepth"].detach().numpy() - o.invdepth).max() < 1e-4
    assert np.abs(out["final_T"].numpy() - o.get("final_T").reshape(-1)).max() < 1e-4
    dense_ref.loss_of(out, case["grad_color"].to(torch.float64), case["grad_invdepth"].to(torch.float64)).backward()
    for k, t in inp.items():
        ok, rel = common.allclose_rel(og[PAIRS[k]].reshape(t.shape), t.grad.numpy(), rtol=2e-4, atol=1e-7)
        assert ok, f"{mode} aa={antialiasing}: oracle d{k} vs autograd rel err {rel:.3e}"


@pytest.mark.parametrize("antialiasing", [False, True])
def test_oracle_f64_backward_is_the_float64_gradient(antialiasing):
    """The oracle's float64 render-backward mode (the yardstick of common.check_rel_truth) against
    torch.autograd of the dense float64 restatement: an order of magnitude closer than the float32
    reference order is (only the float32 preprocess backward and the float32 inputs remain)."""
    case = _small_case()
    o, og = common.run_oracle(case, "sh_scales", antialiasing=antialiasing)
    g64 = o.backward(case["grad_color"], case["grad_invdepth"], f64=True)
    inp = _dense_inputs(case, "sh_scales")
    out = dense_ref.dense_render(inp, dense_ref.ring_cam(case["cam"]), case["H"], case["W"], 3,
                                 case["bg"].to(torch.float64), antialiasing=antialiasing)
    _decisions_agree(o, out)
    dense_ref.loss_of(out, case["grad_color"].to(torch.float64), case["grad_invdepth"].to(torch.float64)).backward()
    for k, t in inp.items():
        ref = t.grad.numpy()
        _, rel32 = common.allclose_rel(og[PAIRS[k]].reshape(t.shape), ref)
        ok, rel64 = common.allclose_rel(g64[PAIRS[k]].reshape(t.shape), ref, rtol=2e-5, atol=1e-9)
        assert ok, f"f64 d{k} vs autograd rel err {rel64:.3e} (float32 order: {rel32:.3e})"
    # the flag is reset: a following backward is the float32 one again
    again = o.backward(case["grad_color"], case["grad_invdepth"])
    np.testing.assert_array_equal(again["dL_dmean2D"], og["dL_dmean2D"])


def test_oracle_near_threshold_flags():
    """gsr_oracle_near_threshold (test infrastructure for the float64 accuracy check): a (H, W)
    mask, monotone in the margin, empty at margin 0 on a case without exact ties, and every
    flagged pixel's walk really holds an alpha within the margin of 1/255 (or a power / test_T
    near its threshold) -- re-derived here in numpy for the alpha criterion."""
    case = _small_case()
    o, _ = common.run_oracle(case, backward=False)
    H, W = case["H"], case["W"]
    m0, m1, m2 = (o.near_threshold(r) for r in (0.0, 1e-4, 1e-2))
    assert m1.shape == (H, W) and not m0.any()
    assert (m1 <= m2).all() and m2.sum() > m1.sum()
    vals, ranges, m2d, co = o.get("vals"), o.get("ranges"), o.get("means2D"), o.get("conic_opacity")
    gx = (W + 15) // 16
    ys, xs = np.nonzero(m2)
    hits = 0
    for y, x in zip(ys[:200], xs[:200]):
        t = (y // 16) * gx + (x // 16)
        ids = vals[ranges[t, 0]:ranges[t, 1]]
        dx = m2d[ids, 0] - np.float32(x)
        dy = m2d[ids, 1] - np.float32(y)
        pw = np.float32(-0.5) * (co[ids, 0] * dx * dx + co[ids, 2] * dy * dy) - co[ids, 1] * dx * dy
        al = np.minimum(np.float32(0.99), co[ids, 3] * np.exp(pw))
        hits += bool((np.abs(al - 1 / 255) <= 1e-2 / 255 * 1.001).any())
    assert hits >= 0.5 * min(200, len(ys))  # the rest: power or test_T criteria


def _fd_case(seed=5):
    """<= 16 Gaussians in front of view 0 of the ring, overlapping on a 48x40 image: every one
    visible, alpha < 0.99 everywhere (no clamp kink), SH colours > 0 (no clamp kink)."""
    P, H, W = 14, 40, 48
    case = common.make_case(P=P, H=H, W=W, seed=seed)
    g = torch.Generator().manual_seed(seed)
    sc = case["scene"]
    sc["means3D"] = (torch.rand(P, 3, generator=g) - 0.5) * torch.tensor([1.4, 1.12, 1.4])
    sc["scales"] = 0.25 + 0.25 * torch.rand(P, 3, generator=g)
    sc["opacities"] = 0.3 + 0.5 * torch.rand(P, 1, generator=g)
    sc["shs"][:, 0] = 1.0 + torch.rand(P, 3, generator=g)
    case["colors_precomp"] = 0.2 + torch.rand(P, 3, generator=g)
    case["bg"] = torch.tensor([0.1, 0.4, 0.7])
    o, _ = common.run_oracle(case, backward=False)
    case["cov3D_precomp"] = torch.from_numpy(o.get("cov3D").copy())
    return case


@pytest.mark.parametrize("mode", ["sh_scales", "colors_cov"])
@pytest.mark.parametrize("antialiasing", [False, True])
def test_finite_differences(mode, antialiasing):
    """central finite differences of the dense float64 forward (its own decisions
    re-made at every evaluation) on 14 Gaussians, against the oracle's analytic backward.
    With antialiasing the reference's AA-scale derivative is evaluated at the dilated covariance
    (backward.cu:213-246, RefAAScale): the finite differences then pin the exact derivative
    (autograd with aa_quirk=False) and the oracle's opacity / colour / SH gradients, which the
    quirk does not touch; the oracle's geometry gradients are pinned to the quirk through
    test_oracle_backward_matches_autograd."""
    case = _fd_case()
    o, og = common.run_oracle(case, mode, antialiasing=antialiasing)
    H, W = case["H"], case["W"]
    cam = dense_ref.ring_cam(case["cam"])
    bg = case["bg"].to(torch.float64)
    gc, gi = case["grad_color"].to(torch.float64), case["grad_invdepth"].to(torch.float64)
    inp = _dense_inputs(case, mode)
    out = dense_ref.dense_render(inp, cam, H, W, 3, bg, antialiasing=antialiasing)
    assert int(out["radii"].gt(0).sum()) == case["scene"]["means3D"].shape[0]
    _decisions_agree(o, out)
    assert not bool(out["tie"].any())
    assert float(out["alpha_max"]) < 0.99 and int((out["n_contrib"] > 0).sum()) > 0.5 * H * W
    assert np.abs(out["color"].detach().numpy() - o.color).max() < 1e-5
    assert np.abs(out["invdepth"].detach().numpy() - o.invdepth).max() < 1e-5
    assert np.abs(out["final_T"].numpy() - o.get("final_T").reshape(-1)).max() < 1e-5

    def loss():
        return dense_ref.loss_of(dense_ref.dense_render(inp, cam, H, W, 3, bg, antialiasing=antialiasing), gc, gi)

    exact = {}
    if antialiasing:
        dense_ref.loss_of(dense_ref.dense_render(inp, cam, H, W, 3, bg, antialiasing=True, aa_quirk=False),
                          gc, gi).backward()
        exact = {k: t.grad.clone() for k, t in inp.items()}
    for k, t in inp.items():
        fd = dense_ref.finite_difference(loss, t.data)
        scale = float(fd.abs().max())
        assert scale > 0
        if antialiasing:  # finite differences == exact autograd of the dense forward
            ok, rel = common.allclose_rel(exact[k].numpy(), fd.numpy(), rtol=1e-5, atol=1e-9)
            assert ok, f"{mode} aa: autograd(exact) d{k} vs finite differences rel err {rel:.3e}"
            if k not in ("opacities", "shs", "colors_precomp"):
                continue
        ok, rel = common.allclose_rel(og[PAIRS[k]].reshape(t.shape), fd.numpy(), rtol=1e-4, atol=1e-8)
        assert ok, f"{mode} aa={antialiasing}: oracle d{k} vs finite differences rel err {rel:.3e}"


def test_binning_invariants():
    case = common.make_case(P=2000, H=200, W=328)
    o, _ = common.run_oracle(case, backward=False)
    keys, vals, ranges = o.get("keys"), o.get("vals"), o.get("ranges")
    L = o.num_rendered
    assert L == int(o.get("tiles_touched").sum())
    assert np.all(np.diff(keys.astype(np.uint64)) >= 0) or np.all(keys[1:] >= keys[:-1])
    # stability: equal keys keep emission (= Gaussian index) order
    same = keys[1:] == keys[:-1]
    assert np.all(vals[1:][same] > vals[:-1][same])
    # ranges partition [0, L) by tile id
    tiles = (keys >> np.uint64(32)).astype(np.int64)
    for t in np.unique(tiles):
        a, b = ranges[t]
        assert np.all(tiles[a:b] == t) and (a == 0 or tiles[a - 1] != t) and (b == L or tiles[b] != t)
    # getHigherMsb (rasterizer_impl.cu:35-50): smallest b with (n >> b) == 0
    for n in [1, 2, 255, 256, 257, 8160, 1 << 20]:
        b = oracle.higher_msb(n)
        assert (n >> b) == 0 and (b == 0 or (n >> (b - 1)) != 0)


def test_mark_visible_matches_depth():
    case = common.make_case(P=500)
    cam = case["cam"]
    vis = oracle.mark_visible(case["scene"]["means3D"], cam.world_view_transform, cam.full_proj_transform)
    pv = torch.cat([case["scene"]["means3D"], torch.ones(500, 1)], 1) @ cam.world_view_transform
    assert np.array_equal(vis, (pv[:, 2] > 0.2).numpy())


def test_prefiltered_violation_raises():
    case = common.make_case(P=20)
    sc = case["scene"]
    sc["means3D"][0] = case["cam"].camera_center * 1.5
    with pytest.raises(RuntimeError, match="prefiltered"):
        oracle.OracleRaster(sc["means3D"], sc["opacities"], case["bg"], case["cam"].world_view_transform,
                            case["cam"].full_proj_transform, case["cam"].camera_center, case["cam"].tanfovx,
                            case["cam"].tanfovy, case["H"], case["W"], shs=sc["shs"], sh_degree=3,
                            scales=sc["scales"], rotations=sc["rotations"], prefiltered=True)


def _golden_files():
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz")) if os.path.isdir(GOLDEN) else []


@pytest.mark.parametrize("fname", _golden_files())
def test_oracle_reproduces_golden(fname):
    """The oracle is deterministic (1 thread): it must reproduce the committed fixtures bit-exactly,
    and its SH colours / covariances must agree with the reference's own Python
    (utils/sh_utils.py eval_sh, utils/general_utils.py build_scaling_rotation) stored in them."""
    z = np.load(os.path.join(GOLDEN, fname), allow_pickle=False)
    o = oracle.OracleRaster(
        z["means3D"], z["opacities"], z["bg"], z["viewmatrix"], z["projmatrix"], z["campos"], float(z["tanfovx"]),
        float(z["tanfovy"]), int(z["H"]), int(z["W"]),
        shs=z["shs"] if z["shs"].size else None, sh_degree=int(z["sh_degree"]),
        colors_precomp=z["colors_precomp"] if z["colors_precomp"].size else None,
        scales=z["scales"] if z["scales"].size else None, rotations=z["rotations"] if z["rotations"].size else None,
        cov3D_precomp=z["cov3D_precomp"] if z["cov3D_precomp"].size else None, antialiasing=bool(z["antialiasing"]),
        scale_modifier=float(z["scale_modifier"]))
    g = o.backward(z["grad_color"].astype(np.float32), z["grad_invdepth"].astype(np.float32))
    assert o.num_rendered == int(z["num_rendered"])
    np.testing.assert_array_equal(o.radii, z["radii"])
    np.testing.assert_array_equal(o.get("keys"), z["keys"])
    np.testing.assert_array_equal(o.get("vals"), z["vals"])
    np.testing.assert_array_equal(o.get("ranges"), z["ranges"])
    np.testing.assert_array_equal(o.color, z["color"])
    np.testing.assert_array_equal(o.invdepth, z["invdepth"])
    np.testing.assert_array_equal(o.get("n_contrib"), z["n_contrib"])
    np.testing.assert_array_equal(o.get("final_T"), z["final_T"])
    np.testing.assert_array_equal(o.get("means2D"), z["means2D"])
    np.testing.assert_array_equal(o.get("conic_opacity"), z["conic_opacity"])
    for k in ["dL_dmeans3D", "dL_dopacity", "dL_dsh", "dL_dcolors", "dL_dscales", "dL_drotations", "dL_dcov3D",
              "dL_dmean2D"]:
        np.testing.assert_array_equal(g[k], z[k], err_msg=k)
    if z["ref_rgb"].size:  # reference eval_sh path (gaussian_renderer/__init__.py:76-80)
        vis = o.radii > 0
        np.testing.assert_allclose(o.get("rgb")[vis], z["ref_rgb"][vis], rtol=0, atol=2e-6)
    if z["ref_cov3D"].size:  # reference build_scaling_rotation path (scene/gaussian_model.py:33-37)
        # fp32, different op order: relative to the largest covariance entry (off-diagonals cancel)
        np.testing.assert_allclose(o.get("cov3D"), z["ref_cov3D"], rtol=1e-5,
                                   atol=1e-6 * float(np.abs(z["ref_cov3D"]).max()))


def test_cpu_abi_matches_oracle():
    """oracle/libgsr_cpu.so -- the C oracle behind include/gsr.h's gsr_forward / gsr_backward
    (resize callbacks, state in the caller's buffers; bench.py's CPU baseline) -- equals the
    oracle's own API bit for bit on config 1 (one thread each: the OpenMP backward's per-Gaussian
    sums follow the thread schedule)."""
    import cpu_abi
    case = common.make_case(P=1000, H=256, W=256)
    o, og = common.run_oracle(case, antialiasing=True)
    sc, cam = case["scene"], case["cam"]
    L, color, inv, radii, g = cpu_abi.CpuRasterizer(nthreads=1).forward_backward(
        sc["means3D"], sc["opacities"], case["bg"], cam.world_view_transform, cam.full_proj_transform,
        cam.camera_center, cam.tanfovx, cam.tanfovy, 256, 256, case["grad_color"], case["grad_invdepth"],
        shs=sc["shs"], sh_degree=3, scales=sc["scales"], rotations=sc["rotations"], antialiasing=True)
    assert L == o.num_rendered
    np.testing.assert_array_equal(radii, o.radii)
    np.testing.assert_array_equal(color, o.color)
    np.testing.assert_array_equal(inv, o.invdepth)
    for k in ("dL_dmean2D", "dL_dopacity", "dL_dcolors", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"):
        np.testing.assert_array_equal(g[k], og[k].reshape(g[k].shape), err_msg=k)


def test_shared_exp_accuracy():
    """gsr_ref_expf (gaussian-splatting-npu_amd/csrc/gsr_ref_exp.h, the exp() the GSR_REF_ALPHA test
    build of the render kernels and the oracle's shared_exp mode both evaluate) is within 1.5 ulp of
    exp over the range the blend uses, 0 below it."""
    import ctypes
    lib = oracle.lib()
    f = lib.gsr_oracle_ref_expf
    f.restype, f.argtypes = ctypes.c_float, [ctypes.c_float]
    xs = np.concatenate([np.linspace(-103, 88, 20001, dtype=np.float32),
                         -np.logspace(-8, 2, 2000).astype(np.float32), np.float32([0.0, -0.0])])
    ys = np.array([f(float(x)) for x in xs], np.float32)
    t = np.exp(xs.astype(np.float64))
    m = t > 1.2e-38
    ulp = np.abs(ys[m].astype(np.float64) - t[m]) / np.spacing(t[m].astype(np.float32)).astype(np.float64)
    assert ulp.max() <= 1.5, ulp.max()
    assert f(0.0) == 1.0 and f(-200.0) == 0.0 and f(float("nan")) == 0.0


def test_shared_exp_oracle_differs_only_at_thresholds():
    """The oracle with the shared exp (OracleRaster(shared_exp=True), the test_ref_alpha_exact
    comparison's checker) against its libm-exp self on config 1: identical binning, images within
    the tolerances of a 1-ulp exp difference."""
    case = common.make_case()
    a, ga = common.run_oracle(case)
    sc, cam = case["scene"], case["cam"]
    b = oracle.OracleRaster(sc["means3D"], sc["opacities"], case["bg"], cam.world_view_transform,
                            cam.full_proj_transform, cam.camera_center, cam.tanfovx, cam.tanfovy, case["H"],
                            case["W"], shs=sc["shs"], sh_degree=3, scales=sc["scales"], rotations=sc["rotations"],
                            shared_exp=True)
    gb = b.backward(case["grad_color"], case["grad_invdepth"])
    np.testing.assert_array_equal(a.get("keys"), b.get("keys"))
    np.testing.assert_array_equal(a.radii, b.radii)
    common.check_render("oracle shared exp vs libm", {"color": b.color, "invdepth": b.invdepth,
                                                      "final_T": b.get("final_T"), "n_contrib": b.get("n_contrib")},
                        {"color": a.color, "invdepth": a.invdepth, "final_T": a.get("final_T"),
                         "n_contrib": a.get("n_contrib")})
    assert not np.array_equal(a.color, b.color)  # the switch is live
    ok, rel = common.allclose_rel(gb["dL_dmeans3D"], ga["dL_dmeans3D"])
    assert ok, rel
