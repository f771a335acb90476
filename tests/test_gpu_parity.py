"""HIP path vs CPU oracle parity (needs an MI355X: -m gpu).

Every comparison goes through the drop-in surface (diff_gaussian_rasterization -> _C ->
libgsr_hip.so C ABI).  Preprocess outputs and the sorted tile|depth keys are compared
bit-exactly; images and gradients with the fp32 tolerances stated in tests/common.py.
"""
import numpy as np
import pytest
import torch

import common

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _dgr():
    import diff_gaussian_rasterization as dgr
    return dgr


def _settings(case, antialiasing=False, prefiltered=False, scale_modifier=1.0, debug=False):
    dgr = _dgr()
    cam = case["cam"]
    return dgr.GaussianRasterizationSettings(
        image_height=case["H"], image_width=case["W"], tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=case["bg"].to(DEV), scale_modifier=scale_modifier, viewmatrix=cam.world_view_transform.to(DEV),
        projmatrix=cam.full_proj_transform.to(DEV), sh_degree=case["sh_degree"], campos=cam.camera_center.to(DEV),
        prefiltered=prefiltered, debug=debug, antialiasing=antialiasing)


def _inputs(case, mode):
    sc = case["scene"]
    t = {k: v.to(DEV).clone().requires_grad_(True) for k, v in sc.items()}
    kw = dict(means3D=t["means3D"], opacities=t["opacities"])
    if mode in ("sh_scales", "sh_cov"):
        kw["shs"] = t["shs"]
    else:
        t["colors_precomp"] = case["colors_precomp"].to(DEV).clone().requires_grad_(True)
        kw["colors_precomp"] = t["colors_precomp"]
    if mode in ("sh_scales", "colors_scales"):
        kw["scales"], kw["rotations"] = t["scales"], t["rotations"]
    else:
        t["cov3D_precomp"] = case["cov3D_precomp"].to(DEV).clone().requires_grad_(True)
        kw["cov3D_precomp"] = t["cov3D_precomp"]
    return t, kw


def run_hip(case, mode="sh_scales", antialiasing=False):
    dgr = _dgr()
    rast = dgr.GaussianRasterizer(_settings(case, antialiasing))
    t, kw = _inputs(case, mode)
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    means2D.retain_grad()
    color, radii, invdepth = rast(means2D=means2D, **kw)
    loss = (color * case["grad_color"].to(DEV)).sum() + (invdepth * case["grad_invdepth"].to(DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    g = {k: v.grad.detach().cpu().numpy() for k, v in t.items() if v.grad is not None}
    g["means2D"] = means2D.grad.detach().cpu().numpy()
    color, invdepth = color.detach().cpu().numpy(), invdepth.detach().cpu().numpy()
    g["_render"] = _hip_render(rast.raster_settings, kw, color, invdepth)
    return color, radii.cpu().numpy(), invdepth, g


def _with_precomp(case):
    g = torch.Generator().manual_seed(7)
    P = case["scene"]["means3D"].shape[0]
    case["colors_precomp"] = torch.rand(P, 3, generator=g)
    o, _ = common.run_oracle(case, "sh_scales", backward=False)
    case["cov3D_precomp"] = torch.from_numpy(o.get("cov3D").copy())
    return case


def _img_state(img, W, H):
    """final_T and n_contrib of a forward, read from its image state buffer (IMG_FINAL_T /
    IMG_N_CONTRIB of gsr_common.h; the reference's ImageState accum_alpha / n_contrib)."""
    lay = _dgr()._C.image_layout(W, H)
    N = W * H
    fT = img[lay[1]:lay[1] + 4 * N].cpu().numpy().view(np.float32)
    nc = img[lay[2]:lay[2] + 4 * N].cpu().numpy().view(np.uint32)
    return fT, nc


def _c_forward(s, kw, dc=None):
    """_C.rasterize_gaussians on the settings and GaussianRasterizer-style inputs `kw`."""
    dgr = _dgr()
    e = torch.Tensor([])
    g = lambda k: kw[k].detach() if k in kw else e  # noqa: E731
    return dgr._C.rasterize_gaussians(
        s.bg, g("means3D"), g("colors_precomp"), g("opacities"), g("scales"), g("rotations"), s.scale_modifier,
        g("cov3D_precomp"), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
        g("shs"), s.sh_degree, s.campos, s.prefiltered, s.antialiasing, False, dc=dc)


def _hip_render(s, kw, color, inv):
    fT, nc = _img_state(_c_forward(s, kw)[5], s.image_width, s.image_height)
    return {"color": color, "invdepth": inv, "final_T": fT, "n_contrib": nc}


def _ora_render(o):
    return {"color": o.color, "invdepth": o.invdepth, "final_T": o.get("final_T"), "n_contrib": o.get("n_contrib")}


@pytest.mark.parametrize("antialiasing", [False, True])
def test_preprocess_and_keys_bit_exact(antialiasing):
    """radii, means2D, depth, conic+opacity, rgb, tile counts and the sorted tile|depth keys
    are bit-identical to the oracle (rasterizer_impl.cu:250-320)."""
    dgr = _dgr()
    case = common.make_case()
    o, _ = common.run_oracle(case, antialiasing=antialiasing, backward=False)
    s = _settings(case, antialiasing)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], torch.Tensor([]), sc["opacities"], sc["scales"], sc["rotations"], 1.0,
        torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
        sc["shs"], s.sh_degree, s.campos, False, antialiasing, False)
    torch.cuda.synchronize()
    P = sc["means3D"].shape[0]
    assert L == o.num_rendered
    r = radii.cpu().numpy()
    np.testing.assert_array_equal(r, o.radii)
    vis = r > 0
    lay = dgr._C.geometry_layout(P)
    gb = geom.cpu().numpy()

    def arr(i, dt, shape):
        n = int(np.prod(shape)) * np.dtype(dt).itemsize
        return gb[lay[i]:lay[i] + n].view(dt).reshape(shape)

    np.testing.assert_array_equal(arr(0, np.uint32, (P,))[vis], o.get("depths").view(np.uint32)[vis])
    np.testing.assert_array_equal(arr(3, np.uint32, (P, 2))[vis], o.get("means2D").view(np.uint32)[vis])
    np.testing.assert_array_equal(arr(4, np.uint32, (P, 4))[vis], o.get("conic_opacity").view(np.uint32)[vis])
    np.testing.assert_array_equal(arr(5, np.uint32, (P, 3))[vis], o.get("rgb").view(np.uint32)[vis])
    np.testing.assert_array_equal(arr(6, np.uint32, (P,)), o.get("tiles_touched"))
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, s.image_width, s.image_height)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))


@pytest.mark.parametrize("mode", ["sh_scales", "colors_scales", "sh_cov", "colors_cov"])
@pytest.mark.parametrize("antialiasing", [False, True])
def test_forward_backward_parity(mode, antialiasing):
    case = _with_precomp(common.make_case())
    o, og = common.run_oracle(case, mode, antialiasing=antialiasing)
    color, radii, inv, g = run_hip(case, mode, antialiasing)
    np.testing.assert_array_equal(radii, o.radii)
    common.check_render(f"{mode} aa={antialiasing}", g["_render"], _ora_render(o))
    checks = {"means3D": "dL_dmeans3D", "opacities": "dL_dopacity", "means2D": "dL_dmean2D"}
    if mode.startswith("sh"):
        checks["shs"] = "dL_dsh"
    else:
        checks["colors_precomp"] = "dL_dcolors"
    if mode.endswith("scales"):
        checks.update(scales="dL_dscales", rotations="dL_drotations")
    else:
        checks["cov3D_precomp"] = "dL_dcov3D"
    for hk, ok in checks.items():
        a, b = g[hk], og[ok].reshape(g[hk].shape)
        ok_, rel = common.allclose_rel(a, b)
        assert ok_, f"{mode} aa={antialiasing}: grad {hk} rel err {rel:.3e}"


def test_loss_without_invdepth_matches_zero_invdepth_gradient():
    """A loss that ignores the invdepth output (train.py without a depth prior): autograd hands the
    backward None for it (no materialised zeros), which must equal the reference's zero dL/dinvdepth."""
    case = common.make_case()
    case["grad_invdepth"] = torch.zeros_like(case["grad_invdepth"])
    o, og = common.run_oracle(case)
    dgr = _dgr()
    t, kw = _inputs(case, "sh_scales")
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    color, radii, inv = dgr.GaussianRasterizer(_settings(case))(means2D=means2D, **kw)
    (color * case["grad_color"].to(DEV)).sum().backward()
    torch.cuda.synchronize()
    for hk, ok in {"means3D": "dL_dmeans3D", "shs": "dL_dsh", "opacities": "dL_dopacity", "scales": "dL_dscales",
                   "rotations": "dL_drotations"}.items():
        ok_, rel = common.allclose_rel(t[hk].grad.cpu().numpy(), og[ok].reshape(t[hk].shape))
        assert ok_, f"grad {hk} rel err {rel:.3e}"
    ok_, rel = common.allclose_rel(means2D.grad.cpu().numpy(), og["dL_dmean2D"])
    assert ok_, f"grad means2D rel err {rel:.3e}"


def test_forward_with_and_without_preallocated_binning():
    """The forward pre-sizes its binning buffer from the previous call: a first call, a call that
    outgrows the guess (falls back to an exact allocation) and a call that fits must agree."""
    dgr = _dgr()
    small, big = common.make_case(P=300), common.make_case(P=3000)
    dgr._C._binning_hint.clear()
    outs = []
    for case in (big, small, big, big):
        t, kw = _inputs(case, "sh_scales")
        with torch.no_grad():
            color, radii, inv = dgr.GaussianRasterizer(_settings(case))(
                means2D=torch.zeros_like(t["means3D"]), **kw)
        outs.append(color.cpu().numpy())
    assert np.array_equal(outs[0], outs[2]) and np.array_equal(outs[2], outs[3])


def test_1080p_view_properties():
    """Full-size view: image/grad parity on a 50k-Gaussian 1080p frame (oracle multi-threaded)."""
    case = common.make_case(P=50000, H=1080, W=1920)
    o, og = common.run_oracle(case, nthreads=8)
    color, radii, inv, g = run_hip(case)
    np.testing.assert_array_equal(radii, o.radii)
    common.check_render("1080p 50k", g["_render"], _ora_render(o))
    for hk, ok in {"means3D": "dL_dmeans3D", "shs": "dL_dsh", "opacities": "dL_dopacity",
                   "scales": "dL_dscales", "rotations": "dL_drotations"}.items():
        ok_, rel = common.allclose_rel(g[hk], og[ok].reshape(g[hk].shape), rtol=5e-4)
        assert ok_, f"grad {hk} rel err {rel:.3e}"


def test_uhd_view_multi_pass_tile_order():
    """3840x2176 (32,640 tiles): the longest-first tile order runs in two 16K-tile passes;
    every tile must still be rendered exactly once, forward and backward."""
    case = common.make_case(P=20000, H=2176, W=3840)
    o, og = common.run_oracle(case, nthreads=8)
    color, radii, inv, g = run_hip(case)
    np.testing.assert_array_equal(radii, o.radii)
    common.check_render("uhd 20k", g["_render"], _ora_render(o))
    for hk, ok in {"means3D": "dL_dmeans3D", "opacities": "dL_dopacity", "means2D": "dL_dmean2D"}.items():
        ok_, rel = common.allclose_rel(g[hk], og[ok].reshape(g[hk].shape), rtol=5e-4)
        assert ok_, f"grad {hk} rel err {rel:.3e}"


def test_8k_view_three_pass_tile_sort():
    """7680x4320 (129,600 tiles: 17-bit tile ids): the tile sort takes three passes -- the fused
    emission pass and two plain ones; keys, Gaussian ids, tile ranges and radii bit-exact against
    the oracle, the image through check_render."""
    dgr = _dgr()
    case = common.make_case(P=3000, H=4320, W=7680)
    o, _ = common.run_oracle(case, nthreads=8, backward=False)
    s = _settings(case)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], torch.Tensor([]), sc["opacities"], sc["scales"], sc["rotations"], 1.0,
        torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
        sc["shs"], s.sh_degree, s.campos, False, False, False)
    torch.cuda.synchronize()
    P = sc["means3D"].shape[0]
    assert L == o.num_rendered and L > 0
    np.testing.assert_array_equal(radii.cpu().numpy(), o.radii)
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, s.image_width, s.image_height)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))
    kw = {"means3D": sc["means3D"], "shs": sc["shs"], "opacities": sc["opacities"], "scales": sc["scales"],
          "rotations": sc["rotations"]}
    common.check_render("8k 3k", _hip_render(s, kw, color.cpu().numpy(), inv.cpu().numpy()), _ora_render(o))


@pytest.mark.parametrize("H,W,P", [(256, 4080, 3000), (256, 4096, 3000), (4080, 256, 3000), (4096, 256, 3000),
                                   (256, 4080, 3001), (256, 4096, 3003), (256, 256, 1001), (256, 256, 3)])
def test_packed_rect_boundary_keys_bit_exact(H, W, P):
    """The 255 / 256-tile boundary: up to 255 x 255 tiles the depth sort carries the tile rect packed
    into one word (a byte per bound) and the tile ranges come from the rects' 2-D difference array
    (tile_hist + the tile-order prefix sums; the tile sort writes no tile ids); above it the depth
    sort gathers the u16x4 rect by id and the ranges come from tile_ranges over the sorted tile ids.
    255 and 256 tiles along either axis give keys, ids and ranges bit-identical to the oracle, and
    every gradient matches it on both sides.  The record slots switch there too: up to 255 tiles the
    tile sort carries no slot and render_bwd derives each instance's slot from the packed rect in the
    render record (emit_start + its index in the rect); above, the tile sort writes the index in the
    rect per instance (BIN_SLOT) and render_bwd reads it.  P not a multiple of 4 (3001, 3003, 1001,
    3) covers tile_hist's tail, the last P mod 4 rects it adds outside its 16-B loads."""
    dgr = _dgr()
    case = common.make_case(P=P, H=H, W=W)
    o, og = common.run_oracle(case, nthreads=8, backward=True)
    s = _settings(case)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], torch.Tensor([]), sc["opacities"], sc["scales"], sc["rotations"], 1.0,
        torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
        sc["shs"], s.sh_degree, s.campos, False, False, False)
    torch.cuda.synchronize()
    P = sc["means3D"].shape[0]
    assert L == o.num_rendered and L > 0
    np.testing.assert_array_equal(radii.cpu().numpy(), o.radii)
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, s.image_width, s.image_height)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))
    del keys, vals, ranges
    fT, nc = _img_state(img, W, H)
    flips = []
    common.check_render(f"rect boundary {W}x{H}", {"color": color.cpu().numpy(), "invdepth": inv.cpu().numpy(),
                                                  "final_T": fT, "n_contrib": nc}, _ora_render(o), flips=flips)
    affected = common.flip_gaussians(flips[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
    gc, gi = case["grad_color"].to(DEV), case["grad_invdepth"].to(DEV)
    out = dgr._C.rasterize_gaussians_backward(
        s.bg, sc["means3D"], radii, torch.Tensor([]), sc["opacities"], sc["scales"], sc["rotations"], 1.0,
        torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, gc, gi, sc["shs"], s.sh_degree, s.campos,
        geom, L, binning, img, False, False)
    torch.cuda.synchronize()
    names = ["dL_dmean2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    for n, t in zip(names, out):
        # 3,000 Gaussians spread over up to 4096 x 256 pixels cover few pixels each: one flipped
        # pixel's term is a larger share of a gradient (measured 2.005e-3 of max, round 5)
        common.check_grad_attributed(f"rect boundary {W}x{H} {n}", t.cpu().numpy(), og[n].reshape(t.shape), affected,
                                     rtol_attr=common.GRAD_RTOL_ATTRIBUTED_SMALL_FOOTPRINT)


def test_mark_visible():
    import oracle
    dgr = _dgr()
    case = common.make_case()
    rast = dgr.GaussianRasterizer(_settings(case))
    vis = rast.markVisible(case["scene"]["means3D"].to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(vis, oracle.mark_visible(case["scene"]["means3D"], case["cam"].world_view_transform,
                                                           case["cam"].full_proj_transform))


def test_empty_and_all_culled():
    dgr = _dgr()
    case = common.make_case(P=10)
    s = _settings(case)
    rast = dgr.GaussianRasterizer(s)
    z = torch.zeros((0, 3), device=DEV)
    color, radii, inv = rast(means3D=z, means2D=z, opacities=torch.zeros((0, 1), device=DEV),
                             shs=torch.zeros((0, 16, 3), device=DEV), scales=z, rotations=torch.zeros((0, 4), device=DEV))
    assert color.shape == (3, case["H"], case["W"]) and float(color.abs().sum()) == 0.0 and radii.numel() == 0
    # every point behind the camera: nothing rendered, image = background
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    cam_c = case["cam"].camera_center.to(DEV)
    behind = cam_c + (cam_c - 0.0) * 0.5 + 0.0 * sc["means3D"]
    color, radii, inv = rast(means3D=behind, means2D=torch.zeros_like(behind), opacities=sc["opacities"],
                             shs=sc["shs"], scales=sc["scales"], rotations=sc["rotations"])
    assert int(radii.abs().sum()) == 0
    assert torch.allclose(color, s.bg.view(3, 1, 1).expand_as(color))


def test_prefiltered_violation_raises():
    dgr = _dgr()
    case = common.make_case(P=10)
    s = _settings(case, prefiltered=True)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    cam_c = case["cam"].camera_center.to(DEV)
    pts = sc["means3D"].clone()
    pts[0] = cam_c * 1.5  # behind the camera -> near-culled although prefiltered
    with pytest.raises(RuntimeError, match="prefiltered"):
        dgr.GaussianRasterizer(s)(means3D=pts, means2D=torch.zeros_like(pts), opacities=sc["opacities"],
                                  shs=sc["shs"], scales=sc["scales"], rotations=sc["rotations"])


def test_argument_errors_match_reference():
    dgr = _dgr()
    case = common.make_case(P=10)
    rast = dgr.GaussianRasterizer(_settings(case))
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    with pytest.raises(Exception, match="excatly one of either SHs"):
        rast(means3D=sc["means3D"], means2D=sc["means3D"], opacities=sc["opacities"], scales=sc["scales"],
             rotations=sc["rotations"])
    with pytest.raises(Exception, match="scale/rotation pair"):
        rast(means3D=sc["means3D"], means2D=sc["means3D"], opacities=sc["opacities"], shs=sc["shs"])
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        dgr._C.rasterize_gaussians(sc["means3D"].new_zeros(4), sc["means3D"].new_zeros(4), torch.Tensor([]),
                                   sc["opacities"], sc["scales"], sc["rotations"], 1.0, torch.Tensor([]),
                                   sc["means3D"], sc["means3D"], 1.0, 1.0, 8, 8, sc["shs"], 3, sc["means3D"][0],
                                   False, False, False)


def _golden_files():
    import os
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".npz")) if os.path.isdir(d) else []


@pytest.mark.parametrize("path", _golden_files(), ids=lambda p: p.rsplit("/", 1)[-1])
def test_hip_matches_golden_fixture(path):
    """The HIP path through GaussianRasterizer on a committed fixture's inputs (reference-built
    matrices, the reference's PLY hand cases, every input mode): keys / values / ranges / radii
    bit-exact, images and gradients within the tests/common.py tolerances of the stored arrays."""
    dgr = _dgr()
    z = np.load(path, allow_pickle=False)
    H, W = int(z["H"]), int(z["W"])
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k], dtype=np.float32)).to(DEV)  # noqa: E731
    s = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(z["tanfovx"]), tanfovy=float(z["tanfovy"]), bg=t("bg"),
        scale_modifier=float(z["scale_modifier"]), viewmatrix=t("viewmatrix"), projmatrix=t("projmatrix"),
        sh_degree=int(z["sh_degree"]), campos=t("campos"), prefiltered=False, debug=False,
        antialiasing=bool(z["antialiasing"]))
    params = {k: t(k).requires_grad_(True) for k in ["means3D", "opacities", "shs", "colors_precomp", "scales",
                                                       "rotations", "cov3D_precomp"] if z[k].size}
    means2D = torch.zeros_like(params["means3D"], requires_grad=True)
    color, radii, inv = dgr.GaussianRasterizer(s)(means2D=means2D, **params)
    torch.autograd.backward([color, inv], [t("grad_color"), t("grad_invdepth")])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(radii.cpu().numpy(), z["radii"])
    # binning of the same inputs through the _C level
    P = params["means3D"].shape[0]
    e = torch.Tensor([])
    L, _, _, geom, binning, img, _ = dgr._C.rasterize_gaussians(
        s.bg, params["means3D"].detach(), params["colors_precomp"].detach() if "colors_precomp" in params else e,
        params["opacities"].detach(), params["scales"].detach() if "scales" in params else e,
        params["rotations"].detach() if "rotations" in params else e, s.scale_modifier,
        params["cov3D_precomp"].detach() if "cov3D_precomp" in params else e, s.viewmatrix, s.projmatrix,
        s.tanfovx, s.tanfovy, H, W, params["shs"].detach() if "shs" in params else e, s.sh_degree, s.campos,
        False, s.antialiasing, False)
    assert L == int(z["num_rendered"])
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, W, H)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), z["keys"])
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), z["vals"])
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), z["ranges"])
    fT, nc = _img_state(img, W, H)
    common.check_render(path.rsplit("/", 1)[-1], {"color": color.detach().cpu().numpy(),
                                                  "invdepth": inv.detach().cpu().numpy(), "final_T": fT,
                                                  "n_contrib": nc},
                        {"color": z["color"], "invdepth": z["invdepth"], "final_T": z["final_T"],
                         "n_contrib": z["n_contrib"]})
    checks = {"means3D": "dL_dmeans3D", "opacities": "dL_dopacity", "shs": "dL_dsh", "colors_precomp": "dL_dcolors",
              "scales": "dL_dscales", "rotations": "dL_drotations", "cov3D_precomp": "dL_dcov3D"}
    for k, gk in checks.items():
        if k in params:
            a = params[k].grad.detach().cpu().numpy()
            ok_, rel = common.allclose_rel(a, z[gk].reshape(a.shape))
            assert ok_, f"{path}: grad {k} rel err {rel:.3e}"
    ok_, rel = common.allclose_rel(means2D.grad.detach().cpu().numpy(), z["dL_dmean2D"])
    assert ok_, f"{path}: grad means2D rel err {rel:.3e}"


def test_callback_forward_matches_split_forward():
    """gsr_forward (the Rasterizer::forward form with resize callbacks, rasterizer.h:31-55 and
    rasterize_points.cu:27-33; the binding INTEGRATION.md shows) gives the same image, radii and
    L as the two-phase entry points the Python package uses."""
    import ctypes
    dgr = _dgr()
    lib = dgr._C.lib
    case = common.make_case()
    s = _settings(case)
    sc = {k: v.to(DEV).contiguous() for k, v in case["scene"].items()}
    P, H, W = sc["means3D"].shape[0], case["H"], case["W"]
    RESIZE = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
    V, I, F, B = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_bool
    lib.gsr_forward.argtypes = [RESIZE, V, RESIZE, V, RESIZE, V, I, I, I, V, I, I, V, V, V, V, V, F, V, V, V, V, V,
                                F, F, B, V, V, B, V, B, V, ctypes.POINTER(I)]
    bufs = [torch.empty(0, dtype=torch.uint8, device=DEV) for _ in range(3)]

    def resizer(k):
        def f(_ctx, n):
            bufs[k].resize_(n)
            return bufs[k].data_ptr()
        return RESIZE(f)

    rg, rb, ri = resizer(0), resizer(1), resizer(2)
    view, proj = s.viewmatrix.contiguous(), s.projmatrix.contiguous()  # the settings hold transposed views
    color = torch.zeros((3, H, W), device=DEV)
    inv = torch.zeros((1, H, W), device=DEV)
    radii = torch.zeros((P,), dtype=torch.int32, device=DEV)
    L = ctypes.c_int(0)
    rc = lib.gsr_forward(rg, None, rb, None, ri, None, P, 3, 16, s.bg.data_ptr(), W, H, sc["means3D"].data_ptr(),
                         sc["shs"].data_ptr(), None, sc["opacities"].data_ptr(), sc["scales"].data_ptr(), 1.0,
                         sc["rotations"].data_ptr(), None, view.data_ptr(), proj.data_ptr(),
                         s.campos.data_ptr(), s.tanfovx, s.tanfovy, False, color.data_ptr(), inv.data_ptr(), False,
                         radii.data_ptr(), False, torch.cuda.current_stream(DEV).cuda_stream, ctypes.byref(L))
    assert rc == 0, lib.gsr_last_error()
    L2, color2, radii2, _, _, _, inv2 = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], torch.Tensor([]), sc["opacities"], sc["scales"], sc["rotations"], 1.0,
        torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, sc["shs"], 3, s.campos, False,
        False, False)
    torch.cuda.synchronize()
    assert L.value == L2 > 0
    assert bufs[1].numel() >= lib.gsr_binning_buffer_size(L2)
    assert torch.equal(radii, radii2)
    assert torch.equal(color, color2) and torch.equal(inv, inv2)


def test_parameter_gradients_share_one_buffer():
    """The backward's parameter gradients arrive as consecutive views of one buffer (multiview
    PARAM_ORDER), so the multi-GPU step can all-reduce them in place (multiview.flat_grad_view)."""
    from diff_gaussian_rasterization import multiview
    case = common.make_case()
    t, kw = _inputs(case, "sh_scales")
    color, radii, inv = _dgr().GaussianRasterizer(_settings(case))(
        means2D=torch.zeros_like(t["means3D"], requires_grad=True), **kw)
    torch.autograd.backward([color, inv], [case["grad_color"].to(DEV), case["grad_invdepth"].to(DEV)])
    params = {"means3D": t["means3D"], "shs": t["shs"], "opacities": t["opacities"], "scales": t["scales"],
              "rotations": t["rotations"]}
    flat = multiview.flat_grad_view(params)
    assert flat is not None
    assert flat.numel() == sum(p.numel() for p in params.values())
    torch.testing.assert_close(flat, multiview.grad_bucket(params), rtol=0, atol=0)

