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


@pytest.mark.parametrize("mode", ["sh_scales", "colors_cov"])
@pytest.mark.parametrize("antialiasing", [False, True])
def test_oracle_backward_matches_autograd(mode, antialiasing):
    case = _small_case()
    o, og = common.run_oracle(case, mode, antialiasing=antialiasing)
    assert o.num_rendered > 100
    contrib = dense_ref.frozen_contributors(o)
    assert sum(len(r) for r in contrib) > 1000
    cam = case["cam"]
    sc = case["scene"]
    d = torch.float64
    inp = {"means3D": sc["means3D"].to(d).requires_grad_(True), "opacities": sc["opacities"].to(d).requires_grad_(True)}
    if mode.startswith("sh"):
        inp["shs"] = sc["shs"].to(d).requires_grad_(True)
    else:
        inp["colors_precomp"] = case["colors_precomp"].to(d).requires_grad_(True)
    if mode.endswith("scales"):
        inp["scales"] = sc["scales"].to(d).requires_grad_(True)
        inp["rotations"] = sc["rotations"].to(d).requires_grad_(True)
    else:
        inp["cov3D_precomp"] = case["cov3D_precomp"].to(d).requires_grad_(True)
    camd = {"view": cam.world_view_transform.to(d), "proj": cam.full_proj_transform.to(d),
            "campos": cam.camera_center.to(d), "tanfovx": cam.tanfovx, "tanfovy": cam.tanfovy}
    col, inv, alpha = dense_ref.dense_forward(inp, camd, case["H"], case["W"], 3, case["bg"].to(d), contrib,
                                              antialiasing=antialiasing)
    assert float(alpha.max()) < 0.99
    # forward agreement (fp32 oracle vs fp64 dense)
    assert np.abs(col.detach().numpy() - o.color).max() < 1e-4
    assert np.abs(inv.detach().numpy() - o.invdepth).max() < 1e-4
    loss = (col * case["grad_color"].to(d)).sum() + (inv * case["grad_invdepth"].to(d)).sum()
    loss.backward()
    pairs = {"means3D": "dL_dmeans3D", "opacities": "dL_dopacity", "shs": "dL_dsh", "colors_precomp": "dL_dcolors",
             "scales": "dL_dscales", "rotations": "dL_drotations", "cov3D_precomp": "dL_dcov3D"}
    for k, t in inp.items():
        ok, rel = common.allclose_rel(og[pairs[k]].reshape(t.shape), t.grad.numpy(), rtol=2e-4, atol=1e-7)
        assert ok, f"{mode} aa={antialiasing}: oracle d{k} vs autograd rel err {rel:.3e}"


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
