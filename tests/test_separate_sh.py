"""Separate-DC rasterizer input (`dc=`), SURVEY.md §8f row 4 (needs an MI355X: -m gpu).

train.py renders with ``rasterizer(dc=features_dc, shs=features_rest, ...)`` whenever the package
exports SparseGaussianAdam (train.py:37-41, 81, 111; gaussian_renderer/__init__.py:82-100).  The
two arrays are the two halves of the (P,16,3) coefficient array the full-SH path takes, so the
separate-DC path must give the SAME results as the full-SH path (itself pinned against the oracle
in test_gpu_parity.py) -- bit for bit, since both evaluate the same coefficients in the same
order: image, radii, invdepth and every gradient, with dL/ddc and dL/dshs being the two halves of
dL/dsh.  Cases: SH degree 3, an active degree below the stored one (train.py's degree ramp,
gaussian_model.py:oneupSHdegree), degree 0 with an empty rest array, antialiasing, rest arrays
narrower than 15 coefficients, and pointers that are only 4-byte aligned (the staging loaders'
scalar path).
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


def _settings(case, degree, antialiasing):
    dgr = _dgr()
    cam = case["cam"]
    return dgr.GaussianRasterizationSettings(
        case["H"], case["W"], cam.tanfovx, cam.tanfovy, case["bg"].to(DEV), 1.0, cam.world_view_transform.to(DEV),
        cam.full_proj_transform.to(DEV), degree, cam.camera_center.to(DEV), False, False, antialiasing)


def _misaligned(t, offset):
    """A contiguous copy of t whose data starts `offset` floats into its storage."""
    if offset == 0:
        return t.clone()
    buf = torch.zeros(t.numel() + offset, dtype=t.dtype, device=t.device)
    out = buf[offset:].view(t.shape)
    out.copy_(t)
    return out


def _run(case, degree, antialiasing, shs=None, dc=None, rest=None):
    dgr = _dgr()
    sc = case["scene"]
    t = {k: sc[k].to(DEV).clone().requires_grad_(True) for k in ("means3D", "opacities", "scales", "rotations")}
    kw = dict(means3D=t["means3D"], opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
    if shs is not None:
        t["shs"] = shs.detach().requires_grad_(True)
        kw["shs"] = t["shs"]
    else:
        t["dc"] = dc.detach().requires_grad_(True)
        t["rest"] = rest.detach().requires_grad_(True)
        kw["dc"], kw["shs"] = t["dc"], t["rest"]
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    color, radii, inv = dgr.GaussianRasterizer(_settings(case, degree, antialiasing))(means2D=means2D, **kw)
    loss = (color * case["grad_color"].to(DEV)).sum() + (inv * case["grad_invdepth"].to(DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    out = {"color": color, "radii": radii, "inv": inv, "means2D": means2D.grad}
    out.update({"d_" + k: v.grad for k, v in t.items()})
    return {k: v.detach().cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("degree,n_coef,antialiasing,offset", [
    (3, 16, False, 0), (3, 16, True, 0), (1, 16, False, 0), (2, 9, False, 0), (3, 16, False, 1), (1, 4, True, 3),
    (3, 21, False, 0), (3, 21, False, 1)])
def test_dc_path_equals_full_sh_path(degree, n_coef, antialiasing, offset):
    """n_coef 21: rows wider than the 16 coefficients degree 3 reads (the padded-row staging
    path); the extra coefficients get zero gradients on both paths."""
    case = common.make_case(P=3000, H=200, W=232)
    full = case["scene"]["shs"]
    if n_coef > full.shape[1]:
        extra = torch.randn((full.shape[0], n_coef - full.shape[1], 3), generator=torch.Generator().manual_seed(3))
        full = torch.cat([full, 0.05 * extra], dim=1)
    full = full[:, :n_coef].contiguous().to(DEV)
    a = _run(case, degree, antialiasing, shs=full)
    b = _run(case, degree, antialiasing, dc=_misaligned(full[:, :1].contiguous(), offset),
             rest=_misaligned(full[:, 1:].contiguous(), offset))
    for k in ("color", "radii", "inv", "means2D", "d_means3D", "d_opacities", "d_scales", "d_rotations"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    np.testing.assert_array_equal(a["d_shs"][:, :1], b["d_dc"])
    np.testing.assert_array_equal(a["d_shs"][:, 1:], b["d_rest"])
    assert b["d_dc"].shape == (3000, 1, 3) and b["d_rest"].shape == (3000, n_coef - 1, 3)


def test_degree0_with_empty_rest():
    """A degree-0 model: features_rest is (P,0,3) (gaussian_model.py max_sh_degree 0)."""
    case = common.make_case(P=2000, H=128, W=128, sh_degree=0)
    full = case["scene"]["shs"][:, :1].contiguous().to(DEV)
    a = _run(case, 0, False, shs=full)
    b = _run(case, 0, False, dc=full.clone(), rest=torch.zeros((2000, 0, 3), device=DEV))
    for k in ("color", "radii", "inv", "means2D", "d_means3D", "d_opacities", "d_scales", "d_rotations"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    np.testing.assert_array_equal(a["d_shs"], b["d_dc"])
    assert b["d_rest"].shape == (2000, 0, 3)


def test_narrow_sh_rows_match_wide_rows():
    """Full-SH path with rows of 4 coefficients (degree 1 model) vs rows of 16 at active degree 1:
    same image and gradients on the first 4 coefficients, exact zeros beyond them, and the narrow
    rows' gradients are not overwritten by a neighbour's zero fill."""
    case = common.make_case(P=2500, H=160, W=160)
    wide = case["scene"]["shs"].contiguous().to(DEV)
    a = _run(case, 1, False, shs=wide)
    b = _run(case, 1, False, shs=wide[:, :4].contiguous())
    for k in ("color", "radii", "inv", "means2D", "d_means3D", "d_opacities"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    np.testing.assert_array_equal(a["d_shs"][:, :4], b["d_shs"])
    assert not a["d_shs"][:, 4:].any()


def test_dc_backward_tuple_layout():
    """_C.rasterize_gaussians_backward with dc returns the accelerated upstream's 9-tuple
    (dL_ddc before dL_dsh); without dc the reference's 8-tuple."""
    dgr = _dgr()
    case = common.make_case(P=500, H=64, W=64)
    s = _settings(case, 3, False)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    dc, rest = sc["shs"][:, :1].contiguous(), sc["shs"][:, 1:].contiguous()
    e = torch.Tensor([])
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, 64, 64, rest, 3, s.campos, False, False, False, dc=dc)
    gc = case["grad_color"].to(DEV)
    g = dgr._C.rasterize_gaussians_backward(
        s.bg, sc["means3D"], radii, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, gc, e, rest, 3, s.campos, geom, L, binning, img, False, False, dc=dc)
    assert len(g) == 9
    assert tuple(g[5].shape) == (500, 1, 3) and tuple(g[6].shape) == (500, 15, 3)
    with pytest.raises(RuntimeError):
        dgr._C.rasterize_gaussians(
            s.bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
            s.projmatrix, s.tanfovx, s.tanfovy, 64, 64, rest, 3, s.campos, False, False, False, dc=dc[:10])


def test_dc_gradients_share_one_buffer():
    """With dc=, the parameter gradients are consecutive views of one buffer in
    multiview.PARAM_ORDER_DC (means3D | dc | rest | opacity | scales | rotations), so the
    multi-GPU step all-reduces them in place as in the single-array layout."""
    from diff_gaussian_rasterization import multiview
    dgr = _dgr()
    case = common.make_case(P=800, H=64, W=80)
    sc = case["scene"]
    t = {"means3D": sc["means3D"], "dc": sc["shs"][:, :1].contiguous(), "shs": sc["shs"][:, 1:].contiguous(),
         "opacities": sc["opacities"], "scales": sc["scales"], "rotations": sc["rotations"]}
    t = {k: v.to(DEV).clone().requires_grad_(True) for k, v in t.items()}
    color, radii, inv = dgr.GaussianRasterizer(_settings(case, 3, False))(
        means2D=torch.zeros_like(t["means3D"], requires_grad=True), **t)
    torch.autograd.backward([color, inv], [case["grad_color"].to(DEV), case["grad_invdepth"].to(DEV)])
    flat = multiview.flat_grad_view(t, multiview.PARAM_ORDER_DC)
    assert flat is not None
    assert flat.numel() == sum(p.numel() for p in t.values())
    torch.testing.assert_close(flat, multiview.grad_bucket(t, multiview.PARAM_ORDER_DC), rtol=0, atol=0)


def test_dc_with_precomputed_colors_raises():
    """dc= is SH input: together with colors_precomp it breaks the reference's exactly-one rule
    (diff_gaussian_rasterization/__init__.py:178-182)."""
    dgr = _dgr()
    case = common.make_case(P=100, H=32, W=32)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    with pytest.raises(Exception, match="exactly one of either SHs or precomputed colors|excatly one"):
        dgr.GaussianRasterizer(_settings(case, 3, False))(
            means3D=sc["means3D"], means2D=torch.zeros_like(sc["means3D"]), opacities=sc["opacities"],
            dc=sc["shs"][:, :1].contiguous(), colors_precomp=torch.rand(100, 3, device=DEV), scales=sc["scales"],
            rotations=sc["rotations"])


def _golden_sh_files():
    import os
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    out = []
    for f in sorted(os.listdir(d)) if os.path.isdir(d) else []:
        if f.endswith(".npz"):
            z = np.load(os.path.join(d, f), allow_pickle=False)
            if z["shs"].size and z["shs"].shape[1] > 1:
                out.append(os.path.join(d, f))
    return out


@pytest.mark.parametrize("path", _golden_sh_files(), ids=lambda p: p.rsplit("/", 1)[-1])
def test_dc_gradients_match_oracle_fixture(path):
    """gsr_backward_dc's dL/ddc and dL/drest against the oracle's dL/dsh (the committed
    fixtures), split into coefficient 0 and the rest -- a direct oracle check of the dc= path,
    not only a comparison with the full-SH HIP path (gaussian_renderer/__init__.py:90-100)."""
    dgr = _dgr()
    z = np.load(path, allow_pickle=False)
    H, W = int(z["H"]), int(z["W"])
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k], dtype=np.float32)).to(DEV)  # noqa: E731
    s = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(z["tanfovx"]), tanfovy=float(z["tanfovy"]), bg=t("bg"),
        scale_modifier=float(z["scale_modifier"]), viewmatrix=t("viewmatrix"), projmatrix=t("projmatrix"),
        sh_degree=int(z["sh_degree"]), campos=t("campos"), prefiltered=False, debug=False,
        antialiasing=bool(z["antialiasing"]))
    kw = {k: t(k).requires_grad_(True) for k in ["means3D", "opacities", "scales", "rotations", "cov3D_precomp"]
          if z[k].size}
    sh = t("shs")
    dc = sh[:, :1].contiguous().requires_grad_(True)
    rest = sh[:, 1:].contiguous().requires_grad_(True)
    means2D = torch.zeros_like(kw["means3D"], requires_grad=True)
    color, radii, inv = dgr.GaussianRasterizer(s)(means2D=means2D, dc=dc, shs=rest, **kw)
    torch.autograd.backward([color, inv], [t("grad_color"), t("grad_invdepth")])
    torch.cuda.synchronize()
    ref = z["dL_dsh"].reshape(sh.shape)
    for name, hip, r in (("dL_ddc", dc.grad, ref[:, :1]), ("dL_drest", rest.grad, ref[:, 1:]),
                         ("dL_dmeans3D", kw["means3D"].grad, z["dL_dmeans3D"])):
        ok, rel = common.allclose_rel(hip.cpu().numpy(), r.reshape(hip.shape))
        assert ok, f"{path}: {name} rel err {rel:.3e}"
