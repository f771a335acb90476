"""In-place gradient accumulation (diff_gaussian_rasterization.accumulate_grads_in_place,
gsr_backward_dc_acc), needs an MI355X: -m gpu.

Several views rendered into the same parameters must leave .grad bit-identical to autograd's own
accumulation (`grad += new`, one fp32 add per element): for every input mode, with dc=, with
non-leaf inputs (activations, which keep the ordinary path) and with a hook on a leaf."""
import numpy as np
import pytest
import torch

import common

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _settings(case, view_cam, antialiasing=False):
    import diff_gaussian_rasterization as dgr
    return dgr.GaussianRasterizationSettings(
        case["H"], case["W"], view_cam.tanfovx, view_cam.tanfovy, case["bg"].to(DEV), 1.0,
        view_cam.world_view_transform.to(DEV), view_cam.full_proj_transform.to(DEV), 3,
        view_cam.camera_center.to(DEV), False, False, antialiasing)


def _run(case, mode, fused, activations=False, hook=False, antialiasing=False):
    import diff_gaussian_rasterization as dgr
    import synthetic
    sc = case["scene"]
    leaves = {"means3D": sc["means3D"], "opacities": sc["opacities"]}
    if mode == "dc":
        leaves["dc"], leaves["shs"] = sc["shs"][:, :1].contiguous(), sc["shs"][:, 1:].contiguous()
    elif mode.startswith("sh"):
        leaves["shs"] = sc["shs"]
    else:
        leaves["colors_precomp"] = case["colors_precomp"]
    if mode.endswith("cov"):
        leaves["cov3D_precomp"] = case["cov3D_precomp"]
    else:
        leaves["scales"], leaves["rotations"] = sc["scales"], sc["rotations"]
    leaves = {k: v.to(DEV).clone().requires_grad_(True) for k, v in leaves.items()}
    if activations:  # scales / rotations through differentiable ops: non-leaf rasterizer inputs
        raw_s = torch.log(leaves.pop("scales")).detach().requires_grad_(True)
        raw_r = leaves.pop("rotations").detach().requires_grad_(True)
        leaves["raw_s"], leaves["raw_r"] = raw_s, raw_r
    if hook:
        leaves["opacities"].register_hook(lambda g: g * 1.0)
    for v in range(3):
        cam = synthetic.Camera(case["W"], case["H"], view=v)
        kw = {k: t for k, t in leaves.items() if not k.startswith("raw")}
        if activations:
            kw["scales"] = torch.exp(leaves["raw_s"])
            kw["rotations"] = torch.nn.functional.normalize(leaves["raw_r"])
        means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
        with dgr.accumulate_grads_in_place(fused):
            color, radii, inv = dgr.GaussianRasterizer(_settings(case, cam, antialiasing))(means2D=means2D, **kw)
        gc, gi = synthetic.make_grads(case["H"], case["W"], seed=10 + v)
        torch.autograd.backward([color, inv], [gc.to(DEV), gi.to(DEV)])
    torch.cuda.synchronize()
    return {k: t.grad.detach().cpu().numpy() for k, t in leaves.items()}


@pytest.mark.parametrize("mode,activations,hook,antialiasing", [
    ("sh_scales", False, False, False), ("sh_scales", False, False, True), ("colors_cov", False, False, False),
    ("dc", False, False, False), ("dc", True, False, False), ("sh_scales", False, True, False)])
def test_in_place_accumulation_is_bit_identical(mode, activations, hook, antialiasing):
    case = common.make_case(P=3000, H=128, W=160)
    g = torch.Generator().manual_seed(7)
    case["colors_precomp"] = torch.rand(3000, 3, generator=g)
    o, _ = common.run_oracle(case, backward=False)
    case["cov3D_precomp"] = torch.from_numpy(o.get("cov3D").copy())
    ref = _run(case, mode, False, activations, hook, antialiasing)
    got = _run(case, mode, True, activations, hook, antialiasing)
    assert ref.keys() == got.keys()
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        assert np.abs(ref[k]).max() > 0, k


def test_accumulate_argument_checks():
    import diff_gaussian_rasterization as dgr
    case = common.make_case(P=200, H=32, W=32)
    sc = {k: v.to(DEV) for k, v in case["scene"].items()}
    e = torch.Tensor([])
    s = _settings(case, case["cam"])
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, 32, 32, sc["shs"], 3, s.campos, False, False, False)
    args = (s.bg, sc["means3D"], radii, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
            s.projmatrix, s.tanfovx, s.tanfovy, case["grad_color"].to(DEV), e, sc["shs"], 3, s.campos, geom, L,
            binning, img, False, False)
    with pytest.raises(RuntimeError, match="accumulate"):
        dgr._C.rasterize_gaussians_backward(*args, accumulate={"means3D": torch.zeros(5, device=DEV)})
    with pytest.raises(RuntimeError, match="unknown"):
        dgr._C.rasterize_gaussians_backward(*args, accumulate={"bogus": torch.zeros(600, device=DEV)})
    dst = torch.ones(200, 3, device=DEV)
    out = dgr._C.rasterize_gaussians_backward(*args, accumulate={"means3D": dst})
    plain = dgr._C.rasterize_gaussians_backward(*args)
    assert out[3] is None
    torch.testing.assert_close(dst, plain[3] + 1.0, rtol=0, atol=0)


def test_views_on_two_streams_match_one_stream():
    """bench.py's step: views alternate between two HIP streams (the forward of one view overlapping
    the backward of the previous); in-place accumulation stays ordered (the backward's event
    fence), so every gradient is bit-identical to the one-stream run."""
    import diff_gaussian_rasterization as dgr
    import synthetic
    case = common.make_case(P=20000, H=270, W=480)
    sc = {k: v.to(DEV).requires_grad_(True) for k, v in case["scene"].items()}
    cams = [synthetic.Camera(480, 270, view=v) for v in range(6)]
    grads = [tuple(t.to(DEV) for t in synthetic.make_grads(270, 480, seed=20 + v)) for v in range(6)]
    main = torch.cuda.current_stream(DEV)
    side = torch.cuda.Stream(DEV)

    def run(n_streams):
        for t in sc.values():
            t.grad = None
        streams = [main, side][:n_streams]
        for st in streams[1:]:
            st.wait_stream(main)
        for i, (cam, (gc, gi)) in enumerate(zip(cams, grads)):
            st = streams[i % n_streams]
            with torch.cuda.stream(st):
                means2D = torch.zeros_like(sc["means3D"], requires_grad=True)
                with dgr.accumulate_grads_in_place():
                    color, radii, inv = dgr.GaussianRasterizer(_settings(case, cam))(means2D=means2D, **sc)
                torch.autograd.backward([color, inv], [gc, gi])
        for st in streams[1:]:
            main.wait_stream(st)
        torch.cuda.synchronize()
        return {k: t.grad.detach().cpu().numpy().copy() for k, t in sc.items()}

    one = run(1)
    two = run(2)
    for k in one:
        np.testing.assert_array_equal(two[k], one[k], err_msg=k)
