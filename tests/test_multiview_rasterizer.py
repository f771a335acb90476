"""MultiViewRasterizer: a batch of views as one autograd node (needs an MI355X: -m gpu).

* forward: every view's image, radii and inverse depth are bit-identical to GaussianRasterizer on
  that view (the same kernels run per view);
* backward (gsr_backward_views: every view's render backward, then ONE preprocess backward over
  the Gaussians): each view's screen-space gradient (means2D.grad[v]) is bit-identical to the
  single-view one; the parameter gradients equal the sum of the single-view gradients up to fp32
  summation order (1e-5 of each tensor's max), and the sum of the C oracle's per-view gradients
  within the common gradient tolerance -- for every input mode, with antialiasing, with dc= and
  with in-place accumulation into existing .grad buffers.
"""
import numpy as np
import pytest
import torch

import common
import synthetic

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
V, P, H, W = 4, 4000, 144, 176


def _settings(cam, antialiasing, bg):
    import diff_gaussian_rasterization as dgr
    return dgr.GaussianRasterizationSettings(
        H, W, cam.tanfovx, cam.tanfovy, bg, 1.0, cam.world_view_transform.to(DEV), cam.full_proj_transform.to(DEV),
        3, cam.camera_center.to(DEV), False, False, antialiasing)


def _case():
    case = common.make_case(P=P, H=H, W=W, bg=(0.1, 0.2, 0.3))
    g = torch.Generator().manual_seed(7)
    case["colors_precomp"] = torch.rand(P, 3, generator=g)
    o, _ = common.run_oracle(case, backward=False)
    case["cov3D_precomp"] = torch.from_numpy(o.get("cov3D").copy())
    case["cams"] = [synthetic.Camera(W, H, view=v) for v in range(V)]
    case["grads"] = [synthetic.make_grads(H, W, seed=30 + v) for v in range(V)]
    return case


def _leaves(case, mode):
    sc = case["scene"]
    t = {"means3D": sc["means3D"], "opacities": sc["opacities"]}
    if mode == "dc":
        t["dc"], t["shs"] = sc["shs"][:, :1].contiguous(), sc["shs"][:, 1:].contiguous()
    elif mode.startswith("sh"):
        t["shs"] = sc["shs"]
    else:
        t["colors_precomp"] = case["colors_precomp"]
    if mode.endswith("cov"):
        t["cov3D_precomp"] = case["cov3D_precomp"]
    else:
        t["scales"], t["rotations"] = sc["scales"], sc["rotations"]
    return {k: v.to(DEV).clone().requires_grad_(True) for k, v in t.items()}


@pytest.mark.parametrize("mode,antialiasing", [("sh_scales", False), ("sh_scales", True), ("colors_cov", False),
                                               ("dc", False), ("dc", True)])
def test_multiview_matches_single_views(mode, antialiasing):
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    settings = [_settings(c, antialiasing, bg) for c in case["cams"]]
    gc = torch.stack([g[0] for g in case["grads"]]).to(DEV)
    gi = torch.stack([g[1] for g in case["grads"]]).to(DEV)

    # single views, gradients accumulated by autograd
    single = _leaves(case, mode)
    imgs, radii, invs, m2 = [], [], [], []
    for v, s in enumerate(settings):
        means2D = torch.zeros_like(single["means3D"], requires_grad=True)
        c, r, i = dgr.GaussianRasterizer(s)(means2D=means2D, **single)
        torch.autograd.backward([c, i], [gc[v], gi[v]])
        imgs.append(c.detach())
        radii.append(r)
        invs.append(i.detach())
        m2.append(means2D.grad)

    multi = _leaves(case, mode)
    means2D = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
    c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **multi)
    torch.autograd.backward([c, i], [gc, gi])
    torch.cuda.synchronize()
    assert torch.equal(c.detach(), torch.stack(imgs)) and torch.equal(i.detach(), torch.stack(invs))
    assert torch.equal(r, torch.stack(radii))
    assert torch.equal(means2D.grad, torch.stack(m2)), "screen-space gradients"
    for k in single:
        a, b = multi[k].grad.cpu().numpy(), single[k].grad.cpu().numpy()
        ok, rel = common.allclose_rel(a, b, rtol=1e-5, atol=1e-9)
        assert ok, f"{mode} aa={antialiasing}: d{k} multi vs sum of single views rel {rel:.3e}"


def test_multiview_matches_oracle_sum():
    """Parameter gradients of the batch against the sum of the C oracle's per-view gradients."""
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    settings = [_settings(c, False, bg) for c in case["cams"]]
    ref = None
    for v, cam in enumerate(case["cams"]):
        cv = dict(case, cam=cam, grad_color=case["grads"][v][0], grad_invdepth=case["grads"][v][1])
        _, og = common.run_oracle(cv, nthreads=8)
        ref = og if ref is None else {k: ref[k] + og[k] for k in ref}
    t = _leaves(case, "sh_scales")
    means2D = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
    c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **t)
    torch.autograd.backward([c, i], [torch.stack([g[0] for g in case["grads"]]).to(DEV),
                                     torch.stack([g[1] for g in case["grads"]]).to(DEV)])
    torch.cuda.synchronize()
    for hk, ok_ in {"means3D": "dL_dmeans3D", "shs": "dL_dsh", "opacities": "dL_dopacity", "scales": "dL_dscales",
                    "rotations": "dL_drotations"}.items():
        a = t[hk].grad.cpu().numpy()
        ok, rel = common.allclose_rel(a, ref[ok_].reshape(a.shape))
        assert ok, f"d{hk} vs oracle sum rel {rel:.3e}"


def test_multiview_in_place_accumulation():
    """A second batch into the same .grad (accumulate_grads_in_place) equals autograd's own add."""
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    settings = [_settings(c, False, bg) for c in case["cams"]]
    gc = torch.stack([g[0] for g in case["grads"]]).to(DEV)
    gi = torch.stack([g[1] for g in case["grads"]]).to(DEV)

    def run(fused):
        t = _leaves(case, "sh_scales")
        for _ in range(2):
            means2D = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
            with dgr.accumulate_grads_in_place(fused):
                c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **t)
            torch.autograd.backward([c, i], [gc, gi])
        torch.cuda.synchronize()
        return {k: v.grad.cpu().numpy() for k, v in t.items()}

    a, b = run(False), run(True)
    for k in a:
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)


def test_multiview_argument_checks():
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    s = [_settings(c, False, bg) for c in case["cams"]]
    with pytest.raises(ValueError):
        dgr.MultiViewRasterizer([s[0], s[1]._replace(antialiasing=True)])
    with pytest.raises(ValueError):
        dgr.MultiViewRasterizer(s * 5)
    t = _leaves(case, "sh_scales")
    with pytest.raises(Exception, match="excatly one"):
        dgr.MultiViewRasterizer(s)(means3D=t["means3D"], means2D=torch.zeros((V, P, 3), device=DEV),
                                   opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])


@pytest.mark.parametrize("mode,antialiasing", [("sh_scales", False), ("colors_cov", False), ("dc", True)])
def test_deferred_backward_matches_multiview(mode, antialiasing):
    """deferred_backward (per-view forward + render backward, one batched preprocess backward at
    the context's exit) against MultiViewRasterizer on the same views: bit-identical parameter and
    screen-space gradients (the same kernels on the same records)."""
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    settings = [_settings(c, antialiasing, bg) for c in case["cams"]]
    gc = torch.stack([g[0] for g in case["grads"]]).to(DEV)
    gi = torch.stack([g[1] for g in case["grads"]]).to(DEV)

    multi = _leaves(case, mode)
    means2D = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
    c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **multi)
    torch.autograd.backward([c, i], [gc, gi])

    deferred = _leaves(case, mode)
    m2 = [torch.zeros((P, 3), device=DEV, requires_grad=True) for _ in range(V)]
    with dgr.deferred_backward():
        for v, s in enumerate(settings):
            cv, rv, iv = dgr.GaussianRasterizer(s)(means2D=m2[v], **deferred)
            torch.autograd.backward([cv, iv], [gc[v], gi[v]])
            assert torch.equal(cv.detach(), c[v].detach()) and torch.equal(rv, r[v])
        assert all(t.grad is None for t in deferred.values()), "gradients arrive at the context's exit"
    torch.cuda.synchronize()
    assert torch.equal(torch.stack([m.grad for m in m2]), means2D.grad)
    for k in multi:
        assert torch.equal(deferred[k].grad, multi[k].grad), k


def test_deferred_backward_after_context_exit():
    """A forward inside deferred_backward whose backward runs after the context has exited: its
    BACKWARD::preprocess runs at once, alone -- the gradients equal the ordinary
    backward's (dL/dmean2D bitwise, the parameters up to the batched kernel's summation order),
    nothing is dropped."""
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    s = _settings(case["cams"][0], False, bg)
    gc, gi = (g.to(DEV) for g in case["grads"][0])

    plain = _leaves(case, "sh_scales")
    m_plain = torch.zeros((P, 3), device=DEV, requires_grad=True)
    c, _, i = dgr.GaussianRasterizer(s)(means2D=m_plain, **plain)
    torch.autograd.backward([c, i], [gc, gi])

    late = _leaves(case, "sh_scales")
    m_late = torch.zeros((P, 3), device=DEV, requires_grad=True)
    with dgr.deferred_backward():
        c2, _, i2 = dgr.GaussianRasterizer(s)(means2D=m_late, **late)
    torch.autograd.backward([c2, i2], [gc, gi])  # after the exit: its batch is already closed
    torch.cuda.synchronize()
    assert torch.equal(m_late.grad, m_plain.grad)
    for k in plain:
        assert late[k].grad is not None, f"d{k} dropped"
        ok, rel = common.allclose_rel(late[k].grad.cpu().numpy(), plain[k].grad.cpu().numpy(), rtol=1e-5,
                                      atol=1e-12)
        assert ok, f"d{k}: late deferred vs plain rel {rel:.3e}"


# (the views alternate between two streams on purpose, so autograd notes that a leaf's gradient
# arrives from another stream than the leaf's own)
@pytest.mark.filterwarnings("ignore:The AccumulateGrad node's stream does not match")
def test_deferred_backward_activations_streams_accumulation():
    """The train.py shape: activations between the parameters and the rasterizer (exp, sigmoid,
    normalize), views alternating between two streams, and a second batch adding into the .grad of
    the first -- against the ordinary per-view backward passes (fp32 summation order: 1e-5)."""
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    settings = [_settings(c, False, bg) for c in case["cams"]]
    sc = case["scene"]
    raw0 = {"xyz": sc["means3D"], "f": sc["shs"], "op": torch.logit(sc["opacities"].clamp(1e-4, 1 - 1e-4)),
            "scl": torch.log(sc["scales"]), "rot": sc["rotations"] * 1.7}

    def run(deferred):
        raw = {k: v.to(DEV).clone().requires_grad_(True) for k, v in raw0.items()}
        streams = [torch.cuda.current_stream(DEV), torch.cuda.Stream(DEV)]
        for rep in range(2):
            inputs = {"means3D": raw["xyz"], "shs": raw["f"], "opacities": torch.sigmoid(raw["op"]),
                      "scales": torch.exp(raw["scl"]), "rotations": torch.nn.functional.normalize(raw["rot"])}
            streams[1].wait_stream(streams[0])
            with (dgr.deferred_backward() if deferred else torch.enable_grad()):
                for v, s in enumerate(settings):
                    with torch.cuda.stream(streams[v % 2]):
                        m2 = torch.zeros((P, 3), device=DEV, requires_grad=True)
                        cv, _, iv = dgr.GaussianRasterizer(s)(means2D=m2, **inputs)
                        # the views share the activations: the ordinary path backs through them per view
                        torch.autograd.backward([cv, iv], [case["grads"][v][0].to(DEV), case["grads"][v][1].to(DEV)],
                                                retain_graph=not deferred)
                streams[0].wait_stream(streams[1])
        torch.cuda.synchronize()
        return {k: v.grad.cpu().numpy() for k, v in raw.items()}

    a, b = run(False), run(True)
    for k in a:
        ok, rel = common.allclose_rel(b[k], a[k], rtol=1e-5, atol=1e-9)
        assert ok, f"d{k}: deferred vs per-view rel {rel:.3e}"


def _settings_hw(cam, H_, W_, bg, scale_modifier=1.0, empty=False):
    import diff_gaussian_rasterization as dgr
    wv = cam.world_view_transform.clone()
    if empty:  # every Gaussian far behind the camera: L = 0 for this view
        wv[3, 2] -= 1000.0
    proj = wv.unsqueeze(0).bmm(cam.projection_matrix.unsqueeze(0)).squeeze(0)
    return dgr.GaussianRasterizationSettings(H_, W_, cam.tanfovx, cam.tanfovy, bg, scale_modifier, wv.to(DEV),
                                             proj.to(DEV), 3, wv.inverse()[3, :3].to(DEV), False, False, False)


@pytest.mark.parametrize("H_,W_", [(144, 176), (304, 400)])
def test_multiview_large_batch_big_splats_empty_view(H_, W_):
    """10 views (two launch groups of the batched kernels), one of them empty (L = 0), splats scaled
    6x so that a 256-rank chunk of the fused emission + tile-sort pass holds several 2,048-instance
    rounds; 99 tiles (the fused pass is the only pass) and 475 tiles (two passes).  Images, radii,
    inverse depths and screen-space gradients bit-identical to single-view GaussianRasterizer calls
    (unfused emission, per-view launches); parameter gradients equal up to summation order."""
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    Vb = 10
    case = common.make_case(P=P, H=H_, W=W_, bg=(0.1, 0.2, 0.3))
    bg = case["bg"].to(DEV)
    cams = [synthetic.Camera(W_, H_, view=v, n_views=Vb) for v in range(Vb)]
    settings = [_settings_hw(c, H_, W_, bg, scale_modifier=6.0, empty=(v == 3)) for v, c in enumerate(cams)]
    grads = [synthetic.make_grads(H_, W_, seed=60 + v) for v in range(Vb)]
    gc = torch.stack([g[0] for g in grads]).to(DEV)
    gi = torch.stack([g[1] for g in grads]).to(DEV)

    single = _leaves(case, "sh_scales")
    imgs, radii, invs, m2, Ls = [], [], [], [], []
    for v, s in enumerate(settings):
        means2D = torch.zeros_like(single["means3D"], requires_grad=True)
        c, r, i = dgr.GaussianRasterizer(s)(means2D=means2D, **single)
        Ls.append(_C._binning_hint[DEV])
        torch.autograd.backward([c, i], [gc[v], gi[v]])
        imgs.append(c.detach())
        radii.append(r)
        invs.append(i.detach())
        m2.append(means2D.grad)
    assert Ls[3] == 0 and min(L for v, L in enumerate(Ls) if v != 3) > 0
    assert max(Ls) > 4 * 2048, f"splats too small for multi-round chunks (L = {max(Ls)})"

    multi = _leaves(case, "sh_scales")
    means2D = torch.zeros((Vb, P, 3), device=DEV, requires_grad=True)
    c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **multi)
    torch.autograd.backward([c, i], [gc, gi])
    torch.cuda.synchronize()
    for v in range(Vb):
        assert torch.equal(c[v].detach(), imgs[v]), f"view {v} image"
        assert torch.equal(i[v].detach(), invs[v]), f"view {v} invdepth"
        assert torch.equal(r[v], radii[v]), f"view {v} radii"
        assert torch.equal(means2D.grad[v], m2[v]), f"view {v} screen-space gradient"
    for k in single:
        ok, rel = common.allclose_rel(multi[k].grad.cpu().numpy(), single[k].grad.cpu().numpy(), rtol=1e-5,
                                      atol=1e-9)
        assert ok, f"d{k} multi vs sum of single views rel {rel:.3e}"


def test_backward_bitwise_reproducible():
    """render_bwd sums an entry's quadrant partials in LDS in a fixed group order (no global float
    atomics): repeated backwards of the same batch give bitwise-identical gradients."""
    import diff_gaussian_rasterization as dgr
    case = _case()
    bg = case["bg"].to(DEV)
    settings = [_settings(c, True, bg) for c in case["cams"]]
    gc = torch.stack([g[0] for g in case["grads"]]).to(DEV)
    gi = torch.stack([g[1] for g in case["grads"]]).to(DEV)
    runs = []
    for _ in range(3):
        t = _leaves(case, "sh_scales")
        means2D = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
        c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **t)
        torch.autograd.backward([c, i], [gc, gi])
        torch.cuda.synchronize()
        runs.append({"means2D": means2D.grad.clone(), **{k: v.grad.clone() for k, v in t.items()}})
    assert any(float(runs[0][k].abs().max()) > 0 for k in runs[0])
    for r in runs[1:]:
        for k in runs[0]:
            assert torch.equal(r[k], runs[0][k]), f"d{k} differs between identical backwards"


@pytest.mark.parametrize("nv,p", [(8, 990), (3, 4000), (10, 1500)])
def test_two_chunk_preprocess_backward_matches_one_chunk_kernel(nv, p):
    """The batched preprocess backward runs as the two-chunk kernel for interleaved SH rows
    (preprocess_bwd_views_pipe_kernel: 3+ views) and as the one-chunk kernel for the separate-DC
    layout: the same arithmetic on the same values, so every gradient is bitwise identical between
    the two layouts -- with an odd number of chunks (a workgroup with one chunk) and 4 / 8 / 16 lanes
    per Gaussian."""
    import diff_gaussian_rasterization as dgr
    case = common.make_case(P=p, H=H, W=W, bg=(0.1, 0.2, 0.3))
    bg = case["bg"].to(DEV)
    cams = [synthetic.Camera(W, H, view=v, n_views=nv) for v in range(nv)]
    settings = [_settings(c, False, bg) for c in cams]
    grads = [synthetic.make_grads(H, W, seed=80 + v) for v in range(nv)]
    gc = torch.stack([g[0] for g in grads]).to(DEV)
    gi = torch.stack([g[1] for g in grads]).to(DEV)
    out = {}
    for mode in ("sh_scales", "dc"):
        t = _leaves(case, mode)
        means2D = torch.zeros((nv, p, 3), device=DEV, requires_grad=True)
        c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **t)
        torch.autograd.backward([c, i], [gc, gi])
        torch.cuda.synchronize()
        g = {k: v.grad for k, v in t.items()}
        if mode == "dc":
            g["shs"] = torch.cat([g.pop("dc"), g["shs"]], dim=1)
        g["means2D"] = means2D.grad
        out[mode] = g
    for k, a in out["sh_scales"].items():
        assert torch.equal(a, out["dc"][k]), f"{nv} views, P={p}: d{k} differs between the two kernels"
