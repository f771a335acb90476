"""BASELINE config 2 at full size, HIP vs the C oracle (needs an MI355X: -m gpu).

The bench's headline workload exactly: 1,000,000 seed-0 Gaussians, SH degree 3, one 1920x1080
ring view (view 0), the bench's dL/dpixel (synthetic.make_grads seed 1), antialiasing off and on.
The oracle runs multi-threaded on the GPU box's host (about a second per case).

* bit-exact: num_rendered, radii, the sorted tile|depth keys, their Gaussian ids and the
  per-tile ranges (rasterizer_impl.cu:250-320);
* render state: colour, inverse depth, final_T and n_contrib through common.check_render
  (forward.cu:277-400);
* all eight outputs of rasterize_gaussians_backward (rasterize_points.cu:222) -- dL/dmean2D,
  dL/dcolors, dL/dopacity, dL/dmeans3D, dL/dcov3D, dL/dsh, dL/dscales, dL/drotations -- within
  1e-4 of max|ref| for every Gaussian outside the walk of a flipped pixel, and every outlier
  attributed to one (common.check_grad_attributed; backward.cu:452-638, 147-449);
* the separate-DC form (dc=, gsr_backward_dc) against the oracle's dL/dsh split into
  coefficient 0 and the rest (gaussian_renderer/__init__.py:90-100).
"""
import os

import numpy as np
import pytest
import torch

import common

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
P, H, W = 1_000_000, 1080, 1920
L_VIEW0 = 5_813_426  # num_rendered of this view with antialiasing off (round-1 bench, profiles/r01_bench.json)


@pytest.fixture(scope="module")
def case():
    return common.make_case(P=P, H=H, W=W)


def _settings(case, antialiasing):
    import diff_gaussian_rasterization as dgr
    cam = case["cam"]
    return dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=case["bg"].to(DEV),
        scale_modifier=1.0, viewmatrix=cam.world_view_transform.to(DEV), projmatrix=cam.full_proj_transform.to(DEV),
        sh_degree=3, campos=cam.camera_center.to(DEV), prefiltered=False, debug=False, antialiasing=antialiasing)


# Gradients: every element within common.GRAD_RTOL (1e-4) of max|ref|, except the Gaussians in the
# walk of a flipped pixel (an alpha within an ulp of 1/255 or of the stop rule; common.check_render),
# whose gradients gain or lose that pixel's term: within common.GRAD_RTOL_ATTRIBUTED there, and the
# test asserts that EVERY element beyond the tolerance belongs to such a Gaussian
# (common.check_grad_attributed).  The bulk is bounded per element by
# common.check_rel, and its accuracy against the float64 render backward (the oracle's decisions)
# by common.check_rel_truth: no worse than 1.5x the reference's own float32 order.


def _grad_check(name, hip, ref, affected, suspect_rows, truth=None):
    # outliers may sit in the walk of any decision suspect (common.DECISION_ATOL), not only of a flipped pixel
    common.check_grad_attributed(name, hip, ref, suspect_rows)
    so = common.check_rel_truth(name, hip, ref, truth, suspect_rows)[1] if truth is not None else None
    # per element, not only relative to the max
    common.check_rel(name, hip, ref, suspect_rows, so)


@pytest.mark.parametrize("antialiasing", [False, True])
def test_config2_full_size(case, antialiasing):
    import diff_gaussian_rasterization as dgr
    from test_gpu_parity import _img_state
    threads = min(16, os.cpu_count() or 1)
    o, og = common.run_oracle(case, antialiasing=antialiasing, nthreads=threads)
    if not antialiasing:
        assert o.num_rendered == L_VIEW0
    s = _settings(case, antialiasing)
    sc = {k: v.to(DEV).contiguous() for k, v in case["scene"].items()}
    e = torch.Tensor([])
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, H, W, sc["shs"], 3, s.campos, False, antialiasing, False)
    torch.cuda.synchronize()
    assert L == o.num_rendered
    np.testing.assert_array_equal(radii.cpu().numpy(), o.radii)
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, W, H)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))
    del keys, vals
    fT, nc = _img_state(img, W, H)
    flips, sus = [], []
    common.check_render(f"config2 aa={antialiasing}",
                        {"color": color.cpu().numpy(), "invdepth": inv.cpu().numpy(), "final_T": fT, "n_contrib": nc},
                        {"color": o.color, "invdepth": o.invdepth, "final_T": o.get("final_T"),
                         "n_contrib": o.get("n_contrib")}, flips=flips, suspects=sus)
    affected = common.flip_gaussians(flips[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
    suspect_rows = common.flip_gaussians(sus[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)

    gc, gi = case["grad_color"].to(DEV), case["grad_invdepth"].to(DEV)
    out = dgr._C.rasterize_gaussians_backward(
        s.bg, sc["means3D"], radii, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, gc, gi, sc["shs"], 3, s.campos, geom, L, binning, img, antialiasing,
        False)
    names = ["dL_dmean2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    torch.cuda.synchronize()
    g64 = o.backward(case["grad_color"], case["grad_invdepth"], f64=True)
    for n, t in zip(names, out):
        _grad_check(f"config2 aa={antialiasing} {n}", t.cpu().numpy(), og[n].reshape(t.shape), affected,
                    suspect_rows, g64[n].reshape(t.shape))
    del out, g64

    # the separate-DC form on the same view: dL/ddc and dL/drest against the oracle's dL/dsh split
    dc, rest = sc["shs"][:, :1].contiguous(), sc["shs"][:, 1:].contiguous()
    L2, color2, radii2, geom2, binning2, img2, inv2 = dgr._C.rasterize_gaussians(
        s.bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, H, W, rest, 3, s.campos, False, antialiasing, False, dc=dc)
    assert L2 == L and torch.equal(color2, color) and torch.equal(radii2, radii)
    out = dgr._C.rasterize_gaussians_backward(
        s.bg, sc["means3D"], radii2, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, gc, gi, rest, 3, s.campos, geom2, L2, binning2, img2, antialiasing,
        False, dc=dc)
    torch.cuda.synchronize()
    sh_ref = og["dL_dsh"].reshape(P, 16, 3)
    _grad_check(f"config2 aa={antialiasing} dc dL_ddc", out[5].cpu().numpy(), sh_ref[:, :1], affected, suspect_rows)
    _grad_check(f"config2 aa={antialiasing} dc dL_drest", out[6].cpu().numpy(), sh_ref[:, 1:], affected, suspect_rows)
    _grad_check(f"config2 aa={antialiasing} dc dL_dmeans3D", out[3].cpu().numpy(), og["dL_dmeans3D"], affected,
                suspect_rows)


def test_config2_batched_views_match_single_views(case):
    """The bench's batched step at full size: a MultiViewRasterizer batch of ring views 0 and 1
    (batched prefix, emission fused into the tile sort, one render launch per pass) against one
    GaussianRasterizer call per view (the path the oracle comparisons above check): images, radii,
    inverse depths and each view's dL/dmean2D bit-identical, parameter gradients equal up to fp32
    summation order (1e-5 of their max)."""
    import diff_gaussian_rasterization as dgr
    import synthetic
    cams = [synthetic.Camera(W, H, view=v) for v in (0, 1)]
    settings = [dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, bg=case["bg"].to(DEV), scale_modifier=1.0,
        viewmatrix=c.world_view_transform.to(DEV), projmatrix=c.full_proj_transform.to(DEV), sh_degree=3,
        campos=c.camera_center.to(DEV), prefiltered=False, debug=False, antialiasing=False) for c in cams]
    grads = [tuple(g.to(DEV) for g in synthetic.make_grads(H, W, seed=1 + v)) for v in (0, 1)]

    def leaves():
        return {k: case["scene"][k].to(DEV).clone().requires_grad_(True)
                for k in ("means3D", "shs", "opacities", "scales", "rotations")}

    single = leaves()
    outs, m2 = [], []
    for s, (gc, gi) in zip(settings, grads):
        means2D = torch.zeros_like(single["means3D"], requires_grad=True)
        c, r, i = dgr.GaussianRasterizer(s)(means2D=means2D, **single)
        torch.autograd.backward([c, i], [gc, gi])
        outs.append((c.detach(), r, i.detach()))
        m2.append(means2D.grad)
    multi = leaves()
    means2D = torch.zeros((2, P, 3), device=DEV, requires_grad=True)
    c, r, i = dgr.MultiViewRasterizer(settings)(means2D=means2D, **multi)
    torch.autograd.backward([c, i], [torch.stack([g[0] for g in grads]), torch.stack([g[1] for g in grads])])
    torch.cuda.synchronize()
    for v in (0, 1):
        assert torch.equal(c[v].detach(), outs[v][0]), f"view {v} image"
        assert torch.equal(r[v], outs[v][1]), f"view {v} radii"
        assert torch.equal(i[v].detach(), outs[v][2]), f"view {v} invdepth"
        assert torch.equal(means2D.grad[v], m2[v]), f"view {v} dL/dmean2D"
    for k in single:
        ok, rel = common.allclose_rel(multi[k].grad.cpu().numpy(), single[k].grad.cpu().numpy(), rtol=1e-5,
                                      atol=1e-12)
        assert ok, f"d{k}: batch vs single views rel {rel:.3e}"
