"""The benchmarked step itself against the C oracle (needs an MI355X: -m gpu).

bench.py's default step, exactly: ONE MultiViewRasterizer call over BASELINE config 4's 8 ring
views of the config-2 scene (1,000,000 seed-0 Gaussians, SH degree 3, 1920x1080), each view's
dL/dpixel from synthetic.make_grads(seed=1 + v) as bench.py draws it, forward and backward
through autograd -- antialiasing off and on.  Per view, against the oracle run on that view
(forward.cu:277-400, backward.cu:452-638, rasterizer_impl.cu:250-320):

* bit-exact: num_rendered, radii, the sorted tile|depth keys, their Gaussian ids and the tile
  ranges (read back from the batch's own saved state through gsr_debug_sorted_keys);
* colour, inverse depth, final_T and n_contrib through common.check_render;
* the view's screen-space gradient means2D.grad[v] (dL/dmean2D) within the gradient tolerance.

The parameter gradients of the batch (one batched BACKWARD::preprocess over the 8 views) against
the SUM of the oracle's 8 per-view gradients: within 1e-4 of max|ref| outside the walks of the
views' flipped pixels, every outlier attributed to one (common.check_grad_attributed), and the
per-element relative-error bounds of common.check_rel.
"""
import os

import numpy as np
import pytest
import torch

import common
import synthetic

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
P, H, W, V = 1_000_000, 1080, 1920, 8
PARAM_KEYS = {"means3D": "dL_dmeans3D", "shs": "dL_dsh", "opacities": "dL_dopacity", "scales": "dL_dscales",
              "rotations": "dL_drotations"}


@pytest.fixture(scope="module")
def scene():
    return synthetic.make_scene(P, seed=0)


def _grad_check(name, hip, ref, affected, suspect_rows):
    # outliers may sit in the walk of any decision suspect (common.DECISION_ATOL), not only of a flipped
    # pixel: a blend decision taken the other way can move the colour by less than IMG_ATOL
    common.check_grad_attributed(name, hip, ref, suspect_rows)
    common.check_rel(name, hip, ref, suspect_rows)


@pytest.mark.parametrize("antialiasing", [False, True])
def test_bench_step_8_views(scene, antialiasing):
    import diff_gaussian_rasterization as dgr
    import oracle
    threads = min(16, os.cpu_count() or 1)
    bg = torch.zeros(3)
    cams = [synthetic.Camera(W, H, view=v, n_views=8) for v in range(V)]
    grads = [synthetic.make_grads(H, W, seed=1 + v) for v in range(V)]
    settings = [dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, bg=bg.to(DEV), scale_modifier=1.0,
        viewmatrix=c.world_view_transform.to(DEV), projmatrix=c.full_proj_transform.to(DEV), sh_degree=3,
        campos=c.camera_center.to(DEV), prefiltered=False, debug=False, antialiasing=antialiasing) for c in cams]

    # the bench step (bench.py step(): MultiViewRasterizer, autograd.backward on colour + invdepth)
    params = {k: v.to(DEV).requires_grad_(True) for k, v in scene.items()}
    means2D = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
    color, radii, inv = dgr.MultiViewRasterizer(settings)(
        means3D=params["means3D"], means2D=means2D, shs=params["shs"], opacities=params["opacities"],
        scales=params["scales"], rotations=params["rotations"])
    node = color.grad_fn  # _RasterizeViews' context: the batch's saved per-view state buffers
    Ls = list(node.num_rendered)
    bufs = node.saved_tensors[9:]
    geoms, bins, imgs = bufs[0::3], bufs[1::3], bufs[2::3]
    torch.autograd.backward([color, inv], [torch.stack([g[0] for g in grads]).to(DEV),
                                           torch.stack([g[1] for g in grads]).to(DEV)])
    torch.cuda.synchronize()

    from test_gpu_parity import _img_state
    # affected: Gaussians in some view's flipped-pixel walk; suspect_rows: in a decision suspect's
    ref_sum, affected, suspect_rows = None, None, None
    for v in range(V):
        o = oracle.OracleRaster(scene["means3D"], scene["opacities"], bg, cams[v].world_view_transform,
                                cams[v].full_proj_transform, cams[v].camera_center, cams[v].tanfovx,
                                cams[v].tanfovy, H, W, shs=scene["shs"], sh_degree=3, scales=scene["scales"],
                                rotations=scene["rotations"], antialiasing=antialiasing, nthreads=threads)
        tag = f"bench step aa={antialiasing} view {v}"
        assert Ls[v] == o.num_rendered, f"{tag}: num_rendered {Ls[v]} vs {o.num_rendered}"
        np.testing.assert_array_equal(radii[v].cpu().numpy(), o.radii, err_msg=f"{tag}: radii")
        keys, vals, ranges = dgr._C.sorted_keys(geoms[v], bins[v], imgs[v], P, Ls[v], W, H)
        np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"), err_msg=f"{tag}: keys")
        np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"), err_msg=f"{tag}: vals")
        np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"),
                                      err_msg=f"{tag}: ranges")
        del keys, vals, ranges
        fT, nc = _img_state(imgs[v], W, H)
        flips, sus = [], []
        common.check_render(tag, {"color": color[v].detach().cpu().numpy(), "invdepth": inv[v].detach().cpu().numpy(),
                                  "final_T": fT, "n_contrib": nc},
                            {"color": o.color, "invdepth": o.invdepth, "final_T": o.get("final_T"),
                             "n_contrib": o.get("n_contrib")}, flips=flips, suspects=sus)
        aff = common.flip_gaussians(flips[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
        saff = common.flip_gaussians(sus[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
        affected = aff if affected is None else affected | aff
        suspect_rows = saff if suspect_rows is None else suspect_rows | saff
        og = o.backward(grads[v][0], grads[v][1])
        del o
        _grad_check(f"{tag} dL_dmean2D", means2D.grad[v].cpu().numpy(), og["dL_dmean2D"], aff, saff)
        og = {k: og[k].astype(np.float64) for k in PARAM_KEYS.values()}
        ref_sum = og if ref_sum is None else {k: ref_sum[k] + og[k] for k in ref_sum}
    for k, ok_ in PARAM_KEYS.items():
        a = params[k].grad.cpu().numpy()
        _grad_check(f"bench step aa={antialiasing} sum of 8 views {ok_}", a, ref_sum[ok_].reshape(a.shape), affected,
                    suspect_rows)
