"""BASELINE config 3's scale on the GPU: a ~6M-Gaussian cloud on one 1297x840 view (needs an MI355X).

Config 3 is the Mip-NeRF360 'garden' train loop (~6M Gaussians, SH degree 3, images_4: 1297x840).
The dataset is not available offline, so this is a SURVEY §8d synthetic cloud of that size
(synthetic.make_scene(6,000,000), seed 0) seen by ring view 0 at garden's images_4 resolution;
L is about 26M instances, 4.5x config 2's.  What it exercises beyond config 2: P and L past
every size the other tests reach (the 32-bit id packing of the second tile-sort pass,
radix.hip tile_sort_fused_batch; the binning buffer's first-call sizing, _C.py; device memory),
against the C oracle on the GPU box's host (16 threads, about 20 s):

* bit-exact: num_rendered, radii, the sorted tile|depth keys, their Gaussian ids and the
  per-tile ranges (rasterizer_impl.cu:250-320);
* render state through common.check_render (forward.cu:277-400);
* all eight outputs of rasterize_gaussians_backward (rasterize_points.cu:222) through
  common.check_grad_attributed, check_rel_truth (float64 yardstick) and check_rel, exactly as
  the config-2 test checks them (backward.cu:452-638, 147-449).
The peak device memory of the forward + backward is logged with the parity statistics.
"""
import os

import numpy as np
import pytest
import torch

import common

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
P, H, W = 6_000_000, 840, 1297


@pytest.fixture(scope="module")
def case():
    return common.make_case(P=P, H=H, W=W)


@pytest.fixture(scope="module")
def oracle_run(case):
    threads = min(16, os.cpu_count() or 1)
    o, og = common.run_oracle(case, antialiasing=False, nthreads=threads)
    return o, og


@pytest.fixture(scope="module")
def hip_forward(case):
    import diff_gaussian_rasterization as dgr
    cam = case["cam"]
    sc = {k: v.to(DEV).contiguous() for k, v in case["scene"].items()}
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(DEV)  # (after the first device call: it needs the context)
    bg = case["bg"].to(DEV)
    vm, pm, cp = cam.world_view_transform.to(DEV), cam.full_proj_transform.to(DEV), cam.camera_center.to(DEV)
    e = torch.Tensor([])
    out = dgr._C.rasterize_gaussians(bg, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, vm,
                                     pm, cam.tanfovx, cam.tanfovy, H, W, sc["shs"], 3, cp, False, False, False)
    torch.cuda.synchronize()
    return dict(sc=sc, bg=bg, vm=vm, pm=pm, cp=cp, out=out)


def test_config3_forward_bit_exact(case, oracle_run, hip_forward):
    import diff_gaussian_rasterization as dgr
    from test_gpu_parity import _img_state
    o, _ = oracle_run
    L, color, radii, geom, binning, img, inv = hip_forward["out"]
    assert L == o.num_rendered and L > 20_000_000, L
    np.testing.assert_array_equal(radii.cpu().numpy(), o.radii)
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, W, H)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    del keys
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))
    del vals, ranges
    fT, nc = _img_state(img, W, H)
    flips, sus = [], []
    common.check_render("config3-scale 6M", {"color": color.cpu().numpy(), "invdepth": inv.cpu().numpy(),
                                             "final_T": fT, "n_contrib": nc},
                        {"color": o.color, "invdepth": o.invdepth, "final_T": o.get("final_T"),
                         "n_contrib": o.get("n_contrib")}, flips=flips, suspects=sus)
    hip_forward["flips"], hip_forward["suspects"], hip_forward["nc"] = flips[0], sus[0], nc


def test_config3_backward(case, oracle_run, hip_forward):
    import diff_gaussian_rasterization as dgr
    o, og = oracle_run
    if "flips" not in hip_forward:
        pytest.skip("the forward test did not run")
    f = hip_forward
    cam, sc = case["cam"], f["sc"]
    L, color, radii, geom, binning, img, inv = f["out"]
    nc = f["nc"]
    affected = common.flip_gaussians(f["flips"], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
    suspect_rows = common.flip_gaussians(f["suspects"], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W,
                                         H, P)
    e = torch.Tensor([])
    out = dgr._C.rasterize_gaussians_backward(
        f["bg"], sc["means3D"], radii, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, f["vm"], f["pm"],
        cam.tanfovx, cam.tanfovy, case["grad_color"].to(DEV), case["grad_invdepth"].to(DEV), sc["shs"], 3, f["cp"],
        geom, L, binning, img, False, False)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(DEV)
    common.PARITY_LOG.append({"name": "config3-scale 6M memory", "P": P, "L": int(L), "width": W, "height": H,
                              "peak_device_bytes_fwd_bwd": int(peak)})
    names = ["dL_dmean2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    hip = [t.cpu().numpy() for t in out]
    del out
    g64 = o.backward(case["grad_color"], case["grad_invdepth"], f64=True)
    for n, t in zip(names, hip):
        ref, truth = og[n].reshape(t.shape), g64[n].reshape(t.shape)
        nm = f"config3-scale 6M {n}"
        common.check_grad_attributed(nm, t, ref, suspect_rows)  # the walks of every decision suspect
        so = common.check_rel_truth(nm, t, ref, truth, suspect_rows)[1]
        common.check_rel(nm, t, ref, suspect_rows, so)
