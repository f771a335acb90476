"""The HIP rasterizer on real geometry: the NeRF-synthetic chair fixture (tests/golden/chair/nerf_chair.npz,
VERDICT r03 item 9) -- the dataset's initial 100k-point cloud initialised as create_from_pcd does
and three of its training cameras at 800 x 800 -- against the C oracle (needs an MI355X: -m gpu).

Per case: the oracle re-run on the box reproduces the fixture's integer digests (so it is the run
made in the build container); num_rendered, radii, the sorted tile|depth keys, their Gaussian ids and the
tile ranges bit-exact; colour / invdepth / final_T / n_contrib through common.check_render; all
eight backward outputs within 1e-4 of max|ref| outside the walks of flipped pixels, every outlier
attributed (common.check_grad_attributed); per element no further from the float64 gradient (the
oracle's render backward in float64 on the same decisions) than 1.5x the reference's own float32
order is, and within REL_P999 of the oracle, outside the walks of decision-suspect pixels
(common.check_rel_truth, common.check_rel; common.DECISION_ATOL).  And the HIP distCUDA2 of the points equals the fixture's brute-force
dist2 bit for bit (the scales create_from_pcd derives from it).
"""
import os

import numpy as np
import pytest
import torch

import common
import make_chair
from test_chair import load_chair

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


@pytest.fixture(scope="module")
def chair():
    return load_chair()


def test_chair_distcuda2_bit_exact(chair):
    from simple_knn._C import distCUDA2
    f, _, _ = chair
    d = distCUDA2(torch.from_numpy(f["xyz"]).to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(d, f["dist2"])


@pytest.mark.parametrize("case", [0, 1, 2, 3, 4])
def test_chair_case(chair, case):
    import diff_gaussian_rasterization as dgr
    from test_gpu_parity import _img_state
    f, base, cases = chair
    cam, deg, aa, bg, seed, scene = cases[case]
    H, W, P = cam.image_height, cam.image_width, scene["means3D"].shape[0]
    o, og = make_chair.run_case(scene, cam, deg, aa, bg, seed, nthreads=min(16, os.cpu_count() or 1))
    d = make_chair.digests(o, og)
    # the oracle run here is the fixture's: its integer results bit for bit (the colour and n_contrib
    # follow this host's libm expf, whose ifunc variant differs between CPUs: those are compared
    # with the HIP path below, through check_render)
    if str(d["sha_radii"]) != str(f[f"case{case}_sha_radii"]):  # diagnostics for a host difference
        os.makedirs(os.path.join(common.ROOT_OUT, "chair"), exist_ok=True)
        np.save(os.path.join(common.ROOT_OUT, "chair", f"oracle_radii_case{case}.npy"), o.radii)
    for k in ("num_rendered", "sha_keys", "sha_vals", "sha_ranges", "sha_radii"):
        assert str(d[k]) == str(f[f"case{case}_{k}"]), k
    sc = {k: v.to(DEV).contiguous() for k, v in scene.items()}
    bg_t = torch.tensor(bg, dtype=torch.float32, device=DEV)
    e = torch.Tensor([])
    vm, pm, cp = cam.world_view_transform.to(DEV), cam.full_proj_transform.to(DEV), cam.camera_center.to(DEV)
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        bg_t, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, vm, pm, cam.tanfovx,
        cam.tanfovy, H, W, sc["shs"], deg, cp, False, aa, False)
    torch.cuda.synchronize()
    tag = f"chair case {case} (deg {deg}, aa {aa})"
    assert L == o.num_rendered, f"{tag}: num_rendered {L} vs {o.num_rendered}"
    np.testing.assert_array_equal(radii.cpu().numpy(), o.radii)
    # the preprocess outputs the blend reads, bit for bit (visible Gaussians)
    vis = o.radii > 0
    lay, gb = dgr._C.geometry_layout(P), geom.cpu().numpy()
    for i, name, w in ((0, "depths", 1), (3, "means2D", 2), (4, "conic_opacity", 4), (5, "rgb", 3)):
        hip_a = gb[lay[i]:lay[i] + 4 * w * P].view(np.uint32).reshape(P, w) if w > 1 else gb[lay[i]:lay[i] + 4 * P].view(np.uint32)
        np.testing.assert_array_equal(hip_a[vis], o.get(name).view(np.uint32).reshape(hip_a.shape)[vis], err_msg=f"{tag} {name}")
    keys, vals, ranges = dgr._C.sorted_keys(geom, binning, img, P, L, W, H)
    np.testing.assert_array_equal(keys.cpu().numpy().view(np.uint64), o.get("keys"))
    np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32), o.get("vals"))
    np.testing.assert_array_equal(ranges.cpu().numpy().view(np.uint32), o.get("ranges"))
    del keys, vals
    fT, nc = _img_state(img, W, H)
    flips, sus = [], []
    common.check_render(tag, {"color": color.cpu().numpy(), "invdepth": inv.cpu().numpy(), "final_T": fT,
                              "n_contrib": nc},
                        {"color": o.color, "invdepth": o.invdepth, "final_T": o.get("final_T"),
                         "n_contrib": o.get("n_contrib")}, flips=flips, suspects=sus)
    affected = common.flip_gaussians(flips[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
    suspect_rows = common.flip_gaussians(sus[0], nc, o.get("n_contrib"), o.get("vals"), o.get("ranges"), W, H, P)
    gc, gi = (g.to(DEV) for g in __import__("synthetic").make_grads(H, W, seed=seed))
    out = dgr._C.rasterize_gaussians_backward(
        bg_t, sc["means3D"], radii, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, vm, pm, cam.tanfovx,
        cam.tanfovy, gc, gi, sc["shs"], deg, cp, geom, L, binning, img, aa, False)
    torch.cuda.synchronize()
    g64 = o.backward(gc.cpu(), gi.cpu(), f64=True)  # the accuracy yardstick (check_rel_truth)
    perturbed = scene is not base  # cases 3 / 4: rotations and anisotropic scales
    for n, t in zip(make_chair.GRAD_NAMES, out):
        hip, ref = t.cpu().numpy(), og[n].reshape(t.shape)
        if perturbed and n in ("dL_drotations", "dL_dscales"):  # the cov3D -> (scale, rotation) chain is live
            assert np.count_nonzero(ref) > 0.01 * ref.size and np.count_nonzero(hip) > 0.01 * hip.size, n
        # outliers may sit in the walk of any decision suspect (a decision taken the other way that moved
        # the colour by less than IMG_ATOL: common.DECISION_ATOL), not only of a flipped pixel
        common.check_grad_attributed(f"{tag} {n}", hip, ref, suspect_rows)
        try:
            _, so = common.check_rel_truth(f"{tag} {n}", hip, ref, g64[n].reshape(t.shape), suspect_rows)
        except AssertionError:  # what the diagnosis needs (tools/dbg), then the failure
            os.makedirs(os.path.join(common.ROOT_OUT, "chair"), exist_ok=True)
            np.savez_compressed(os.path.join(common.ROOT_OUT, "chair", f"truth_case{case}_{n}.npz"), hip=hip,
                                oracle=ref, f64=g64[n].reshape(t.shape), affected=suspect_rows,
                                color_hip=color.cpu().numpy(), color_oracle=o.color, nc_hip=nc,
                                nc_oracle=o.get("n_contrib"))
            raise
        # case 4 (perturbed anisotropic splats over many tiles, densely packed behind few pixels): its 15
        # decision-suspect pixels' walks hold 11.4 % of the Gaussians (round 5); every other case <= 10 %
        common.check_rel(f"{tag} {n}", hip, ref, suspect_rows, so,
                         max_left_out_frac=0.2 if case == 4 else common.REL_LEFT_OUT_FRAC)
