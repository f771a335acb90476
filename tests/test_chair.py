"""The NeRF-synthetic chair fixture (tests/golden/chair/nerf_chair.npz, make_chair.py) on CPU: the C
oracle re-run from the committed inputs reproduces the committed digests (so the GPU test's oracle
run on the box is the one generated here), with a different thread count than the generator's."""
import os

import numpy as np
import pytest

import nerf_synthetic as ns

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "chair", "nerf_chair.npz")


class FixtureCamera:
    """A camera of the fixture: the matrices as computed where the fixture was made (another host's
    CPU linear algebra may round them differently), the fields of view and the image size."""

    def __init__(self, f, frame):
        import math
        import torch
        self.world_view_transform = torch.from_numpy(f["viewmatrix"][frame].copy())
        self.full_proj_transform = torch.from_numpy(f["projmatrix"][frame].copy())
        self.camera_center = torch.from_numpy(f["campos"][frame].copy())
        self.FoVx, self.FoVy = float(f["fovx"][frame]), float(f["fovy"][frame])
        self.tanfovx, self.tanfovy = float(f["tanfovx"][frame]), float(f["tanfovy"][frame])
        self.image_width, self.image_height = int(f["width"]), int(f["height"])


def load_chair():
    """(fixture dict, activated Gaussians, [cases: (camera, sh_degree, antialiasing, bg, grad_seed,
    scene)]) -- each case's scene is the create_from_pcd cloud or, for the perturbed cases, that cloud
    with the fixture's random rotations and anisotropic scales."""
    import make_chair
    f = dict(np.load(FIX))
    scene = ns.initial_gaussians(f["xyz"], f["rgb"], f["dist2"], scale=f["scale"], opacity=f["opacity"])
    pscene = make_chair.perturbed_scene(scene, f)
    cases = []
    for i, (frame, deg, aa, bg, pert) in enumerate(make_chair.CASES):
        cases.append((FixtureCamera(f, frame), deg, aa, bg, 100 + i, pscene if pert else scene))
    return f, scene, cases


def test_chair_inputs():
    import make_chair
    f, scene, cases = load_chair()
    assert f["xyz"].shape == (100_000, 3) and f["rgb"].shape == (100_000, 3)
    assert np.all(np.abs(f["xyz"]) <= 1.3)  # the dataset's initial cloud: U(-1.3, 1.3)^3
    assert np.all(f["dist2"] > 0)
    # create_from_pcd: identity rotations, opacity 0.1, isotropic scales sqrt(dist2)
    assert np.all(scene["rotations"].numpy() == np.array([1, 0, 0, 0], np.float32))
    np.testing.assert_allclose(scene["opacities"].numpy(), 0.1, rtol=1e-6)
    np.testing.assert_allclose(scene["scales"][:, 0].numpy() ** 2, np.maximum(f["dist2"], 1e-7), rtol=1e-5)
    # the stored activations are this host's create_from_pcd (up to the last bit elsewhere)
    here = ns.initial_gaussians(f["xyz"], f["rgb"], f["dist2"])
    np.testing.assert_allclose(here["scales"].numpy(), scene["scales"].numpy(), rtol=1e-6)
    np.testing.assert_allclose(here["opacities"].numpy(), scene["opacities"].numpy(), rtol=1e-6)
    for i, (cam, *_) in enumerate(cases):
        # the stored matrices are those nerf_synthetic's restatement of the reference's readers builds
        frame = make_chair.CASES[i][0]
        ref = ns.camera(f["R"][frame], f["T"][frame], float(f["fovx"][frame]), float(f["fovy"][frame]),
                        int(f["width"]), int(f["height"]))
        np.testing.assert_allclose(cam.full_proj_transform.numpy(), ref.full_proj_transform.numpy(), atol=1e-6)
        np.testing.assert_allclose(cam.world_view_transform.numpy(), ref.world_view_transform.numpy(), atol=1e-6)
        # a camera on the Blender sphere (radius ~4.03) looking at the origin: the origin projects
        # near the image centre, in front of the camera
        c = cam.camera_center.numpy()
        assert 3.9 < np.linalg.norm(c) < 4.2
        p = np.array([0, 0, 0, 1], np.float32) @ cam.full_proj_transform.numpy()
        assert p[3] > 0 and abs(p[0] / p[3]) < 0.2 and abs(p[1] / p[3]) < 0.2


def test_chair_perturbation():
    """The perturbed cases' rotations are unit quaternions and their scales anisotropic around the
    create_from_pcd scale (the stored arrays are the generator's, made in float64)."""
    import make_chair
    f, scene, cases = load_chair()
    q, s = make_chair.perturbation(f["scale"])
    np.testing.assert_allclose(f["rot_perturbed"], q, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(f["scale_perturbed"], s, rtol=1e-6)
    np.testing.assert_allclose(np.linalg.norm(f["rot_perturbed"].astype(np.float64), axis=1), 1.0, atol=1e-6)
    ratio = f["scale_perturbed"].max(1) / f["scale_perturbed"].min(1)
    assert np.median(ratio) > 1.5
    assert sum(c[5] is not scene for c in cases) == 2


@pytest.mark.parametrize("case", [0, 3])
def test_chair_oracle_reproduces_digests(case):
    import make_chair
    f, scene, cases = load_chair()
    cam, deg, aa, bg, seed, scene = cases[case]
    o, g = make_chair.run_case(scene, cam, deg, aa, bg, seed, nthreads=3)
    d = make_chair.digests(o, g)
    for k, v in d.items():
        want = f[f"case{case}_{k}"]
        if k.startswith("sha") or k == "num_rendered":
            assert str(v) == str(want), k
        else:  # the oracle's backward sums per Gaussian in thread-count-dependent order
            scale = float(f[f"case{case}_abs" + k[len("abs"):]] if k.startswith("abs")
                          else f[f"case{case}_abs{k}"])
            assert abs(float(v) - float(want)) <= 1e-6 * scale, (k, v, want)
