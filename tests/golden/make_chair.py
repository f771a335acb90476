#!/usr/bin/env python3
"""Generates tests/golden/chair/nerf_chair.npz: a real-geometry fixture from reference-held data
 -- the NeRF-synthetic `chair` scene's initial point cloud and three of its
training cameras at the dataset's 800 x 800 (GS-IRON's workload), read as the reference reads them
(nerf_synthetic.py restates scene/dataset_readers.py:228-269, fetchPly and create_from_pcd; the
reference's Python is not imported).

Runs only in the build container (it reads /root/reference/nerf_synthetic/chair, which does not
exist on the GPU box).  The fixture holds the INPUTS -- points (x, y, z as float32, colours as
uint8), distCUDA2 of the points by the brute-force oracle (oracle/knn_oracle.c), the cameras' R, T
and fields of view -- and, per case, digests of the C oracle's outputs: num_rendered, SHA-256 of the
sorted keys / values / tile ranges / radii / colour / n_contrib, and float64 sums of every gradient.
The full arrays (tens of MB at 800 x 800) are recomputed by the oracle wherever a test needs them;
the digests pin that recomputation to this one (tests/test_chair.py on CPU, tests/test_chair_gpu.py
on the GPU box against the HIP path).

Usage: python tests/golden/make_chair.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import nerf_synthetic as ns  # noqa: E402
import oracle  # noqa: E402
import synthetic  # noqa: E402

SCENE = "/root/reference/nerf_synthetic/chair"
FRAMES = (0, 1, 2)
# (frame, sh_degree, antialiasing, background, perturbed): iteration 1 of training renders at SH
# degree 0 (active_sh_degree starts at 0, train.py:95-96); one view at degree 3 with AA, one on white.
# create_from_pcd's identity rotations and isotropic scales make dL/drotations identically zero, so
# cases 3 and 4 render the cloud with seeded random rotations and anisotropic scales (the fixture's
# `rot_perturbed` / `scale_perturbed`): the cov3D -> (scale, rotation) chain of
# backward.cu:330-393 on real geometry
CASES = ((0, 0, False, (0.0, 0.0, 0.0), False), (1, 3, True, (0.0, 0.0, 0.0), False),
         (2, 0, False, (1.0, 1.0, 1.0), False), (0, 3, False, (0.0, 0.0, 0.0), True),
         (2, 0, True, (1.0, 1.0, 1.0), True))
PERTURB_SEED = 7


def perturbation(scale, seed=PERTURB_SEED):
    """Seeded unit quaternions and per-axis scale factors exp(U(-0.7, 0.7)) around the isotropic
    create_from_pcd scale (float64 math, stored as float32 in the fixture)."""
    rng = np.random.default_rng(seed)
    P = scale.shape[0]
    q = rng.standard_normal((P, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    s = np.asarray(scale, np.float64)[:, None] * np.exp(rng.uniform(-0.7, 0.7, (P, 3)))
    return q.astype(np.float32), s.astype(np.float32)


def perturbed_scene(scene, f):
    """The scene with the fixture's perturbed rotations and scales."""
    out = dict(scene)
    out["rotations"] = torch.from_numpy(np.ascontiguousarray(f["rot_perturbed"]))
    out["scales"] = torch.from_numpy(np.ascontiguousarray(f["scale_perturbed"]))
    return out


GRAD_NAMES = ("dL_dmean2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_case(scene, cam, sh_degree, antialiasing, bg, grad_seed, nthreads=8):
    """The oracle on one case: (OracleRaster, gradients)."""
    gc, gi = synthetic.make_grads(cam.image_height, cam.image_width, seed=grad_seed)
    o = oracle.OracleRaster(scene["means3D"], scene["opacities"], torch.tensor(bg, dtype=torch.float32),
                            cam.world_view_transform, cam.full_proj_transform, cam.camera_center, cam.tanfovx,
                            cam.tanfovy, cam.image_height, cam.image_width, shs=scene["shs"], sh_degree=sh_degree,
                            scales=scene["scales"], rotations=scene["rotations"], antialiasing=antialiasing,
                            nthreads=nthreads)
    return o, o.backward(gc, gi)


def digests(o, g):
    d = {"num_rendered": np.int64(o.num_rendered), "sha_keys": sha(o.get("keys")), "sha_vals": sha(o.get("vals")),
         "sha_ranges": sha(o.get("ranges")), "sha_radii": sha(o.radii), "sha_color": sha(o.color),
         "sha_n_contrib": sha(o.get("n_contrib"))}
    for n in GRAD_NAMES:
        d["sum_" + n] = np.float64(np.asarray(g[n], np.float64).sum())
        d["abssum_" + n] = np.float64(np.abs(np.asarray(g[n], np.float64)).sum())
    return d


def main():
    xyz, rgb = ns.read_points_ply(os.path.join(SCENE, "points3d.ply"))
    dist2 = oracle.knn_dist2(xyz, nthreads=8)
    cams = ns.read_transforms(os.path.join(SCENE, "transforms_train.json"), frames=set(FRAMES))
    scene = ns.initial_gaussians(xyz, rgb, dist2)
    # the cameras' matrices as computed here are part of the fixture: numpy's / torch's CPU linear
    # algebra (inverse, bmm) may round differently on another host's CPU, and one ulp in a matrix
    # can move a radius across a ceil (tests rebuild the cameras from these, not from R, T)
    full = [ns.camera(c[0], c[1], c[2], c[3], c[4], c[5]) for c in cams]
    out = {"xyz": xyz, "rgb": rgb, "dist2": dist2,
           "R": np.stack([c[0] for c in cams]), "T": np.stack([c[1] for c in cams]),
           "fovx": np.array([c[2] for c in cams]), "fovy": np.array([c[3] for c in cams]),
           "width": np.int32(cams[0][4]), "height": np.int32(cams[0][5]),
           "file_path": np.array([c[6] for c in cams]),
           "viewmatrix": np.stack([c.world_view_transform.numpy() for c in full]),
           "projmatrix": np.stack([c.full_proj_transform.numpy() for c in full]),
           "campos": np.stack([c.camera_center.numpy() for c in full]),
           # likewise the host math of the parameters (torch's vectorised exp / log / sigmoid and
           # libm's tan may round differently on another CPU): the activated scale (isotropic) and
           # opacity, and the tangents of the half fields of view, as computed here
           "scale": scene["scales"][:, 0].numpy().copy(), "opacity": scene["opacities"][0, 0].numpy().copy(),
           "tanfovx": np.array([c.tanfovx for c in full], np.float32),
           "tanfovy": np.array([c.tanfovy for c in full], np.float32)}
    out["rot_perturbed"], out["scale_perturbed"] = perturbation(out["scale"])
    pscene = perturbed_scene(scene, out)
    for i, (frame, deg, aa, bg, pert) in enumerate(CASES):
        cam = full[frame]
        o, g = run_case(pscene if pert else scene, cam, deg, aa, bg, grad_seed=100 + i)
        for k, v in digests(o, g).items():
            out[f"case{i}_{k}"] = v
        print(f"case {i}: frame {frame} deg {deg} aa {aa} bg {bg} perturbed {pert}: L={o.num_rendered} "
              f"visible={(o.radii > 0).sum()} |dL/drot|={np.abs(g['dL_drotations']).sum():.4g}")
    np.savez_compressed(os.path.join(HERE, "chair", "nerf_chair.npz"), **out)


if __name__ == "__main__":
    main()
