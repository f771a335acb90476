#!/usr/bin/env python3
"""Generates tests/golden/chair/chair_frames.npz: 25 training and 8 test frames of the
NeRF-synthetic chair as the dataset's own PNG files (their bytes, undecoded: data the reference
holds), with their cameras, for the "PSNR vs ref" training tests (tests/test_chair_train.py,
VERDICT r04 item 2).  The tests decode and resize them exactly as the reference does:

* scene/dataset_readers.py:228-271 readCamerasFromTransforms: R, T from `transform_matrix`
  (nerf_synthetic.read_transforms restates it) and FovY = focal2fov(fov2focal(FovX, w), h).  It
  also composites the RGBA image on the background (:253-258), but keeps only its size: the
  image train.py trains on is re-opened by utils/camera_utils.py:20-66 loadCam;
* loadCam: resolution = round(800 / r) for `-r r`; scene/cameras.py:40-47 then takes
  PILtoTorch(image, resolution) (utils/general_utils.py:21-27: PIL `resize` with its default
  filter, / 255), original_image = its RGB channels and alpha_mask = its alpha channel; train.py
  multiplies the render by alpha_mask before the loss (train.py:119-121).
The fixture also holds the matrices of scene/cameras.py as computed here (another host's CPU linear
algebra may round them differently; they do not depend on the resolution for these square frames)
and scene.cameras_extent (scene/__init__.py via dataset_readers.getNerfppNorm over ALL training
cameras: 1.1 x the largest camera-centre distance from their mean), which scales the position
learning rate (gaussian_model.py:178).

Runs only in the build container (it reads /root/reference/nerf_synthetic/chair).
Usage: python tests/golden/make_chair_images.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import nerf_synthetic as ns  # noqa: E402

SCENE = "/root/reference/nerf_synthetic/chair"
TRAIN = tuple(range(0, 100, 4))   # 25 of the 100 training frames
TEST = tuple(range(0, 200, 25))   # 8 of the 200 test frames


def frames(split, idx):
    cams = ns.read_transforms(os.path.join(SCENE, f"transforms_{split}.json"), frames=set(idx))
    pngs, full = [], []
    for R, T, fovx, fovy, w, h, path in cams:
        with open(os.path.join(SCENE, path + ".png"), "rb") as f:
            pngs.append(f.read())
        full.append(ns.camera(R, T, fovx, fovy, w, h))
    return pngs, full, [c[6] for c in cams]


def nerfpp_radius(split="train"):
    """dataset_readers.getNerfppNorm: centres from inv(getWorld2View2(R, T)), radius = 1.1 x max
    distance from their mean."""
    cams = ns.read_transforms(os.path.join(SCENE, f"transforms_{split}.json"))
    centers = []
    for R, T, *_ in cams:
        W2C = np.zeros((4, 4))
        W2C[:3, :3] = R.transpose()
        W2C[:3, 3] = T
        W2C[3, 3] = 1.0
        centers.append(np.linalg.inv(W2C)[:3, 3:4])
    centers = np.hstack(centers)
    center = np.mean(centers, axis=1, keepdims=True)
    return float(np.max(np.linalg.norm(centers - center, axis=0)) * 1.1)


def main():
    out = {"extent": np.float64(nerfpp_radius())}
    for split, idx in (("train", TRAIN), ("test", TEST)):
        pngs, full, paths = frames(split, idx)
        # the PNG files' bytes, concatenated, with their offsets
        out[f"{split}_png"] = np.frombuffer(b"".join(pngs), np.uint8)
        out[f"{split}_png_offsets"] = np.cumsum([0] + [len(p) for p in pngs]).astype(np.int64)
        out[f"{split}_frames"] = np.array(idx, np.int32)
        out[f"{split}_paths"] = np.array(paths)
        out[f"{split}_viewmatrix"] = np.stack([c.world_view_transform.numpy() for c in full])
        out[f"{split}_projmatrix"] = np.stack([c.full_proj_transform.numpy() for c in full])
        out[f"{split}_campos"] = np.stack([c.camera_center.numpy() for c in full])
        out[f"{split}_tanfov"] = np.array([[c.tanfovx, c.tanfovy] for c in full], np.float32)
        print(split, len(pngs), "frames,", sum(len(p) for p in pngs) / 1e6, "MB of PNG")
    with open(os.path.join(SCENE, "transforms_train.json")) as f:
        out["camera_angle_x"] = np.float64(json.load(f)["camera_angle_x"])
    np.savez(os.path.join(HERE, "chair", "chair_frames.npz"), **out)  # PNG bytes: already compressed
    print("extent", out["extent"])


if __name__ == "__main__":
    main()
