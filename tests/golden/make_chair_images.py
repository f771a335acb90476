#!/usr/bin/env python3
"""Generates tests/golden/chair/chair_images.npz and chair_images_r2.npz: the NeRF-synthetic chair's
training and test images at train.py's `-r 4` (200 x 200) and `-r 2` (400 x 400) resolutions with
their cameras, for the "PSNR vs ref" training tests (tests/test_chair_train.py).

What the reference does with a frame (restated, not imported):
* scene/dataset_readers.py:228-271 readCamerasFromTransforms: R, T from `transform_matrix`
  (nerf_synthetic.read_transforms restates it) and FovY = focal2fov(fov2focal(FovX, w), h).  It
  also composites the RGBA image on the background (:253-258), but keeps only its size: the
  image train.py trains on is re-opened by utils/camera_utils.py:20-66 loadCam;
* loadCam: resolution = round(800 / r) = 200 for `-r 4`; scene/cameras.py:40-47 then takes
  PILtoTorch(image, resolution) (utils/general_utils.py:21-27: PIL `resize` with its default
  filter, / 255), original_image = its RGB channels and alpha_mask = its alpha channel; train.py
  multiplies the render by alpha_mask before the loss (train.py:119-121).
So the fixture stores each frame as the uint8 RGBA array of `Image.open(png).resize((200, 200))`
(this container's Pillow), the matrices of scene/cameras.py as computed here (another host's CPU
linear algebra may round them differently), and scene.cameras_extent (scene/__init__.py via
dataset_readers.getNerfppNorm over ALL training cameras: 1.1 x the largest camera-centre distance
from their mean), which scales the position learning rate (gaussian_model.py:178).

Runs only in the build container (it reads /root/reference/nerf_synthetic/chair).
Usage: python tests/golden/make_chair_images.py
"""
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import nerf_synthetic as ns  # noqa: E402

SCENE = "/root/reference/nerf_synthetic/chair"
RES = 200                         # train.py -r 4 on the 800 x 800 frames
TRAIN = tuple(range(0, 100, 4))   # 25 of the 100 training frames
TEST = tuple(range(0, 200, 25))   # 8 of the 200 test frames


def frames(split, idx, res=RES):
    cams = ns.read_transforms(os.path.join(SCENE, f"transforms_{split}.json"), frames=set(idx), width=res,
                              height=res)
    imgs, full = [], []
    for R, T, fovx, fovy, w, h, path in cams:
        im = Image.open(os.path.join(SCENE, path + ".png"))
        imgs.append(np.array(im.resize((res, res))))  # PILtoTorch's resize (default filter)
        full.append(ns.camera(R, T, fovx, fovy, w, h))
    return np.stack(imgs), full, [c[6] for c in cams]


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


def main(res=RES, name="chair_images.npz"):
    out = {"extent": np.float64(nerfpp_radius()), "res": np.int32(res)}
    for split, idx in (("train", TRAIN), ("test", TEST)):
        imgs, full, paths = frames(split, idx, res)
        out[f"{split}_rgba"] = imgs
        out[f"{split}_frames"] = np.array(idx, np.int32)
        out[f"{split}_paths"] = np.array(paths)
        out[f"{split}_viewmatrix"] = np.stack([c.world_view_transform.numpy() for c in full])
        out[f"{split}_projmatrix"] = np.stack([c.full_proj_transform.numpy() for c in full])
        out[f"{split}_campos"] = np.stack([c.camera_center.numpy() for c in full])
        out[f"{split}_tanfov"] = np.array([[c.tanfovx, c.tanfovy] for c in full], np.float32)
        print(split, imgs.shape, "alpha>0:", float((imgs[..., 3] > 0).mean()))
    with open(os.path.join(SCENE, "transforms_train.json")) as f:
        out["camera_angle_x"] = np.float64(json.load(f)["camera_angle_x"])
    np.savez_compressed(os.path.join(HERE, "chair", name), **out)
    print("extent", out["extent"])


if __name__ == "__main__":
    main()
    main(400, "chair_images_r2.npz")  # train.py -r 2: the longer HIP-only run (test_chair_train_py_hip_long)
