"""NeRF-synthetic (Blender) scene inputs, read the way the reference reads them -- test and
fixture infrastructure, not product code (the product path takes device tensors only).

* cameras: scene/dataset_readers.py:228-269 readCamerasFromTransforms (c2w from
  `transform_matrix`, OpenGL -> COLMAP axes by negating columns 1 and 2, w2c = inv(c2w),
  R = w2c[:3,:3]^T, T = w2c[:3,3]; FovY = focal2fov(fov2focal(FovX, W), H),
  utils/graphics_utils.py:73-77), assembled into the matrices of scene/cameras.py:80-89 by
  synthetic.Camera;
* points: scene/dataset_readers.py fetchPly (x, y, z; red, green, blue / 255) of `points3d.ply`
  (binary little-endian, float xyz + float normals + uchar rgb);
* initial Gaussians: scene/gaussian_model.py:149-176 create_from_pcd (SH DC = RGB2SH(rgb), the
  rest zero, scales = log(sqrt(max(distCUDA2(points), 1e-7))) on all three axes, identity
  rotations, opacity inverse_sigmoid(0.1)), activated as the getters :102-135 do.
The reference's Python is restated here, not imported.
"""
import json
import math

import numpy as np
import torch

import synthetic

C0 = 0.28209479177387814  # utils/sh_utils.py C0


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


def read_transforms(path, frames=None, width=800, height=800):
    """[(R, T, FovX, FovY, W, H, file_path)] of transforms_*.json (every frame, or the indices in
    `frames`); the image size is the dataset's (800 x 800), passed in (no image is read)."""
    with open(path) as f:
        contents = json.load(f)
    fovx = contents["camera_angle_x"]
    out = []
    for idx, frame in enumerate(contents["frames"]):
        if frames is not None and idx not in frames:
            continue
        c2w = np.array(frame["transform_matrix"])
        c2w[:3, 1:3] *= -1
        w2c = np.linalg.inv(c2w)
        R = np.transpose(w2c[:3, :3])
        T = w2c[:3, 3]
        fovy = focal2fov(fov2focal(fovx, width), height)
        out.append((R, T, fovx, fovy, width, height, frame["file_path"]))
    return out


def camera(R, T, fovx, fovy, W, H):
    return synthetic.Camera(W, H, R=R, T=T, fovx=fovx, fovy=fovy)


def read_points_ply(path):
    """(xyz float32 (n,3), rgb uint8 (n,3)) of a binary little-endian vertex PLY with float and
    uchar properties (the dataset's points3d.ply)."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    n, fields = 0, []
    for line in data[:end].decode("ascii").splitlines():
        parts = line.split()
        if parts[:2] == ["element", "vertex"]:
            n = int(parts[2])
        elif parts[:1] == ["property"]:
            fields.append((parts[2], {"float": "<f4", "uchar": "u1", "double": "<f8"}[parts[1]]))
    v = np.frombuffer(data[end:], dtype=np.dtype(fields), count=n)
    xyz = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float32)
    rgb = np.stack([v["red"], v["green"], v["blue"]], 1).astype(np.uint8)
    return xyz, rgb


def initial_gaussians(xyz, rgb, dist2, scale=None, opacity=None):
    """create_from_pcd + activations: {means3D, shs (P,16,3), scales, rotations, opacities}, float32.
    dist2 = distCUDA2(xyz) (simple-knn's mean squared 3-NN distance).  scale (P,) / opacity: the
    activated values when already known (a fixture's, computed on another host), instead of this
    host's exp(log(sqrt(dist2))) and sigmoid(inverse_sigmoid(0.1))."""
    P = xyz.shape[0]
    colors = torch.tensor(rgb.astype(np.float64) / 255.0).float()
    fused = (colors - 0.5) / C0                                   # RGB2SH
    shs = torch.zeros((P, 16, 3), dtype=torch.float32)
    shs[:, 0, :] = fused
    d2 = torch.clamp_min(torch.as_tensor(dist2, dtype=torch.float32), 0.0000001)
    scaling = torch.log(torch.sqrt(d2))[..., None].repeat(1, 3)
    rots = torch.zeros((P, 4), dtype=torch.float32)
    rots[:, 0] = 1
    opac = torch.log(torch.tensor(0.1) / (1 - torch.tensor(0.1))) * torch.ones((P, 1))  # inverse_sigmoid(0.1)
    scales = torch.exp(scaling) if scale is None else torch.as_tensor(scale, dtype=torch.float32)[:, None].repeat(1, 3)
    opacities = torch.sigmoid(opac) if opacity is None else torch.full((P, 1), float(opacity), dtype=torch.float32)
    return {"means3D": torch.as_tensor(xyz).contiguous(), "shs": shs.contiguous(),
            "scales": scales.contiguous(),
            "rotations": torch.nn.functional.normalize(rots).contiguous(),
            "opacities": opacities.contiguous()}
