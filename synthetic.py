"""Synthetic scenes and cameras for the parity tests and bench.py.

Cameras follow the reference conventions exactly:
  * world_view_transform = getWorld2View2(R, T).T            (scene/cameras.py:86)
  * projection_matrix    = getProjectionMatrix(0.01, 100, fovX, fovY).T   (scene/cameras.py:87)
  * full_proj_transform  = world_view @ projection            (scene/cameras.py:88)
  * camera_center        = world_view.inverse()[3, :3]        (scene/cameras.py:89)
with getWorld2View2 / getProjectionMatrix restated from utils/graphics_utils.py:38-71.
tests/golden/make_golden.py checks these restatements against the reference's own
functions (imported from /root/reference in the build container).
"""
import math

import numpy as np
import torch


def get_world2view2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    """utils/graphics_utils.py:38-49"""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = C2W[:3, 3]
    cam_center = (cam_center + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def get_projection_matrix(znear, zfar, fovX, fovY):
    """utils/graphics_utils.py:51-71"""
    tanHalfFovY = math.tan((fovY / 2))
    tanHalfFovX = math.tan((fovX / 2))
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def ring_camera_RT(view, n_views=8, radius=4.0, height=-0.5):
    """COLMAP-convention (x right, y down, z forward) camera on a ring looking at the origin.
    Returns (R, T) as stored by the reference Camera: R is camera-to-world, T world-to-camera."""
    theta = 2.0 * math.pi * view / n_views
    C = np.array([radius * math.cos(theta), height, radius * math.sin(theta)])
    z = -C / np.linalg.norm(C)
    down = np.array([0.0, 1.0, 0.0])
    x = np.cross(down, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z], axis=1)  # columns = camera axes in world
    T = -R.T @ C
    return R, T


class Camera:
    """Minimal stand-in for scene/cameras.py::Camera (matrix part only)."""

    def __init__(self, width, height, view=0, n_views=8, fovy_deg=50.0, znear=0.01, zfar=100.0, R=None, T=None,
                 fovx=None, fovy=None):
        """A ring view (`view` of `n_views`), or -- with R, T, fovx, fovy -- the camera of a dataset
        (scene/cameras.py:19-89: R camera-to-world rotation as the readers store it, T the
        world-to-camera translation, trans 0, scale 1)."""
        self.image_width = int(width)
        self.image_height = int(height)
        if R is None:
            self.FoVy = math.radians(fovy_deg)
            self.FoVx = 2.0 * math.atan(math.tan(self.FoVy * 0.5) * width / height)
            R, T = ring_camera_RT(view, n_views)
        else:
            self.FoVx, self.FoVy = float(fovx), float(fovy)
        self.znear, self.zfar = znear, zfar
        self.R, self.T = R, T
        self.world_view_transform = torch.tensor(get_world2view2(R, T)).transpose(0, 1)
        self.projection_matrix = get_projection_matrix(znear, zfar, self.FoVx, self.FoVy).transpose(0, 1)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0))).squeeze(0)
        self.camera_center = self.world_view_transform.inverse()[3, :3]

    @property
    def tanfovx(self):
        return math.tan(self.FoVx * 0.5)

    @property
    def tanfovy(self):
        return math.tan(self.FoVy * 0.5)


def make_scene(P, seed=0, sh_degree=3):
    """Seeded synthetic Gaussian cloud, drawn in the SURVEY §8d order on a CPU generator."""
    g = torch.Generator().manual_seed(seed)
    means = torch.rand(P, 3, generator=g) * 3.0 - 1.5
    lo, hi = math.log(0.003), math.log(0.02)
    scales = torch.exp(torch.rand(P, 3, generator=g) * (hi - lo) + lo)
    rots = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=1)
    opac = torch.sigmoid(torch.randn(P, 1, generator=g))
    M = (sh_degree + 1) ** 2
    dc = torch.rand(P, 1, 3, generator=g) * 3.0 - 1.5
    rest = torch.randn(P, M - 1, 3, generator=g) * 0.05
    shs = torch.cat([dc, rest], dim=1).contiguous()
    return {"means3D": means.contiguous(), "scales": scales.contiguous(), "rotations": rots.contiguous(),
            "opacities": opac.contiguous(), "shs": shs}


def make_grads(H, W, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(3, H, W, generator=g), torch.randn(1, H, W, generator=g) * 0.01
