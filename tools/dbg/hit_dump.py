"""Debug: dump the forward's per-entry quadrant contribution bits (BIN_HIT), the tile ranges and
each tile's largest n_contrib (config 2, view 0) to gpurun_out/hit_dump.npz, so that render_bwd's
group-slot occupancy can be simulated on the CPU (tools/dbg/hit_sim.py)."""
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (root, os.path.join(root, "gaussian-splatting-npu_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import synthetic  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

dev = torch.device("cuda", 0)
P, H, W = 1_000_000, 1080, 1920
sc = {k: v.to(dev) for k, v in synthetic.make_scene(P, seed=0).items()}
cam = synthetic.Camera(W, H, view=0)
L, color, radii, geom, binning, img, inv = _C.rasterize_gaussians(
    torch.zeros(3, device=dev), sc["means3D"], torch.Tensor([]), sc["opacities"], sc["scales"], sc["rotations"], 1.0,
    torch.Tensor([]), cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.tanfovx, cam.tanfovy,
    H, W, sc["shs"], 3, cam.camera_center.to(dev), False, False, False)
torch.cuda.synchronize()
bl = _C.binning_layout(L)
il = _C.image_layout(W, H)
T = 120 * 68
hit = binning[bl[-2]:bl[-2] + L].cpu().numpy()  # BIN_HIT
ranges = img[il[0]:il[0] + 8 * T].view(torch.int32).cpu().numpy().reshape(-1, 2)
work = img[il[4]:il[4] + 4 * T].view(torch.int32).cpu().numpy()  # IMG_TILE_WORK
os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(root, "gpurun_out", "hit_dump.npz"), hit=hit, ranges=ranges, work=work, L=L)
print("dumped", L, "entries")
