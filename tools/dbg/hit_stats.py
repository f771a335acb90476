"""Debug: distribution of the forward's per-entry contribution bits (config 2, view 0)."""
import os, sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (root, os.path.join(root, "gaussian-splatting-npu_amd")):
    sys.path.insert(0, p)
import numpy as np
import torch
import synthetic
from diff_gaussian_rasterization import _C

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
hit = binning[bl[-2]:bl[-2] + L].cpu().numpy()  # BIN_HIT: the last array
ranges = img[il[0]:il[0] + 8 * T].view(torch.int32).cpu().numpy().reshape(-1, 2)
work = img[il[4]:il[4] + 4 * T].view(torch.int32).cpu().numpy()  # IMG_TILE_WORK
sel = np.concatenate([hit[a:a + w] for (a, b), w in zip(ranges, work)])
print("L", L, "entries below tmax", sel.size, "fraction of L", sel.size / L)
nz = sel[sel != 0]
print("entries with any contribution", nz.size, nz.size / sel.size)
lo, hi = nz & 3, (nz >> 2) & 3
halves = (lo != 0).astype(int) + (hi != 0).astype(int)
print("halves per entry: 1:", (halves == 1).mean(), "2:", (halves == 2).mean())
full = lambda h: (h == 3)
print("half evaluations", halves.sum(), "with both quadrants used", full(lo).sum() + full(hi).sum(),
      "fraction of pair slots wasted", 1 - (np.bitwise_count(nz.astype(np.uint8)).sum() / (2 * halves.sum())))
print("quadrant count histogram", np.bincount(np.bitwise_count(nz.astype(np.uint8)), minlength=5))
