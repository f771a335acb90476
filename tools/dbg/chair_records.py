#!/usr/bin/env python3
"""GPU diagnostic: the HIP render backward's per-(tile, Gaussian) gradient records of selected
Gaussians on one chair case, with the geometry state they came from, saved for an offline
comparison against per-tile float64 records (tools/dbg/chair_records_cmp.py).
Usage (GPU box): python tools/dbg/chair_records.py <case> <gaussian id>...  -> gpurun_out/chair/records_case<case>.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "tests/golden", "gaussian-splatting-npu_amd", ".")]
import synthetic  # noqa: E402
from test_chair import load_chair  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402


def main():
    case = int(sys.argv[1])
    ids = np.array([int(x) for x in sys.argv[2:]], np.int64)
    dev = torch.device("cuda:0")
    f, _, cases = load_chair()
    cam, deg, aa, bg, seed, scene = cases[case]
    H, W, P = cam.image_height, cam.image_width, scene["means3D"].shape[0]
    sc = {k: v.to(dev).contiguous() for k, v in scene.items()}
    bg_t = torch.tensor(bg, dtype=torch.float32, device=dev)
    e = torch.Tensor([])
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        bg_t, sc["means3D"], e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, vm, pm, cam.tanfovx,
        cam.tanfovy, H, W, sc["shs"], deg, cp, False, aa, False)
    gc, gi = (g.to(dev) for g in synthetic.make_grads(H, W, seed=seed))
    out = dgr._C.rasterize_gaussians_backward(
        bg_t, sc["means3D"], radii, e, sc["opacities"], sc["scales"], sc["rotations"], 1.0, e, vm, pm, cam.tanfovx,
        cam.tanfovy, gc, gi, sc["shs"], deg, cp, geom, L, binning, img, aa, False)
    torch.cuda.synchronize()
    gl, bl = dgr._C.geometry_layout(P), dgr._C.binning_layout(L)
    gb, bb = geom.cpu().numpy(), binning.cpu().numpy()

    def garr(i, dt, shape):
        n = int(np.prod(shape)) * np.dtype(dt).itemsize
        return gb[gl[i]:gl[i] + n].view(dt).reshape(shape).copy()

    emit = garr(11, np.uint32, (P,))
    tt = garr(6, np.uint32, (P,))
    recs, slots = [], []
    rec = dgr._C.grad_record_floats()  # the build's record size (10 floats = 40 B)
    grad = bb[bl[3]:bl[3] + 4 * rec * L].view(np.float32).reshape(L, rec)
    for g in ids:
        s = np.arange(emit[g], emit[g] + tt[g], dtype=np.int64)
        slots.append(s)
        recs.append(grad[s].copy())
    valid = bb[bl[5]:bl[5] + 4 * ((L + 31) // 32)].view(np.uint32).copy()
    os.makedirs(os.path.join(ROOT, "gpurun_out", "chair"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "chair", f"records_case{case}.npz"), ids=ids, L=L,
                        depths=garr(0, np.float32, (P,)), means2D=garr(3, np.float32, (P, 2)),
                        conic_opacity=garr(4, np.float32, (P, 4)), rgb=garr(5, np.float32, (P, 3)),
                        tiles_touched=tt, emit_start=emit, rect4=garr(12, np.uint32, (P,)),
                        rec_mask=garr(17, np.uint32, (P,)), valid=valid, slots=np.concatenate(slots),
                        records=np.concatenate(recs), dL_dmean2D=out[0].cpu().numpy(), dL_dcolors=out[1].cpu().numpy(),
                        dL_dopacity=out[2].cpu().numpy(), radii=radii.cpu().numpy())
    print("saved", len(ids), "Gaussians,", sum(len(s) for s in slots), "slots")


if __name__ == "__main__":
    main()
