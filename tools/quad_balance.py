"""render_bwd load balance over its four quadrant groups, measured on the bench scene (one view).

Runs one forward, reads the per-instance quadrant hit bits, the tile ranges and n_contrib from the
state buffers and models render_bwd's batches: per 64-entry batch each quadrant group walks the
entries whose hit bit it has, all four groups in lock step, three entries per reduction.  Prints
the group utilisation (useful group-iterations / issued group-iterations).  GPU only (diagnostic).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gaussian-splatting-npu_amd"))
import synthetic  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402


def layout(fn, *args, n=16):
    offs = (ctypes.c_size_t * n)()
    k = fn(*args, offs, n)
    return [offs[i] for i in range(k)]


def main():
    dev = torch.device("cuda:0")
    H, W, P = 1080, 1920, 1_000_000
    scene = synthetic.make_scene(P, seed=0)
    prm = {k: v.to(dev) for k, v in scene.items()}
    cam = synthetic.Camera(W, H, view=0, n_views=8)
    L, color, radii, geom, binning, img, inv = dgr._C.rasterize_gaussians(
        torch.zeros(3, device=dev), prm["means3D"], torch.empty(0, device=dev), prm["opacities"], prm["scales"],
        prm["rotations"], 1.0, torch.empty(0, device=dev), cam.world_view_transform.to(dev),
        cam.full_proj_transform.to(dev), cam.tanfovx, cam.tanfovy, H, W, prm["shs"], 3, cam.camera_center.to(dev),
        False, False, False)
    torch.cuda.synchronize()
    lib = dgr._C.lib
    for f in (lib.gsr_binning_layout, lib.gsr_image_layout):
        f.restype = ctypes.c_int
    bo = layout(lib.gsr_binning_layout, ctypes.c_int(L))
    io = layout(lib.gsr_image_layout, ctypes.c_int(W), ctypes.c_int(H))
    b = binning.cpu().numpy()
    im = img.cpu().numpy()
    BIN_HIT, IMG_RANGES, IMG_N_CONTRIB = 6, 0, 2
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    hit = b[bo[BIN_HIT]:bo[BIN_HIT] + L]
    ranges = im[io[IMG_RANGES]:io[IMG_RANGES] + 8 * T].view(np.uint32).reshape(T, 2)
    nc = im[io[IMG_N_CONTRIB]:io[IMG_N_CONTRIB] + 4 * W * H].view(np.uint32).reshape(H, W)
    ncp = np.zeros((gy * 16, gx * 16), np.uint32)
    ncp[:H, :W] = nc
    tmax = ncp.reshape(gy, 16, gx, 16).max(axis=(1, 3)).reshape(T)
    if len(sys.argv) > 1:  # the arrays, for models off the GPU box
        np.savez_compressed(sys.argv[1], hit=hit, ranges=ranges, tmax=tmax)
    useful = issued = issued_g3 = 0
    qsum = np.zeros(4)
    ms = []  # per batch: the iterations its groups run (the largest quadrant count)
    for t in range(T):
        n = int(tmax[t])
        if n == 0:
            continue
        h = hit[ranges[t, 0]:ranges[t, 0] + n]
        for p0 in range(0, n, 64):
            hb = h[p0:p0 + 64]
            cq = np.array([((hb >> q) & 1).sum() for q in range(4)])
            qsum += cq
            m = int(cq.max())
            ms.append(m)
            useful += int(cq.sum())
            issued += 4 * m
            issued_g3 += 4 * 3 * ((m + 2) // 3)
    print(f"L={L} tiles={T} entries(hit)={useful} group-iterations issued={issued} (G=3: {issued_g3})")
    print(f"utilisation {useful / issued:.3f} (G=3 rounding: {useful / issued_g3:.3f}); per-quadrant totals {qsum}")
    ms = np.array(ms)
    print(f"batches {len(ms)}; iterations per batch: mean {ms.mean():.1f}, p50 {np.percentile(ms, 50):.0f}, "
          f"p90 {np.percentile(ms, 90):.0f}, p99 {np.percentile(ms, 99):.0f}, max {ms.max()}")
    for c in (12, 15, 18, 21, 24, 27, 30, 33, 42):
        big = ms > c
        print(f"  > {c}: {big.mean():.4f} of the batches, {ms[big].sum() / ms.sum():.4f} of the iterations")


if __name__ == "__main__":
    main()
