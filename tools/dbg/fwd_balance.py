"""render_fwd's four quadrant waves against each other (diagnostic, GPU only).

Loads a GSR_FWD_STATS=1 build (tools/build_variant.sh, ab/fwdstats.so), renders the bench view
(config 2, view 0) and reads, per (tile, 256-entry batch, wave), the entries the wave walked.
The waves of a tile meet at a barrier per batch, so a batch lasts as long as its busiest wave:
prints the waves' utilisation under that lock step (sum / (4 x max) per batch) and what it
would be if each wave walked its whole list alone (sum / (4 x the busiest wave's total)).
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-npu_amd"))
import synthetic  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402


def main():
    lib = dgr._C._load(os.path.join(ROOT, "ab", "fwdstats.so"))
    dgr._C.lib = lib
    dev = torch.device("cuda:0")
    H, W, P = 1080, 1920, 1_000_000
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    stats = torch.zeros(T * 32 * 4, dtype=torch.int32, device=dev)
    lib.gsr_debug_fwd_stats.restype = ctypes.c_int
    assert lib.gsr_debug_fwd_stats(ctypes.c_void_p(stats.data_ptr())) == 0
    scene = synthetic.make_scene(P, seed=0)
    prm = {k: v.to(dev) for k, v in scene.items()}
    cam = synthetic.Camera(W, H, view=0, n_views=8)
    out = dgr._C.rasterize_gaussians(
        torch.zeros(3, device=dev), prm["means3D"], torch.empty(0, device=dev), prm["opacities"], prm["scales"],
        prm["rotations"], 1.0, torch.empty(0, device=dev), cam.world_view_transform.to(dev),
        cam.full_proj_transform.to(dev), cam.tanfovx, cam.tanfovy, H, W, prm["shs"], 3, cam.camera_center.to(dev),
        False, False, False)
    torch.cuda.synchronize()
    s = stats.cpu().numpy().reshape(T, 32, 4).astype(np.int64)
    done = s > 0
    w = np.where(done, s - 1, 0)
    bmax = w.max(axis=2)
    lock = w.sum() / max(1, 4 * bmax.sum())
    tot = w.sum(axis=1)  # per tile and wave
    alone = w.sum() / max(1, 4 * tot.max(axis=1).sum())
    nb = done.any(axis=2).sum(axis=1)
    print(f"L={out[0]}  tiles={T}  batches/tile mean {nb.mean():.2f} max {nb.max()}")
    print(f"entries walked per wave-batch: mean {w[done].mean():.1f}")
    print(f"utilisation, waves in lock step per batch: {lock:.3f}")
    print(f"utilisation, each wave alone over its tile: {alone:.3f}")
    print(f"walked (wave-entries) total {w.sum()}, lock-step slots {4 * bmax.sum()}, alone slots {4 * tot.max(axis=1).sum()}")
    # slot time a wave holds after its last batch with work (what exiting at a batch boundary frees)
    act = w > 0
    last = np.where(act.any(axis=1), 31 - np.argmax(act[:, ::-1, :], axis=1), -1)  # (T, 4)
    bidx = np.arange(32)[None, :, None]
    after = (bidx > last[:, None, :]) & done.any(axis=2)[:, :, None]
    freed = (after * bmax[:, :, None]).sum()
    idle = 4 * bmax.sum() - w.sum()
    print(f"idle slot time {idle} ({idle / (4 * bmax.sum()):.3f}); after a wave's last active batch {freed} "
          f"({freed / (4 * bmax.sum()):.3f})")
    # tiles' walk relative to the tile with most
    ws = tot.max(axis=1)
    print("busiest-wave walk per tile: p50 %d p90 %d p99 %d max %d" % tuple(np.percentile(ws, [50, 90, 99, 100])))


if __name__ == "__main__":
    main()
