#!/usr/bin/env python3
"""Offline half of tools/dbg/chair_records.py: per-(tile, Gaussian) records of the HIP render
backward against float64 records computed on the oracle's decisions, for the dumped Gaussians.
Usage: python tools/dbg/chair_records_cmp.py <case>   (reads gpurun_out/chair/records_case<case>.npz)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "tests/golden", "oracle", ".")]
import make_chair  # noqa: E402
import synthetic  # noqa: E402
from test_chair import load_chair  # noqa: E402

NAMES = ["Sx", "Sy", "Sxx", "Sxy", "Syy", "S", "cr", "cg", "cb", "ci"]


def tile_records_f64(o, t, W, H, dp3, dinv, bgv):
    """float64 records of every entry of tile t's list below its largest n_contrib."""
    gx = (W + 15) // 16
    tx, ty = t % gx, t // gx
    ys, xs = np.meshgrid(np.arange(16) + 16 * ty, np.arange(16) + 16 * tx, indexing="ij")
    m = (xs < W) & (ys < H)
    xs, ys = xs[m], ys[m]
    pid = ys * W + xs
    ranges, vals, nc = o.get("ranges"), o.get("vals"), o.get("n_contrib")
    m2, co, rgb, dep = o.get("means2D"), o.get("conic_opacity"), o.get("rgb"), o.get("depths")
    lc = nc[pid].astype(np.int64)
    n = int(lc.max())
    ids = vals[ranges[t, 0]:ranges[t, 0] + n]
    f32 = np.float32
    dxf = m2[ids, 0][:, None] - xs[None].astype(f32)
    dyf = m2[ids, 1][:, None] - ys[None].astype(f32)
    a_, b_, c_, op = (co[ids, k][:, None] for k in range(4))
    power = f32(-0.5) * (a_ * dxf * dxf + c_ * dyf * dyf) - b_ * dxf * dyf
    alf = np.minimum(f32(0.99), op * np.exp(power).astype(f32))
    contrib = (np.arange(n)[:, None] < lc[None]) & ~(power > 0) & ~(alf < f32(1 / 255))
    dx, dy = dxf.astype(np.float64), dyf.astype(np.float64)
    G = np.where(contrib, np.exp(-0.5 * (a_ * dx * dx + c_ * dy * dy) - b_ * dx * dy), 0.0)
    al = np.where(contrib, np.minimum(0.99, op * G), 0.0)
    Tc = np.cumprod(np.vstack([np.ones((1, al.shape[1])), 1 - al]), axis=0)
    Tj, Tfin = Tc[:-1], Tc[-1]
    dp = dp3[:, pid].astype(np.float64)
    di = dinv[pid].astype(np.float64)
    col = rgb[ids].astype(np.float64)
    invd = 1.0 / dep[ids].astype(np.float64)
    cd = col @ dp + invd[:, None] * di[None]
    light = al * Tj * cd
    behind = np.cumsum(light[::-1], axis=0)[::-1] - light + Tfin * (bgv.astype(np.float64) @ dp)
    dLda = Tj * cd - behind / (1 - al)
    u = G * dLda
    aT = al * Tj
    rec = np.stack([(u * dx).sum(1), (u * dy).sum(1), (u * dx * dx).sum(1), (u * dx * dy).sum(1), (u * dy * dy).sum(1),
                    u.sum(1), (aT * dp[0]).sum(1), (aT * dp[1]).sum(1), (aT * dp[2]).sum(1), (aT * di).sum(1)], 1)
    return ids, rec, contrib.any(1)


def main():
    case = int(sys.argv[1])
    d = np.load(os.path.join(ROOT, "gpurun_out", "chair", f"records_case{case}.npz"))
    f, scene, cases = load_chair()
    cam, deg, aa, bg, seed = cases[case]
    H, W = cam.image_height, cam.image_width
    o, og = make_chair.run_case(scene, cam, deg, aa, bg, seed, nthreads=8)
    for nm in ("depths", "means2D", "conic_opacity", "rgb"):
        same = np.array_equal(d[nm].view(np.uint32), o.get(nm).view(np.uint32).reshape(d[nm].shape))
        print(f"HIP {nm} bit-identical to the oracle's: {same}")
    gc, gi = synthetic.make_grads(H, W, seed=seed)
    dp3, dinv = gc.numpy().reshape(3, -1), gi.numpy().reshape(-1)
    bgv = np.asarray(bg, np.float32)
    gx = (W + 15) // 16
    ids, emit, tt, r4 = d["ids"], d["emit_start"], d["tiles_touched"], d["rect4"]
    mask, valid, slots, recs = d["rec_mask"], d["valid"], d["slots"], d["records"]
    k = 0
    cache = {}
    for g in ids:
        n = int(tt[g])
        rs, ss = recs[k:k + n], slots[k:k + n]
        k += n
        r = int(r4[g])
        x0, y0, x1, y1 = r & 0xFF, (r >> 8) & 0xFF, (r >> 16) & 0xFF, r >> 24
        w = max(x1 - x0, 1)
        tot64 = np.zeros(10)
        tothip = np.zeros(10)
        worst = []
        for loc in range(n):
            t = (y0 + loc // w) * gx + (x0 + loc % w)
            if t not in cache:
                cache[t] = tile_records_f64(o, t, W, H, dp3, dinv, bgv)
            tids, trec, tany = cache[t]
            pos = np.nonzero(tids == g)[0]
            ref = trec[pos[0]] if len(pos) and tany[pos[0]] else np.zeros(10)
            flag = bool((mask[g] >> loc) & 1) if loc < 32 else bool((valid[(emit[g] + loc) >> 5] >> ((emit[g] + loc) & 31)) & 1)
            hip = rs[loc, :10].astype(np.float64) if flag else np.zeros(10)
            tot64 += ref
            tothip += hip
            err = np.abs(hip - ref).max() / max(np.abs(ref).max(), 1e-30)
            worst.append((err, loc, t, flag, bool(len(pos) and tany[pos[0]]), np.abs(ref).max()))
        worst.sort(reverse=True)
        sc = np.abs(tot64).max()
        print(f"g {g}: {n} tiles, total rel err {np.abs(tothip - tot64).max() / sc:.2e}; worst tiles (err, local, tile, hip flag, ref nonzero, |ref|/|total|):",
              [(f"{e:.1e}", l, t, fl, nz, f"{m / sc:.1e}") for e, l, t, fl, nz, m in worst[:3]])


if __name__ == "__main__":
    main()
