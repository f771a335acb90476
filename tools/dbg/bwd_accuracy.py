#!/usr/bin/env python3
"""Accuracy of the render backward's formulations on the chair fixture (CPU, numpy emulation).

Per (tile, Gaussian) record -- the ten per-Gaussian sums render_bwd writes (opacity, mean2D x/y,
conic a/b/c, colour r/g/b) -- three ways, for a sample of tiles of one chair case:
  f64  : float64 arithmetic, the oracle's float32 contribution decisions (the yardstick);
  ref  : the reference's float32 order (backward.cu:452-638: back to front, T rebuilt by division,
         accum_rec per channel);
  hip  : render_bwd's float32 formulation (front to back, B = R - sum alpha T (c . dL), R from
         the forward's accumulated colour), with VARIANTS of the B bookkeeping;
  hip_b2f: back to front as the reference, T rebuilt by the reciprocal of (1 - alpha), the colour
         behind carried as ONE normalised scalar (c . dL behind, a convex recurrence).
Prints p99 / p99.9 of |x - f64| / |f64| over records with |f64| > 1e-3 max, per variant.
Usage: python tools/dbg/bwd_accuracy.py [case] [ntiles]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "tests/golden", "oracle", ".")]
import make_chair  # noqa: E402
import synthetic  # noqa: E402
from test_chair import load_chair  # noqa: E402

f32 = np.float32
RNG = np.random.default_rng(1)
LOG2E = f32(1.4426950408889634)


def tile_pixels(tx, ty, W, H):
    ys, xs = np.meshgrid(np.arange(16) + 16 * ty, np.arange(16) + 16 * tx, indexing="ij")
    m = (xs < W) & (ys < H)
    return xs[m].astype(np.int64), ys[m].astype(np.int64)


def run(case=2, ntiles=200, seed=0):
    f, scene, cases = load_chair()
    cam, deg, aa, bg, gseed = cases[case]
    o, _ = make_chair.run_case(scene, cam, deg, aa, bg, gseed, nthreads=8)
    H, W = cam.image_height, cam.image_width
    gc, _ = synthetic.make_grads(H, W, seed=gseed)
    dLp = gc.numpy().astype(f32).reshape(3, -1)
    vals, ranges = o.get("vals"), o.get("ranges")
    nc, fT = o.get("n_contrib"), o.get("final_T")
    m2, co, rgb = o.get("means2D"), o.get("conic_opacity"), o.get("rgb")
    bgv = np.asarray(bg, f32)
    gx = (W + 15) // 16
    rng = np.random.default_rng(seed)
    nonempty = np.nonzero(ranges[:, 1] > ranges[:, 0])[0]
    tiles = rng.choice(nonempty, size=min(ntiles, nonempty.size), replace=False)
    out = {k: [] for k in ("f64", "ref", "hip", "hip_split", "hip_chan", "hip_b2f", "hip_b2f_rcp1", "hip_b2fq", "hip_b2fq_rcp1", "hip_g", "hip_fold")}
    for t in tiles:
        tx, ty = t % gx, t // gx
        xs, ys = tile_pixels(tx, ty, W, H)
        pid = ys * W + xs
        px, py = xs.astype(f32), ys.astype(f32)
        r0, r1 = int(ranges[t, 0]), int(ranges[t, 1])
        lc = nc[pid].astype(np.int64)
        n = int(lc.max()) if lc.size else 0
        ids = vals[r0:r0 + n]
        dp = dLp[:, pid]  # (3, npix)
        # decisions, float32 as the oracle (power > 0, alpha < 1/255, position < last contributor)
        dxf = m2[ids, 0][:, None] - px[None]
        dyf = m2[ids, 1][:, None] - py[None]
        a_, b_, c_, op = (co[ids, k][:, None] for k in range(4))
        power = f32(-0.5) * (a_ * dxf * dxf + c_ * dyf * dyf) - b_ * dxf * dyf
        Gf = np.exp(power).astype(f32)
        alf = np.minimum(f32(0.99), op * Gf)
        pos = np.arange(n)[:, None]
        contrib = (pos < lc[None]) & ~(power > 0) & ~(alf < f32(1 / 255))
        col = rgb[ids]  # (n, 3)
        # ---- f64 ----
        dx, dy = dxf.astype(np.float64), dyf.astype(np.float64)
        G = np.where(contrib, np.exp(-0.5 * (a_ * dx * dx + c_ * dy * dy) - b_ * dx * dy), 0.0)
        al = np.where(contrib, np.minimum(0.99, op * G), 0.0)
        T = np.cumprod(np.vstack([np.ones((1, al.shape[1])), 1 - al]), axis=0)
        Tj, Tfin = T[:-1], T[-1]
        cd = col.astype(np.float64) @ dp.astype(np.float64)  # (n, npix)
        light = al * Tj * cd
        behind = np.cumsum(light[::-1], axis=0)[::-1] - light + Tfin * (bgv.astype(np.float64) @ dp)
        dLda = Tj * cd - behind / (1 - al)
        out["f64"].append(records(G, dLda, al * Tj, dx, dy, dp.astype(np.float64), contrib))
        # ---- reference float32 order ----
        Gr, alr = np.where(contrib, Gf, f32(0)), np.where(contrib, alf, f32(0))
        Tr = fT[pid].astype(f32).copy()
        acc_rec = np.zeros((3, len(pid)), f32)
        last_a = np.zeros(len(pid), f32)
        last_c = np.zeros((3, len(pid)), f32)
        dLda_r = np.zeros((n, len(pid)), f32)
        aT_r = np.zeros((n, len(pid)), f32)
        bgd = (bgv[:, None] * dp).sum(0, dtype=f32)
        for j in range(n - 1, -1, -1):
            c = contrib[j]
            Tr = np.where(c, Tr / (f32(1) - alr[j]), Tr).astype(f32)
            d = np.zeros(len(pid), f32)
            for ch in range(3):
                ar = (last_a * last_c[ch] + (f32(1) - last_a) * acc_rec[ch]).astype(f32)
                acc_rec[ch] = np.where(c, ar, acc_rec[ch])
                last_c[ch] = np.where(c, col[j, ch], last_c[ch])
                d = d + (col[j, ch] - acc_rec[ch]) * dp[ch]
            d = d * Tr + (-fT[pid] / (f32(1) - alr[j])) * bgd
            last_a = np.where(c, alr[j], last_a)
            dLda_r[j] = np.where(c, d, 0)
            aT_r[j] = np.where(c, alr[j] * Tr, 0)
        out["ref"].append(records(Gr, dLda_r, aT_r, dxf, dyf, dp, contrib))
        # ---- hip: forward-order B ----
        for var in ("hip_b2f_rcp1", "hip_fold"):
            out[var].append(hip_records(var, contrib, Gr, alr, col, dp, dxf, dyf, fT[pid], bgv))
        # the render kernels' falloff: conic pre-scaled into log2 units (preprocess.hip), p2 by two
        # fused multiply-adds, exp2 (render.hip bwd_pair)
        ka, kb, kc = f32(-0.5 * 1.4426950408889634) * a_, f32(-1.4426950408889634) * b_, f32(-0.5 * 1.4426950408889634) * c_
        d64 = lambda x: x.astype(np.float64)
        bq = (kb * dyf).astype(f32)
        cq = ((kc * dyf).astype(f32) * dyf).astype(f32)
        inner = (d64(ka) * d64(dxf) + d64(bq)).astype(f32)
        p2 = (d64(inner) * d64(dxf) + d64(cq)).astype(f32)
        Gh = np.where(contrib, np.exp2(p2).astype(f32), f32(0))
        alh = np.where(contrib, np.minimum(f32(0.99), Gh * op), f32(0)).astype(f32)
        out["hip_g"] = out.get("hip_g", [])
        out["hip_g"].append(hip_records("hip_b2fq", contrib, Gh, alh, col, dp, dxf, dyf, fT[pid], bgv))
    f64 = np.concatenate(out["f64"])
    sel = np.abs(f64) > 1e-3 * np.abs(f64).max(axis=0, keepdims=True)
    names = ["opacity", "mean_x", "mean_y", "conic_a", "conic_b", "conic_c", "col_r", "col_g", "col_b"]
    for k in ("ref", "hip_b2f_rcp1", "hip_fold"):
        x = np.concatenate(out[k]).astype(np.float64)
        rel = np.abs(x - f64) / np.where(sel, np.abs(f64), 1)
        line = " ".join(f"{nm}={np.quantile(rel[:, i][sel[:, i]], 0.999):.1e}" for i, nm in enumerate(names))
        print(f"{k:10s} p99.9: {line}")


def records(G, dLda, aT, dx, dy, dp, contrib):
    """(n_entries, 9) per-record sums of the tile's pixels (entries with any contribution)."""
    u = G * dLda
    rec = np.stack([u.sum(1), (u * dx).sum(1), (u * dy).sum(1), (u * dx * dx).sum(1), (u * dx * dy).sum(1),
                    (u * dy * dy).sum(1), (aT * dp[0]).sum(1), (aT * dp[1]).sum(1), (aT * dp[2]).sum(1)], 1)
    return rec[contrib.any(1)]


def hip_records(var, contrib, G, al, col, dp, dx, dy, fT, bgv):
    n, npx = G.shape
    def rcp(x, noisy):
        r = (f32(1) / x).astype(f32)
        if noisy:  # v_rcp_f32: up to 1 ulp; model it as a random +-1 ulp error
            r = np.where(RNG.random(r.shape) < 0.5, np.nextafter(r, f32(np.inf)), np.nextafter(r, f32(0))).astype(f32)
        return r
    if var.startswith("hip_b2fq"):  # back to front: T_j = T_final / prod_{k >= j} (1 - alpha_k)
        noisy = var.endswith("rcp1")
        Tf = fT.astype(f32)
        bgd = (bgv[:, None] * dp).sum(0, dtype=f32)
        Q = np.ones(npx, f32)
        Bn = np.zeros(npx, f32)
        dLda = np.zeros((n, npx), f32)
        aT = np.zeros((n, npx), f32)
        for j in range(n - 1, -1, -1):
            a = np.where(contrib[j], al[j], f32(0))
            Qn = (Q * (f32(1) - a)).astype(f32)
            T = (Tf * rcp(Qn, noisy)).astype(f32)
            cd = (col[j, 0] * dp[0] + col[j, 1] * dp[1] + col[j, 2] * dp[2]).astype(f32)
            diff = (cd - Bn).astype(f32)
            dLda[j] = np.where(contrib[j], T * (diff - Q * bgd), 0)
            Bn = (Bn + a * diff).astype(f32)
            aT[j] = a * T
            Q = Qn
        return records(G, dLda, aT, dx, dy, dp, contrib)
    if var == "hip_fold":  # back to front, the background folded into the colour behind (render.hip)
        T = fT.astype(f32).copy()
        Bn = (bgv[:, None] * dp).sum(0, dtype=f32).astype(f32)
        dLda = np.zeros((n, npx), f32)
        aT = np.zeros((n, npx), f32)
        for j in range(n - 1, -1, -1):
            a = np.where(contrib[j], al[j], f32(0))
            r = np.where(a > 0, rcp(f32(1) - a, True), f32(1))
            T = (T * r).astype(f32)
            cd = (col[j, 0] * dp[0] + col[j, 1] * dp[1] + col[j, 2] * dp[2]).astype(f32)
            diff = (cd - Bn).astype(f32)
            dLda[j] = np.where(contrib[j], T * diff, 0)
            Bn = (Bn + a * diff).astype(f32)
            aT[j] = a * T
        return records(G, dLda, aT, dx, dy, dp, contrib)
    if var.startswith("hip_b2f"):  # back to front: T rebuilt by the reciprocal, normalised colour behind
        noisy = var.endswith("rcp1")
        T = fT.astype(f32).copy()
        K = (fT.astype(f32) * (bgv[:, None] * dp).sum(0, dtype=f32)).astype(f32)
        Bn = np.zeros(npx, f32)
        dLda = np.zeros((n, npx), f32)
        aT = np.zeros((n, npx), f32)
        for j in range(n - 1, -1, -1):
            a = np.where(contrib[j], al[j], f32(0))
            r = np.where(a > 0, rcp(f32(1) - a, noisy), f32(1))
            T = (T * r).astype(f32)
            cd = (col[j, 0] * dp[0] + col[j, 1] * dp[1] + col[j, 2] * dp[2]).astype(f32)
            diff = (cd - Bn).astype(f32)
            dLda[j] = np.where(contrib[j], T * diff - r * K, 0)
            Bn = (Bn + a * diff).astype(f32)
            aT[j] = a * T
        return records(G, dLda, aT, dx, dy, dp, contrib)
    # the forward's accumulated colour, float32 front to back (render_fwd)
    T = np.ones(npx, f32)
    acc = np.zeros((3, npx), f32)
    for j in range(n):
        c = contrib[j]
        for ch in range(3):
            acc[ch] = np.where(c, acc[ch] + col[j, ch] * (al[j] * T), acc[ch]).astype(f32)
        T = np.where(c, T * (f32(1) - al[j]), T).astype(f32)
    Tfin = fT.astype(f32)
    R_acc = (acc * dp).sum(0, dtype=f32)
    R_bg = Tfin * (bgv[:, None] * dp).sum(0, dtype=f32)
    T = np.ones(npx, f32)
    if var == "hip":
        B = (R_acc + R_bg).astype(f32)
    elif var == "hip_split":
        B = R_acc.copy()
    else:
        Bc = acc.copy()  # per channel: acc_c - running sum, exact order of the forward
        S = np.zeros((3, npx), f32)
    dLda = np.zeros((n, npx), f32)
    aT = np.zeros((n, npx), f32)
    for j in range(n):
        c = contrib[j]
        a = np.where(c, al[j], f32(0))
        cd = (col[j, 0] * dp[0] + col[j, 1] * dp[1] + col[j, 2] * dp[2]).astype(f32)
        at = (a * T).astype(f32)
        r = (f32(1) / (f32(1) - a)).astype(f32)
        if var == "hip":
            B = (B - at * cd).astype(f32)
            d = T * cd - B * r
        elif var == "hip_split":
            B = (B - at * cd).astype(f32)
            d = T * cd - (B + R_bg) * r
        else:
            for ch in range(3):
                S[ch] = np.where(c, S[ch] + col[j, ch] * at, S[ch]).astype(f32)
            Bj = ((acc - S) * dp).sum(0, dtype=f32) + R_bg
            d = T * cd - Bj * r
        dLda[j] = np.where(c, d, 0)
        aT[j] = at
        T = (T * (f32(1) - a)).astype(f32)
    return records(G, dLda, aT, dx, dy, dp, contrib)


if __name__ == "__main__":
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 2, int(sys.argv[2]) if len(sys.argv) > 2 else 200)
