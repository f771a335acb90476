"""Shared helpers for the parity tests: build a case, run the oracle and the HIP path on it."""
import os

import numpy as np
import torch

import synthetic

ROOT_OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")

# Tolerances (fp32).  Preprocess outputs and the sorted key/value arrays are compared
# bit-exactly.  Render outputs differ from the oracle only through exp() (v_exp_f32 vs
# glibc expf) and summation order of the gradient atomics, so they are compared with
# these tolerances, relative to each tensor's max-abs:
IMG_ATOL = 2e-5          # pixel RGB / invdepth / final_T absolute
GRAD_RTOL = 1e-4         # gradients: |a-b| <= GRAD_RTOL * max|b| + GRAD_ATOL (per element)
GRAD_ATOL = 1e-6
# A pixel whose contributor set differs because an alpha sits within ~1 ulp of the
# 1/255 or 1e-4 thresholds ("flipped": n_contrib differs, or some channel is off by more than
# IMG_ATOL) is allowed to differ; at most this fraction of pixels may, and even there by at
# most FLIP_MAX_ABS.  Bound of one flipped decision (forward.cu:364-370): a Gaussian k with
# alpha_k ~ 1/255 blended or not changes the pixel by alpha_k T_k (c_k - C_behind_k), and the
# stop rule moves the stopping Gaussian's alpha T c with T (1 - alpha) ~ 1e-4, so
# |d colour| <= (1/255) |c_k - C_behind| ~ 5e-3 for the synthetic scenes' rgb (<= 1.2), and
# |d final_T| <= 1/255.  Measured (GPU round 2, gpurun_out/*/parity_stats.json): config 2
# (1M, 1080p) 8 of 2.07M pixels flipped, largest 5.9e-4; the 3840x2176 case 2 of 8.4M pixels,
# 2.05e-3 (a flip at T ~ 1, final_T off by 1/255); every other case none.
FLIP_FRACTION = 1e-4
FLIP_MAX_ABS = 5e-3
# A decision taken the other way can also move a pixel by less than IMG_ATOL: an alpha at 1/255
# blended at T ~ 1e-3 changes the colour by ~4e-6.  Such a pixel is not "flipped" (the image is
# within tolerance) but the Gaussians of its walk gain or lose one pixel's term, ~1e-4 of their
# gradient (chair fixture, case 1, pixel (600, 29): 7.5e-6, every walk Gaussian's record for that
# tile off by ~1e-4 -- tools/dbg/chair_records_cmp.py).  Pixels off by more than DECISION_ATOL
# (the remaining differences are the rounding of the colour sums: ~1e-7, a handful of pixels per
# million up to ~1e-6) are "decision suspects": the per-element relative checks (check_rel,
# check_rel_truth) leave their walks' Gaussians out, which check_grad_attributed bounds instead.
DECISION_ATOL = 1e-6
# every check_render call appends its statistics here; conftest writes them to
# gpurun_out/parity_stats.json at the end of a session that has any
PARITY_LOG = []


def check_render(name, hip, ora, flips=None, suspects=None):
    """hip / ora: dicts with 'color' (3,H,W), 'invdepth' (1,H,W) and optionally 'final_T' (N)
    and 'n_contrib' (N).  Flipped pixels: n_contrib differs (when both have it) or some
    colour / invdepth / final_T value is off by more than IMG_ATOL.  Asserts: flipped fraction
    <= FLIP_FRACTION, every value of a flipped pixel within FLIP_MAX_ABS (final_T within
    1/255 + IMG_ATOL), all others within IMG_ATOL with the same n_contrib.  `flips`: a list that
    receives the flipped pixels' mask (bool (N,)), for flip_gaussians; `suspects` the mask of the
    flipped pixels and those off by more than DECISION_ATOL."""
    c = np.abs(np.asarray(hip["color"], np.float64) - np.asarray(ora["color"], np.float64))
    N = c.shape[-1] * c.shape[-2]
    err = c.reshape(c.shape[0], N).max(0)
    if "invdepth" in hip and "invdepth" in ora:
        err = np.maximum(err, np.abs(np.asarray(hip["invdepth"], np.float64)
                                     - np.asarray(ora["invdepth"], np.float64)).reshape(N))
    terr = None
    if "final_T" in hip and "final_T" in ora:
        terr = np.abs(np.asarray(hip["final_T"], np.float64) - np.asarray(ora["final_T"], np.float64)).reshape(N)
    flip = err > IMG_ATOL
    if terr is not None:
        flip |= terr > IMG_ATOL
    nc_diff = 0
    if "n_contrib" in hip and "n_contrib" in ora:
        d = np.asarray(hip["n_contrib"]).reshape(N) != np.asarray(ora["n_contrib"]).reshape(N)
        nc_diff = int(d.sum())
        flip |= d
    n_flip = int(flip.sum())
    if flips is not None:
        flips.append(flip)
    suspect = flip | (err > DECISION_ATOL)
    if terr is not None:
        suspect |= terr > DECISION_ATOL
    if suspects is not None:
        suspects.append(suspect)
    stats = {"name": name, "pixels": N, "flipped": n_flip, "frac": n_flip / max(N, 1), "n_contrib_diff": nc_diff,
             "max_err_flipped": float(err[flip].max()) if n_flip else 0.0,
             "max_err_other": float(err[~flip].max()) if n_flip < N else 0.0,
             "max_T_err_flipped": float(terr[flip].max()) if (n_flip and terr is not None) else 0.0,
             "decision_suspects": int(suspect.sum())}
    PARITY_LOG.append(stats)
    assert stats["frac"] <= FLIP_FRACTION, f"{name}: {n_flip} of {N} pixels flipped ({stats})"
    assert stats["max_err_flipped"] <= FLIP_MAX_ABS, f"{name}: flipped pixel off by {stats['max_err_flipped']:.3e}"
    assert stats["max_T_err_flipped"] <= 1.0 / 255.0 + IMG_ATOL, f"{name}: final_T off ({stats})"
    return stats


def make_case(P=1000, H=256, W=256, view=0, seed=0, sh_degree=3, bg=(0.0, 0.0, 0.0)):
    sc = synthetic.make_scene(P, seed=seed, sh_degree=sh_degree)
    cam = synthetic.Camera(W, H, view)
    gc, gi = synthetic.make_grads(H, W, seed=seed + 1)
    return dict(scene=sc, cam=cam, H=H, W=W, bg=torch.tensor(bg, dtype=torch.float32), sh_degree=sh_degree,
                grad_color=gc, grad_invdepth=gi)


def run_oracle(case, mode="sh_scales", antialiasing=False, nthreads=1, backward=True, scale_modifier=1.0):
    import oracle
    sc, cam = case["scene"], case["cam"]
    kw = {}
    if mode in ("sh_scales", "sh_cov"):
        kw.update(shs=sc["shs"], sh_degree=case["sh_degree"])
    else:
        kw.update(colors_precomp=case["colors_precomp"])
    if mode in ("sh_scales", "colors_scales"):
        kw.update(scales=sc["scales"], rotations=sc["rotations"])
    else:
        kw.update(cov3D_precomp=case["cov3D_precomp"])
    o = oracle.OracleRaster(sc["means3D"], sc["opacities"], case["bg"], cam.world_view_transform,
                            cam.full_proj_transform, cam.camera_center, cam.tanfovx, cam.tanfovy, case["H"],
                            case["W"], antialiasing=antialiasing, nthreads=nthreads, scale_modifier=scale_modifier,
                            **kw)
    grads = o.backward(case["grad_color"], case["grad_invdepth"]) if backward else None
    return o, grads


# Per-element relative error of a gradient (a tolerance relative to each
# tensor's max can hide large relative errors on the many small elements).  Over the elements with
# |ref| > REL_FLOOR * max|ref|: the 99.9th percentile of |hip - ref| / |ref| must stay within
# REL_P999, and at most REL_OUT_FRAC of them may exceed REL_OUT (fp32 reassociation of sums with
# cancellation -- an element that is a small difference of large per-pixel terms -- and the
# flipped pixels of check_render are the sources).
REL_FLOOR = 1e-3
REL_P999 = 1e-3
REL_OUT = 1e-2
REL_OUT_FRAC = 1e-4
# check_rel: at most this share of the rows may be left out as decision suspects (0.1; round 5 raised the
# global cap to 0.2 for one case -- chair case 4 -- which now passes its own cap, test_chair_gpu.py)
REL_LEFT_OUT_FRAC = 0.1


def rel_stats(hip, ref, floor=REL_FLOOR):
    """Per-element relative-error statistics of hip against ref over |ref| > floor * max|ref|."""
    a = np.asarray(hip, np.float64).reshape(-1)
    b = np.asarray(ref, np.float64).reshape(-1)
    scale = np.abs(b).max() if b.size else 0.0
    sel = np.abs(b) > floor * scale
    n = int(sel.sum())
    if n == 0:
        return {"considered": 0, "p99": 0.0, "p999": 0.0, "max": 0.0, "n_over_1e-3": 0, "n_over_REL_OUT": 0}
    r = np.abs(a[sel] - b[sel]) / np.abs(b[sel])
    return {"considered": n, "p99": float(np.quantile(r, 0.99)), "p999": float(np.quantile(r, 0.999)),
            "max": float(r.max()), "n_over_1e-3": int((r > 1e-3).sum()), "n_over_REL_OUT": int((r > REL_OUT).sum())}


def check_rel(name, hip, ref, affected=None, truth_stats=None, max_left_out_frac=REL_LEFT_OUT_FRAC):
    """Asserts the per-element relative-error bounds above over the rows (Gaussians) outside
    `affected` (the walks of decision-suspect pixels: their rows are bounded by
    check_grad_attributed); returns (and logs) the statistics.  truth_stats: the oracle's own
    statistics against the float64 yardstick (check_rel_truth) -- the HIP-vs-oracle difference is
    at most the sum of the two errors, so the bound on it becomes max(REL_P999, (1 + TRUTH_FACTOR)
    x the oracle's p99.9 + TRUTH_SLACK): where the reference's float32 order is itself 9e-4 from
    float64 (the chair on white), a 1e-3 bound between two float32 results tests the oracle."""
    if affected is not None:
        keep = ~np.asarray(affected, bool)
        hip = np.asarray(hip).reshape(len(keep), -1)[keep]
        ref = np.asarray(ref).reshape(len(keep), -1)[keep]
    st = rel_stats(hip, ref)
    bound = REL_P999 if truth_stats is None else max(REL_P999, (1 + TRUTH_FACTOR) * truth_stats["p999"] + TRUTH_SLACK)
    left_out = 0 if affected is None else int((~keep).sum())
    PARITY_LOG.append({"name": name + " rel", "rows_left_out": left_out, "p999_bound": bound, **st})
    # the rows left out (decision suspects' walks) stay a small share of the Gaussians (measured: at most
    # 11.4 % on the chair fixture's perturbed case 4, whose 100k Gaussians are densely packed behind
    # few pixels -- 15 suspect pixels -- which passes its own cap; 0.05 % at config 3's scale)
    assert left_out <= max_left_out_frac * max(len(keep) if affected is not None else 0, 1), \
        f"{name}: {left_out} rows left out of the per-element check"
    assert st["p999"] <= bound, f"{name}: 99.9th percentile relative error {st['p999']:.3e} > {bound:.3e} ({st})"
    assert st["n_over_REL_OUT"] <= max(2, REL_OUT_FRAC * st["considered"]), f"{name}: {st}"
    return st


# Accuracy against float64 (the oracle's render backward in float64 arithmetic on the same
# contribution decisions, OracleRaster.backward(f64=True)): the HIP gradients may be at most
# TRUTH_FACTOR times as far from it (99.9th percentile of the per-element relative error, over
# the elements above REL_FLOOR of the max) as the reference's own float32 order is, plus
# TRUTH_SLACK.  This pins the ACCURACY of the HIP formulation to the reference's, where the
# HIP-vs-oracle comparison alone cannot tell whose rounding an element's difference is.  The
# Gaussians in the walks of decision-suspect pixels (`affected`: flip_gaussians of check_render's
# `suspects`) are left out: there the HIP path may have taken a float32 blend decision the other
# way (an alpha within an ulp of 1/255), which the float64 yardstick, built on the oracle's
# decisions, does not share (check_grad_attributed bounds those rows).
TRUTH_FACTOR = 1.5
TRUTH_SLACK = 5e-5


def check_rel_truth(name, hip, ref, truth, affected=None):
    """Logs hip-vs-truth and oracle-vs-truth relative-error statistics over the rows (Gaussians)
    outside `affected`; asserts the bound above."""
    hip, ref, truth = (np.asarray(x, np.float64).reshape(len(x), -1) for x in (hip, ref, truth))
    keep = np.ones(len(truth), bool) if affected is None else ~np.asarray(affected, bool)
    sh, so = rel_stats(hip[keep], truth[keep]), rel_stats(ref[keep], truth[keep])
    PARITY_LOG.append({"name": name + " vs float64", "rows_left_out": int((~keep).sum()), "hip": sh,
                       "oracle_f32": so})
    assert sh["p999"] <= TRUTH_FACTOR * so["p999"] + TRUTH_SLACK, \
        f"{name}: p99.9 error vs float64 {sh['p999']:.3e}, the reference order's {so['p999']:.3e}"
    return sh, so


def allclose_rel(a, b, rtol=GRAD_RTOL, atol=GRAD_ATOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max() if b.size else 0.0, 1e-30)
    err = np.abs(a - b)
    return bool(np.all(err <= rtol * scale + atol)), float(err.max() / scale if err.size else 0.0)


# ---- attribution of gradient outliers to flipped pixels -------------------
# A flipped pixel (check_render) changes the blend of every Gaussian its walk passes: the reference's
# backward replays the pixel's list from its n_contrib down (backward.cu:452-638), and dL/dalpha of
# each of those Gaussians holds the colour behind it and T in front of it (forward.cu:359-370: one
# Gaussian blended or skipped at the 1/255 threshold, or the stop rule firing one entry earlier or
# later, shifts both).  The Gaussians at list positions [0, max(n_contrib_hip, n_contrib_oracle))
# of a flipped pixel's tile are the only ones whose gradients a flip can move.  Every gradient
# element beyond GRAD_RTOL of max|ref| (or beyond REL_OUT relative to itself) must belong to such
# a Gaussian; outside that set the plain tolerance holds, inside it GRAD_RTOL_ATTRIBUTED.
# (Round 5 raised it to 5e-3 after a 2.005e-3 attributed row in a 3,001-Gaussian, 4080 x 256 case of
# test_packed_rect_boundary_keys_bit_exact: where a Gaussian covers few pixels, one flipped pixel's term
# is a larger share of its gradient.  Round 6 restored 2e-3 here; that test passes its own
# GRAD_RTOL_ATTRIBUTED_SMALL_FOOTPRINT.  The count of such rows is capped below.  That the flips are
# the only source is shown by tests/test_ref_alpha_exact.py: with the blend in the reference's
# operation order there are no flipped pixels and no row beyond GRAD_RTOL.)
GRAD_RTOL_ATTRIBUTED = 2e-3
GRAD_RTOL_ATTRIBUTED_SMALL_FOOTPRINT = 5e-3
# and only a few of the attributed Gaussians may actually be off beyond GRAD_RTOL: at most
# max(ATTR_ROWS_MIN, ATTR_ROWS_FRAC x the walks' Gaussians) rows (measured through round 4: at most
# 16 rows of 17,250 for the 8-view sum, a ratio of at most 0.0018 per view), so a real regression
# cannot hide among the thousands of Gaussians a handful of flipped pixels' walks pass
ATTR_ROWS_MIN = 64
ATTR_ROWS_FRAC = 0.01


def flip_gaussians(flip, nc_hip, nc_ora, vals, ranges, W, H, P):
    """bool (P,): the Gaussians in the walk of some flipped pixel (flip: bool (N,) from
    check_render; nc_*: n_contrib (N,); vals / ranges: the oracle's sorted Gaussian ids and
    per-tile [start, end) ranges)."""
    out = np.zeros(P, dtype=bool)
    tiles_x = (W + 15) // 16
    vals = np.asarray(vals)
    ranges = np.asarray(ranges).reshape(-1, 2)
    nc_hip = np.asarray(nc_hip).reshape(-1)
    nc_ora = np.asarray(nc_ora).reshape(-1)
    for pix in np.flatnonzero(np.asarray(flip).reshape(-1)):
        y, x = divmod(int(pix), W)
        t = (y // 16) * tiles_x + x // 16
        start, end = int(ranges[t, 0]), int(ranges[t, 1])
        n = min(max(int(nc_hip[pix]), int(nc_ora[pix])), end - start)
        out[vals[start:start + n]] = True
    return out


def check_grad_attributed(name, hip, ref, affected, rtol_attr=GRAD_RTOL_ATTRIBUTED):
    """Per-Gaussian gradient (P, ...) against the oracle with outliers attributed to flips:
    rows (Gaussians) holding an element beyond GRAD_RTOL * max|ref| + GRAD_ATOL, or beyond REL_OUT
    relative to |ref| where |ref| > REL_FLOOR * max|ref|, must lie in `affected` (flip_gaussians);
    every element of an affected row within rtol_attr * max|ref|.  Logs the attributed and
    unattributed counts; asserts no unattributed row."""
    P = affected.shape[0]
    a = np.asarray(hip, np.float64).reshape(P, -1)
    b = np.asarray(ref, np.float64).reshape(P, -1)
    scale = max(float(np.abs(b).max()) if b.size else 0.0, 1e-30)
    err = np.abs(a - b)
    over = err > GRAD_RTOL * scale + GRAD_ATOL
    sel = np.abs(b) > REL_FLOOR * scale
    with np.errstate(divide="ignore", invalid="ignore"):
        over_rel = sel & (err > REL_OUT * np.abs(b))
    rows = (over | over_rel).any(axis=1)
    unattr = rows & ~affected
    st = {"name": name + " attributed", "elements": int(err.size), "affected_gaussians": int(affected.sum()),
          "rows_over": int(rows.sum()), "attributed_rows": int((rows & affected).sum()),
          "unattributed_rows": int(unattr.sum()),
          "max_rel_to_max_outside": float(err[~affected].max() / scale) if (~affected).any() else 0.0,
          "max_rel_to_max_inside": float(err[affected].max() / scale) if affected.any() else 0.0}
    PARITY_LOG.append(st)
    assert st["unattributed_rows"] == 0, (
        f"{name}: {st['unattributed_rows']} Gaussians off beyond tolerance outside every flipped pixel's walk "
        f"(rows {np.flatnonzero(unattr)[:8].tolist()}, {st})")
    assert st["max_rel_to_max_inside"] <= rtol_attr, f"{name}: attributed error too large ({st})"
    assert st["attributed_rows"] <= max(ATTR_ROWS_MIN, ATTR_ROWS_FRAC * st["affected_gaussians"]), \
        f"{name}: {st['attributed_rows']} attributed rows off beyond tolerance ({st})"
    return st
