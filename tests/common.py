"""Shared helpers for the parity tests: build a case, run the oracle and the HIP path on it."""
import numpy as np
import torch

import synthetic

# Tolerances (fp32).  Preprocess outputs and the sorted key/value arrays are compared
# bit-exactly.  Render outputs differ from the oracle only through exp() (v_exp_f32 vs
# glibc expf) and summation order of the gradient atomics, so they are compared with
# these tolerances, relative to each tensor's max-abs:
IMG_ATOL = 2e-5          # pixel RGB / invdepth / final_T absolute
GRAD_RTOL = 1e-4         # gradients: |a-b| <= GRAD_RTOL * max|b| + GRAD_ATOL (per element)
GRAD_ATOL = 1e-6
# A pixel whose contributor set differs because an alpha sits within ~1 ulp of the
# 1/255 or 1e-4 thresholds is allowed to differ; at most this fraction of pixels may.
FLIP_FRACTION = 1e-3


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


def allclose_rel(a, b, rtol=GRAD_RTOL, atol=GRAD_ATOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max() if b.size else 0.0, 1e-30)
    err = np.abs(a - b)
    return bool(np.all(err <= rtol * scale + atol)), float(err.max() / scale if err.size else 0.0)
