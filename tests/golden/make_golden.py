#!/usr/bin/env python3
"""Generates the committed golden fixtures tests/golden/*.npz.

Runs only in the build container (it reads /root/reference, which does not exist on the GPU
box).  Each fixture holds the inputs of one rasterizer call, the CPU oracle's outputs
(oracle/gsr_oracle.c, 1 thread, deterministic) and the values the reference's OWN Python
computes for the same inputs, which pin the parts of the path that the reference can run
here:

* viewmatrix / projmatrix / campos: utils/graphics_utils.py getWorld2View2 (:38-49) and
  getProjectionMatrix (:51-71), assembled as scene/cameras.py:86-89 does;
* ref_rgb: gaussian_renderer/__init__.py:76-80 (eval_sh, utils/sh_utils.py:57-112, + 0.5,
  clamp_min 0), the Python twin of forward.cu computeColorFromSH;
* ref_cov3D: scene/gaussian_model.py:33-37 (build_scaling_rotation + strip_symmetric,
  utils/general_utils.py:64-112), the Python twin of forward.cu computeCov3D;
* the single / two Gaussian hand cases: attribute rows read from the reference's own PLY
  fixtures GS-IRON/npu-1/{single_gaussian,two_gaussians}.ply, activated as
  scene/gaussian_model.py:263-320 + :100-125 do (exp scales, sigmoid opacity, normalised
  quaternion, f_rest reshaped (P,3,15) then transposed).

The reference rasterizer itself (CUDA) cannot run here, so the image /
key / gradient arrays are the oracle's; tests/test_oracle.py checks that the oracle
reproduces them bit-exactly and agrees with the ref_* arrays, and tests/test_gpu_parity.py
checks the HIP path against them on the GPU.

Usage: python tests/golden/make_golden.py   (rewrites tests/golden/*.npz)
"""
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, REF)

import oracle  # noqa: E402
import synthetic  # noqa: E402
from utils.graphics_utils import getProjectionMatrix, getWorld2View2  # noqa: E402  (reference)
from utils.sh_utils import eval_sh  # noqa: E402  (reference)
import utils.general_utils as ref_gu  # noqa: E402  (reference)


def ref_camera(W, H, view):
    """Matrices through the reference's own functions (scene/cameras.py:86-89)."""
    R, t = synthetic.ring_camera_RT(view)
    fovy = math.radians(50.0)
    fovx = 2.0 * math.atan(math.tan(fovy / 2) * W / H)
    wv = torch.tensor(getWorld2View2(R, t, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
    proj = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
    campos = wv.inverse()[3, :3]
    return wv.float(), full.float(), campos.float(), math.tan(fovx * 0.5), math.tan(fovy * 0.5)


def ref_rgb(means3D, shs, campos, deg):
    """gaussian_renderer/__init__.py:76-80 with the reference's eval_sh."""
    shs_view = torch.as_tensor(shs).transpose(1, 2).reshape(-1, 3, shs.shape[1])
    dir_pp = torch.as_tensor(means3D) - campos.repeat(shs.shape[0], 1)
    dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    sh2rgb = eval_sh(deg, shs_view, dir_pp_normalized)
    return torch.clamp_min(sh2rgb + 0.5, 0.0).numpy().astype(np.float32)


def ref_cov3D(scales, rotations, scale_modifier):
    """scene/gaussian_model.py:33-37 with the reference's build_scaling_rotation / strip_symmetric.
    build_rotation allocates on device='cuda' (general_utils.py:83); there is no GPU here, so
    torch.zeros is redirected to the CPU for the duration of the call (math unchanged)."""
    orig = torch.zeros

    def zeros_cpu(*a, **k):
        k.pop("device", None)
        return orig(*a, **k)

    ref_gu.torch.zeros = zeros_cpu
    try:
        L = ref_gu.build_scaling_rotation(scale_modifier * torch.as_tensor(scales), torch.as_tensor(rotations))
        cov = L @ L.transpose(1, 2)
        return ref_gu.strip_symmetric(cov).numpy().astype(np.float32)
    finally:
        ref_gu.torch.zeros = orig


def read_ply(path):
    """Binary little-endian PLY with one float vertex element (the reference fixtures' format)."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    header = data[:end].decode("ascii").splitlines()
    n = 0
    props = []
    for line in header:
        parts = line.split()
        if parts[:2] == ["element", "vertex"]:
            n = int(parts[2])
        elif parts[:2] == ["property", "float"]:
            props.append(parts[2])
    arr = np.frombuffer(data[end:end + 4 * n * len(props)], dtype="<f4").reshape(n, len(props))
    return {p: arr[:, i].copy() for i, p in enumerate(props)}


def ply_scene(path):
    """Activated parameters as GaussianModel.load_ply (:276-320) + getters (:100-125) build them."""
    v = read_ply(path)
    P = v["x"].shape[0]
    means = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float32)
    dc = np.stack([v["f_dc_0"], v["f_dc_1"], v["f_dc_2"]], 1)[:, None, :]           # (P,1,3)
    rest = np.stack([v[f"f_rest_{i}"] for i in range(45)], 1).reshape(P, 3, 15)      # (P,3,15)
    shs = np.concatenate([dc, rest.transpose(0, 2, 1)], 1).astype(np.float32)       # (P,16,3)
    scales = np.exp(np.stack([v[f"scale_{i}"] for i in range(3)], 1)).astype(np.float32)
    rot = np.stack([v[f"rot_{i}"] for i in range(4)], 1)
    rot = (rot / np.linalg.norm(rot, axis=1, keepdims=True)).astype(np.float32)
    opac = (1.0 / (1.0 + np.exp(-v["opacity"])))[:, None].astype(np.float32)
    return dict(means3D=means, shs=shs, scales=scales, rotations=rot, opacities=opac)


def make(name, scene, H, W, view, mode="sh_scales", antialiasing=False, sh_degree=3, bg=(0, 0, 0),
         scale_modifier=1.0, grad_seed=1):
    view_m, proj_m, campos, tanfovx, tanfovy = ref_camera(W, H, view)
    # the build's own camera helper must agree with the reference's matrices
    cam = synthetic.Camera(W, H, view)
    np.testing.assert_allclose(cam.world_view_transform.numpy(), view_m.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(cam.full_proj_transform.numpy(), proj_m.numpy(), rtol=0, atol=1e-6)
    sc = {k: np.ascontiguousarray(np.asarray(v), dtype=np.float32) for k, v in scene.items()}
    P = sc["means3D"].shape[0]
    empty = np.zeros((0,), np.float32)
    shs = sc["shs"] if mode.startswith("sh") else empty
    colors = empty if mode.startswith("sh") else ref_rgb(sc["means3D"], sc["shs"], campos, sh_degree)
    use_scales = mode.endswith("scales")
    cov = ref_cov3D(sc["scales"], sc["rotations"], scale_modifier)
    gc, gi = synthetic.make_grads(H, W, seed=grad_seed)
    # stored as float16 (exactly representable inputs, half the fixture size)
    gc, gi = gc.half(), gi.half()
    bg = np.asarray(bg, np.float32)
    o = oracle.OracleRaster(sc["means3D"], sc["opacities"], bg, view_m, proj_m, campos, tanfovx, tanfovy, H, W,
                            shs=shs if shs.size else None, sh_degree=sh_degree,
                            colors_precomp=colors if colors.size else None,
                            scales=sc["scales"] if use_scales else None,
                            rotations=sc["rotations"] if use_scales else None,
                            cov3D_precomp=None if use_scales else cov, scale_modifier=scale_modifier,
                            antialiasing=antialiasing, nthreads=1)
    g = o.backward(gc.float(), gi.float())
    out = dict(
        means3D=sc["means3D"], opacities=sc["opacities"], bg=bg, viewmatrix=view_m.numpy(),
        projmatrix=proj_m.numpy(), campos=campos.numpy(), tanfovx=np.float32(tanfovx),
        tanfovy=np.float32(tanfovy), H=np.int32(H), W=np.int32(W), shs=shs, sh_degree=np.int32(sh_degree),
        colors_precomp=colors, scales=sc["scales"] if use_scales else empty,
        rotations=sc["rotations"] if use_scales else empty, cov3D_precomp=empty if use_scales else cov,
        scale_modifier=np.float32(scale_modifier), antialiasing=np.bool_(antialiasing),
        grad_color=gc.numpy(), grad_invdepth=gi.numpy(),
        num_rendered=np.int64(o.num_rendered), radii=o.radii, keys=o.get("keys"), vals=o.get("vals"),
        ranges=o.get("ranges"), color=o.color, invdepth=o.invdepth, final_T=o.get("final_T"),
        n_contrib=o.get("n_contrib"), means2D=o.get("means2D"), conic_opacity=o.get("conic_opacity"),
        depths=o.get("depths"),
        ref_rgb=ref_rgb(sc["means3D"], sc["shs"], campos, sh_degree) if mode.startswith("sh") else empty,
        ref_cov3D=cov if use_scales else empty,
        **g)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(f"{name}: P={P} L={o.num_rendered} visible={(o.radii > 0).sum()}")


def main():
    torch.set_num_threads(1)
    cfg1 = {k: v.numpy() for k, v in synthetic.make_scene(1000, seed=0).items()}
    # BASELINE config 1 (1k Gaussians, 256x256, view 0), AA off / on
    make("config1_sh_scales_aa0", cfg1, 256, 256, 0)
    make("config1_sh_scales_aa1", cfg1, 256, 256, 0, antialiasing=True)
    # the other input modes of the boundary (colors_precomp / cov3D_precomp, rasterize_points.cu:35-56)
    make("config1_colors_cov3D_aa0", cfg1, 256, 256, 0, mode="colors_cov3D")
    make("config1_sh_cov3D_aa1", cfg1, 256, 256, 3, mode="sh_cov3D", antialiasing=True)
    # lower active SH degree than stored (training warm-up), coloured background, scale modifier,
    # non-square image whose width is not a tile multiple
    make("config1_deg1_bg_mod", cfg1, 200, 328, 5, sh_degree=1, bg=(0.2, 0.5, 1.0), scale_modifier=0.8)
    # the reference's own hand fixtures (GS-IRON/npu-1/*.ply)
    one = ply_scene(os.path.join(REF, "GS-IRON/npu-1/single_gaussian.ply"))
    two = ply_scene(os.path.join(REF, "GS-IRON/npu-1/two_gaussians.ply"))
    make("ply_single_gaussian_aa0", one, 96, 120, 0)
    make("ply_two_gaussians_aa1", two, 96, 120, 0, antialiasing=True)


if __name__ == "__main__":
    main()
