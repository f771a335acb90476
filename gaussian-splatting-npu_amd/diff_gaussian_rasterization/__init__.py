"""MI355X-native drop-in for the reference's ``diff_gaussian_rasterization`` package.

Public surface kept verbatim from diff-gaussian-rasterization-npu/diff_gaussian_rasterization/
__init__.py: ``GaussianRasterizationSettings`` (:143-156), ``GaussianRasterizer`` (:158-207),
``rasterize_gaussians`` (:21-42) and the autograd function ``_RasterizeGaussians`` (:44-141), so
``gaussian_renderer/__init__.py`` (and therefore train.py / render.py) import and call it
unchanged.  It also carries the accelerated upstream surface that train.py switches to when the
package exports ``SparseGaussianAdam`` (train.py:37-41, 180-183): ``GaussianRasterizer.forward``
takes ``dc=`` (SH coefficient 0 apart from the rest, gaussian_renderer/__init__.py:82-100) and
``SparseGaussianAdam.step(visibility, N)`` updates only visible Gaussians
(scene/gaussian_model.py:194-196).  All compute is the HIP library behind ``_C`` (gfx950); there is
no CPU path.
"""
import contextlib
import threading
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "SparseGaussianAdam",
           "accumulate_grads_in_place"]

_state = threading.local()


@contextlib.contextmanager
def accumulate_grads_in_place(enabled=True):
    """Forwards run inside this context hand their backward an in-place accumulation: a
    rasterizer input that is a leaf tensor with an existing float32 ``.grad`` of its own shape
    gets this view's gradient ADDED to that ``.grad`` by the HIP backward kernel itself
    (gsr_backward_dc_acc: one fp32 add per element, the arithmetic of autograd's AccumulateGrad
    ``grad += new``), and the autograd function returns None for it -- instead of a fresh
    gradient tensor that autograd then adds with a separate pass over it.  A multi-view step
    (several views into one set of parameter gradients) saves that pass per view.
    Inputs without a ``.grad`` yet (a step's first view), non-leaf inputs (activations) and
    leaves with gradient hooks take the ordinary path.  Off by default: outside the context every
    call is exactly the reference's."""
    prev = getattr(_state, "accumulate", False)
    _state.accumulate = bool(enabled)
    try:
        yield
    finally:
        _state.accumulate = prev


def _accumulation_target(t):
    """t's existing .grad, if the backward may add into it in place."""
    if t is None or t.numel() == 0 or not t.requires_grad or not t.is_leaf or t._backward_hooks \
            or getattr(t, "_post_accumulate_grad_hooks", None):
        return None
    g = t.grad
    if g is None or g.dtype != torch.float32 or g.device != t.device or g.shape != t.shape or not g.is_contiguous():
        return None
    return g


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings, dc=None):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings, dc)


class _RasterizeGaussians(torch.autograd.Function):
    """Forward returns (color (3,H,W), radii int32 (P), invdepth (1,H,W)); backward returns the
    input gradients in input order, with d(means2D) = the screen-space gradient (P,3)
    that the caller's densification statistics read (scene/gaussian_model.py:471-473).  The last
    input, ``dc`` (None unless the separate-DC surface is used), gets its own gradient."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, dc=None):
        s = raster_settings
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer, invdepths = _C.rasterize_gaussians(
            s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered, s.antialiasing, s.debug, dc=dc)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        # in-place accumulation (accumulate_grads_in_place): the inputs whose .grad the backward
        # may add into, kept by reference (leaves: the same tensors save_for_backward keeps)
        ctx.acc_inputs = None
        if getattr(_state, "accumulate", False):
            ctx.acc_inputs = {"means3D": means3D, "dc": dc, "sh": sh, "opacities": opacities, "scales": scales,
                              "rotations": rotations, "cov3D_precomp": cov3Ds_precomp,
                              "colors_precomp": colors_precomp}
        # outputs without a gradient (always radii; invdepth when the loss ignores it) arrive as None
        # instead of zero tensors that autograd would fill with a kernel of its own; backward treats
        # None as zero
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities,
                              geomBuffer, binningBuffer, imgBuffer, dc)
        return color, radii, invdepths

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_out_depth):
        s = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, geomBuffer,
         binningBuffer, imgBuffer, dc) = ctx.saved_tensors
        if grad_out_color is None:
            grad_out_color = torch.zeros((3, s.image_height, s.image_width), dtype=torch.float32,
                                         device=means3D.device)
        if grad_out_depth is None:
            grad_out_depth = torch.Tensor([])  # no invdepth term (rasterize_points.cu:174-182 with zeros)
        accumulate = None
        if ctx.acc_inputs is not None:
            accumulate = {k: g for k, g in ((k, _accumulation_target(t)) for k, t in ctx.acc_inputs.items())
                          if g is not None}
            if "dc" in accumulate and (dc is None or dc.numel() == 0):
                del accumulate["dc"]
        grads = _C.rasterize_gaussians_backward(
            s.bg, means3D, radii, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, grad_out_depth, sh, s.sh_degree,
            s.campos, geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, s.antialiasing, s.debug, dc=dc,
            accumulate=accumulate)
        if len(grads) == 9:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_dc, grad_sh,
             grad_scales, grad_rotations) = grads
        else:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
             grad_scales, grad_rotations) = grads
            grad_dc = None
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                grad_rotations, grad_cov3Ds_precomp, None, grad_dc)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Frustum near-plane test (z_view > 0.2) per point, as a bool tensor, without autograd."""
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, dc=None):
        """``dc`` (P,1,3), keyword only in practice (gaussian_renderer/__init__.py:91-100): SH
        coefficient 0, with ``shs`` then holding coefficients 1.. (features_rest)."""
        s = self.raster_settings
        if (shs is None) == (colors_precomp is None) or (dc is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        absent = torch.Tensor([])
        return rasterize_gaussians(
            means3D, means2D,
            absent if shs is None else shs,
            absent if colors_precomp is None else colors_precomp,
            opacities,
            absent if scales is None else scales,
            absent if rotations is None else rotations,
            absent if cov3D_precomp is None else cov3D_precomp,
            s, dc)


class SparseGaussianAdam(torch.optim.Adam):
    """Adam that updates only the rows of visible Gaussians (train.py:180-183:
    ``optimizer.step(radii > 0, radii.shape[0])``; constructed as ``SparseGaussianAdam(l, lr=0.0,
    eps=1e-15)``, scene/gaussian_model.py:194-196).  One parameter tensor per group, as the
    caller's per-attribute groups are; state keeps torch.optim.Adam's keys (``exp_avg``,
    ``exp_avg_sq``, ``step``), so GaussianModel's densification surgery on ``optimizer.state``
    (gaussian_model.py:316-400) works unchanged.  The update is the published upstream one:
    betas fixed at (0.9, 0.999), no bias correction.  Where the upstream class launches
    ``_C.adamUpdate`` once per group, all groups of a step go in ONE HIP launch here
    (``_C.adam_update_groups``; per group the same update)."""

    def __init__(self, params, lr, eps):
        super().__init__(params=params, lr=lr, eps=eps)

    @torch.no_grad()
    def step(self, visibility, N):
        batch = []
        for group in self.param_groups:
            lr = group["lr"]
            eps = group["eps"]
            if len(group["params"]) != 1:
                raise AssertionError("more than one tensor in group")
            param = group["params"][0]
            if param.grad is None:
                continue
            state = self.state[param]
            if len(state) == 0:
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
            if param.numel() != (param.numel() // N) * N:
                raise RuntimeError(f"parameter of {param.numel()} elements is not N = {N} rows")
            batch.append((param, param.grad, state["exp_avg"], state["exp_avg_sq"], lr, eps))
        _C.adam_update_groups(batch, visibility, 0.9, 0.999, N)
