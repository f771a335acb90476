"""Drop-in for the reference's optional `fused_ssim` module (submodule fused-ssim, un-vendored;
train.py:31-35 imports `from fused_ssim import fused_ssim` and uses it at train.py:121-124).

fused_ssim(img1, img2, padding="same", train=True) -> mean SSIM, differentiable w.r.t. img1,
with the semantics of the reference's PyTorch ssim (utils/loss_utils.py:56-86).  The map and its
gradient are computed by the HIP kernels behind include/fused_ssim.h; there is no CPU path.
"""
import ctypes

import torch

from diff_gaussian_rasterization import _C as _gsr

_lib = _gsr.lib
_vp, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_lib.gsr_ssim_forward.restype = _i
_lib.gsr_ssim_forward.argtypes = [_i, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
_lib.gsr_ssim_backward.restype = _i
_lib.gsr_ssim_backward.argtypes = [_i, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]

allowed_padding = ["same", "valid"]


def _planes(img):
    if img.device.type != "cuda":
        raise RuntimeError(f"fused_ssim runs on the GPU only (HIP); got a tensor on {img.device}")
    if img.dim() < 2:
        raise RuntimeError("images must be (..., H, W)")
    H, W = img.shape[-2], img.shape[-1]
    return (img.numel() // (H * W) if H * W else 0), H, W


def _f32(t):
    return t.detach().float().contiguous()


def fusedssim(C1, C2, img1, img2, train=True):
    """(ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12); the last three are empty if not train."""
    if img1.shape != img2.shape:
        raise RuntimeError("img1 and img2 must have the same shape")
    n, H, W = _planes(img1)
    a, b = _f32(img1), _f32(img2)
    out = torch.empty_like(a)
    parts = [torch.empty_like(a) for _ in range(3)] if train else [torch.empty(0, device=a.device)] * 3
    ptr = [p.data_ptr() if train else None for p in parts]
    with torch.cuda.device(a.device):
        stream = torch.cuda.current_stream(a.device).cuda_stream
        _gsr._check(_lib.gsr_ssim_forward(n, H, W, C1, C2, a.data_ptr(), b.data_ptr(), out.data_ptr(), ptr[0],
                                          ptr[1], ptr[2], stream))
    return (out, *parts)


def fusedssim_backward(C1, C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12):
    n, H, W = _planes(img1)
    a, b, g = _f32(img1), _f32(img2), _f32(dL_dmap)
    grad = torch.empty_like(a)
    with torch.cuda.device(a.device):
        stream = torch.cuda.current_stream(a.device).cuda_stream
        _gsr._check(_lib.gsr_ssim_backward(n, H, W, C1, C2, a.data_ptr(), b.data_ptr(), g.data_ptr(),
                                           dm_dmu1.data_ptr(), dm_dsigma1_sq.data_ptr(), dm_dsigma12.data_ptr(),
                                           grad.data_ptr(), stream))
    return grad


class FusedSSIMMap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, C1, C2, img1, img2, padding="same", train=True):
        ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = fusedssim(C1, C2, img1, img2, train)
        if padding == "valid":
            ssim_map = ssim_map[..., 5:-5, 5:-5]
        ctx.save_for_backward(img1.detach(), img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        ctx.C1, ctx.C2, ctx.padding, ctx.train = C1, C2, padding, train
        return ssim_map

    @staticmethod
    def backward(ctx, opt_grad):
        img1, img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = ctx.saved_tensors
        if not ctx.train:
            raise RuntimeError("fused_ssim(train=False) keeps no state for a backward pass")
        dL_dmap = opt_grad
        if ctx.padding == "valid":
            dL_dmap = torch.zeros_like(img1)
            dL_dmap[..., 5:-5, 5:-5] = opt_grad
        grad = fusedssim_backward(ctx.C1, ctx.C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        return None, None, grad.to(img1.dtype), None, None, None


def fused_ssim(img1, img2, padding="same", train=True):
    C1 = 0.01 ** 2
    C2 = 0.03 ** 2
    assert padding in allowed_padding
    img1 = img1.contiguous()
    ssim_map = FusedSSIMMap.apply(C1, C2, img1, img2, padding, train)
    return ssim_map.mean()
