"""`simple_knn._C.distCUDA2` over the C ABI of include/simple_knn.h.

distCUDA2(points) -> dist2: points is a float32 (P, 3) GPU tensor; dist2[i] is the mean of
the squared distances from point i to its 3 nearest other points (simple-knn's definition;
its one call site is scene/gaussian_model.py:159-160).  Runs on the tensor's device and
torch's current HIP stream.  Non-GPU input or a missing library raises: no CPU fallback.
"""
import ctypes

import torch

from diff_gaussian_rasterization import _C as _gsr

_lib = _gsr.lib
_lib.gsr_knn_workspace_size.restype = ctypes.c_size_t
_lib.gsr_knn_workspace_size.argtypes = [ctypes.c_int]
_lib.gsr_knn_dist2.restype = ctypes.c_int
_lib.gsr_knn_dist2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]


def distCUDA2(points):
    if points.device.type != "cuda":
        raise RuntimeError(f"distCUDA2 runs on the GPU only (HIP); got a tensor on {points.device}")
    if points.dim() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    pts = points.float().contiguous()
    P = pts.size(0)
    dist2 = torch.empty((P,), dtype=torch.float32, device=pts.device)
    if P == 0:
        return dist2
    with torch.cuda.device(pts.device):
        ws = torch.empty((_lib.gsr_knn_workspace_size(P),), dtype=torch.uint8, device=pts.device)
        stream = torch.cuda.current_stream(pts.device).cuda_stream
        _gsr._check(_lib.gsr_knn_dist2(P, pts.data_ptr(), dist2.data_ptr(), ws.data_ptr(), stream))
    return dist2
