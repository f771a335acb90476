"""ctypes front-end of oracle/libgsr_cpu.so: the C oracle behind include/gsr.h's gsr_forward /
gsr_backward (gsr_cpu_abi.c), called with the product's argument lists -- resize callbacks for
the geometry / binning / image buffers, then the backward on them.

TEST INFRASTRUCTURE ONLY: used by tests/ and bench.py's cpu_baseline leg (the CPU baseline runs
the same host calling sequence as the HIP library).  Never imported by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libgsr_cpu.so")
_lib = None
_vp, _i, _f, _b = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_bool
RESIZE = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)  # gsr_resize_fn


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(["make", "-s", "-C", _HERE, "libgsr_cpu.so"])
        L = ctypes.CDLL(_LIB)
        L.gsr_last_error.restype = ctypes.c_char_p
        L.gsr_forward.argtypes = [RESIZE, _vp, RESIZE, _vp, RESIZE, _vp, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp,
                                  _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _f, _f, _b, _vp, _vp, _b, _vp, _b, _vp,
                                  ctypes.POINTER(_i)]
        L.gsr_backward.argtypes = [_i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp,
                                   _vp, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _b, _b, _vp]
        L.gsr_cpu_release.argtypes = [_vp]
        L.gsr_cpu_set_threads.argtypes = [_i]
        _lib = L
    return _lib


def _np(t):
    if t is None:
        return None
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    return np.ascontiguousarray(t, dtype=np.float32)


def _p(a):
    return None if a is None or a.size == 0 else a.ctypes.data


class CpuRasterizer:
    """One gsr_forward + gsr_backward of the C oracle through the C ABI (host arrays)."""

    def __init__(self, nthreads=1):
        self.L = lib()
        self.L.gsr_cpu_set_threads(int(nthreads))

    def forward_backward(self, means3D, opacities, bg, viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W,
                         dL_dcolor, dL_dinvdepth, shs=None, sh_degree=0, scales=None, rotations=None,
                         colors_precomp=None, cov3D_precomp=None, antialiasing=False, scale_modifier=1.0):
        L = self.L
        a = {k: _np(v) for k, v in dict(means3D=means3D, opacities=opacities, bg=bg, view=viewmatrix,
                                          proj=projmatrix, campos=campos, shs=shs, scales=scales, rots=rotations,
                                          colors=colors_precomp, cov3D=cov3D_precomp).items()}
        P = a["means3D"].shape[0]
        M = 0 if a["shs"] is None or a["shs"].size == 0 else a["shs"].shape[1]
        bufs = {}

        def resize(name):
            def fn(ctx, nbytes):
                bufs[name] = np.zeros(max(int(nbytes), 1), np.uint8)
                return bufs[name].ctypes.data
            return RESIZE(fn)
        cbs = [resize("geom"), resize("binning"), resize("img")]
        color = np.zeros((3, H, W), np.float32)
        inv = np.zeros((1, H, W), np.float32)
        radii = np.zeros((P,), np.int32)
        nr = _i(0)
        rc = L.gsr_forward(cbs[0], None, cbs[1], None, cbs[2], None, P, int(sh_degree), M, _p(a["bg"]), W, H,
                           _p(a["means3D"]), _p(a["shs"]), _p(a["colors"]), _p(a["opacities"]), _p(a["scales"]),
                           float(scale_modifier), _p(a["rots"]), _p(a["cov3D"]), _p(a["view"]), _p(a["proj"]),
                           _p(a["campos"]), float(tanfovx), float(tanfovy), False, color.ctypes.data,
                           inv.ctypes.data, bool(antialiasing), radii.ctypes.data, False, None, ctypes.byref(nr))
        if rc:
            raise RuntimeError(L.gsr_last_error().decode())
        g = {"dL_dmean2D": np.zeros((P, 3), np.float32), "dL_dconic": np.zeros((P, 2, 2), np.float32),
             "dL_dopacity": np.zeros((P, 1), np.float32), "dL_dcolors": np.zeros((P, 3), np.float32),
             "dL_dinvdepth": np.zeros((P, 1), np.float32), "dL_dmeans3D": np.zeros((P, 3), np.float32),
             "dL_dcov3D": np.zeros((P, 6), np.float32), "dL_dsh": np.zeros((P, max(M, 1), 3), np.float32),
             "dL_dscales": np.zeros((P, 3), np.float32), "dL_drotations": np.zeros((P, 4), np.float32)}
        dpix, dinv = _np(dL_dcolor), _np(dL_dinvdepth)
        try:
            rc = L.gsr_backward(P, int(sh_degree), M, nr.value, _p(a["bg"]), W, H, _p(a["means3D"]), _p(a["shs"]),
                                _p(a["colors"]), _p(a["opacities"]), _p(a["scales"]), float(scale_modifier),
                                _p(a["rots"]), _p(a["cov3D"]), _p(a["view"]), _p(a["proj"]), _p(a["campos"]),
                                float(tanfovx), float(tanfovy), radii.ctypes.data, bufs["geom"].ctypes.data,
                                bufs["binning"].ctypes.data, bufs["img"].ctypes.data, _p(dpix), _p(dinv),
                                *[g[k].ctypes.data for k in ("dL_dmean2D", "dL_dconic", "dL_dopacity", "dL_dcolors",
                                                             "dL_dinvdepth", "dL_dmeans3D", "dL_dcov3D", "dL_dsh",
                                                             "dL_dscales", "dL_drotations")],
                                bool(antialiasing), False, None)
            if rc:
                raise RuntimeError(L.gsr_last_error().decode())
        finally:
            L.gsr_cpu_release(bufs["geom"].ctypes.data)
        if M == 0:
            g["dL_dsh"] = g["dL_dsh"][:, :0]
        return nr.value, color, inv, radii, g
