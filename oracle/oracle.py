"""ctypes front-end of the CPU oracle (gsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  Never imported by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libgsr_oracle.so")
_lib = None

_ITEMS = ["depths", "clamped", "radii", "means2D", "cov3D", "conic_opacity", "rgb", "tiles_touched",
          "point_offsets", "keys_unsorted", "vals_unsorted", "keys", "vals", "ranges", "final_T", "n_contrib"]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = ctypes.CDLL(_LIB)
        _lib.gsr_oracle_forward.restype = ctypes.c_void_p
        _lib.gsr_oracle_backward.restype = ctypes.c_int
        _lib.gsr_oracle_get.restype = ctypes.c_int
        _lib.gsr_oracle_free.restype = None
        _lib.gsr_oracle_last_error.restype = ctypes.c_char_p
        _lib.gsr_oracle_higher_msb.restype = ctypes.c_uint32
    return _lib


def _f(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def _p(a):
    return None if a is None or a.size == 0 else a.ctypes.data_as(ctypes.c_void_p)


def _np(t):
    if t is None:
        return None
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    return np.ascontiguousarray(t, dtype=np.float32)


class OracleRaster:
    """One forward (and optionally backward) of the oracle; mirrors Rasterizer::forward/backward."""

    def __init__(self, means3D, opacities, bg, viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W,
                 shs=None, sh_degree=0, colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
                 scale_modifier=1.0, prefiltered=False, antialiasing=False, nthreads=1, shared_exp=False):
        """shared_exp: the blend's exp() is gsr_ref_expf (gsr_ref_exp.h) instead of the host libm's
        expf, in the forward and in every later backward / near_threshold of this object -- the
        function the GSR_REF_ALPHA test build of the HIP render kernels evaluates (bit-exact parity
        of the blend, tests/test_ref_alpha_exact.py)."""
        L = lib()
        self.shared_exp = bool(shared_exp)
        self.args = dict(means3D=_np(means3D), opacities=_np(opacities), bg=_np(bg), view=_np(viewmatrix),
                         proj=_np(projmatrix), campos=_np(campos), shs=_np(shs), colors=_np(colors_precomp),
                         scales=_np(scales), rots=_np(rotations), cov3D=_np(cov3D_precomp))
        a = self.args
        self.P = P = a["means3D"].shape[0]
        self.H, self.W = H, W
        self.D = sh_degree
        self.M = 0 if a["shs"] is None or a["shs"].size == 0 else a["shs"].shape[1]
        self.scale_modifier, self.tanfovx, self.tanfovy = scale_modifier, tanfovx, tanfovy
        self.antialiasing, self.nthreads = antialiasing, nthreads
        self.color = np.zeros((3, H, W), np.float32)
        self.invdepth = np.zeros((1, H, W), np.float32)
        self.radii = np.zeros((P,), np.int32)
        nr = ctypes.c_int(0)
        L.gsr_oracle_set_shared_exp(ctypes.c_int(int(self.shared_exp)))
        self.h = L.gsr_oracle_forward(
            ctypes.c_int(P), ctypes.c_int(sh_degree), ctypes.c_int(self.M), _p(a["bg"]), ctypes.c_int(W),
            ctypes.c_int(H), _p(a["means3D"]), _p(a["shs"]), _p(a["colors"]), _p(a["opacities"]),
            _p(a["scales"]), ctypes.c_float(scale_modifier), _p(a["rots"]), _p(a["cov3D"]), _p(a["view"]),
            _p(a["proj"]), _p(a["campos"]), ctypes.c_float(tanfovx), ctypes.c_float(tanfovy),
            ctypes.c_int(int(prefiltered)), ctypes.c_int(int(antialiasing)), _p(self.color), _p(self.invdepth),
            _p(self.radii), ctypes.c_int(nthreads), ctypes.byref(nr))
        L.gsr_oracle_set_shared_exp(ctypes.c_int(0))
        if not self.h:
            raise RuntimeError(L.gsr_oracle_last_error().decode())
        self.num_rendered = nr.value
        self.tiles = L.gsr_oracle_num_tiles(ctypes.c_void_p(self.h))

    def get(self, name):
        P, Lr, N, T = self.P, self.num_rendered, self.H * self.W, self.tiles
        shapes = {"depths": ((P,), np.float32), "clamped": ((P,), np.uint8), "radii": ((P,), np.int32),
                  "means2D": ((P, 2), np.float32), "cov3D": ((P, 6), np.float32),
                  "conic_opacity": ((P, 4), np.float32), "rgb": ((P, 3), np.float32),
                  "tiles_touched": ((P,), np.uint32), "point_offsets": ((P,), np.uint32),
                  "keys_unsorted": ((Lr,), np.uint64), "vals_unsorted": ((Lr,), np.uint32),
                  "keys": ((Lr,), np.uint64), "vals": ((Lr,), np.uint32), "ranges": ((T, 2), np.uint32),
                  "final_T": ((N,), np.float32), "n_contrib": ((N,), np.uint32)}
        shape, dt = shapes[name]
        out = np.zeros(shape, dt)
        if out.size:
            lib().gsr_oracle_get(ctypes.c_void_p(self.h), ctypes.c_int(_ITEMS.index(name)),
                                 out.ctypes.data_as(ctypes.c_void_p))
        return out

    def backward(self, dL_dcolor, dL_dinvdepth=None, f64=False, tile_sums=False):
        """f64: the render backward's arithmetic in float64 (gsr_oracle_set_bwd_f64) -- the
        accuracy yardstick of tests/common.check_rel_truth, not the reference's float32 order.
        tile_sums: each pixel's float32 terms summed per tile list entry first, then per Gaussian
        (gsr_oracle_set_bwd_tile_sums) instead of one atomic add per term -- another order of the
        same terms, several times faster on dense scenes (the training tests' oracle loops)."""
        a = self.args
        P, M = self.P, self.M
        g = dict(dL_dmean2D=np.zeros((P, 3), np.float32), dL_dconic=np.zeros((P, 2, 2), np.float32),
                 dL_dopacity=np.zeros((P, 1), np.float32), dL_dcolors=np.zeros((P, 3), np.float32),
                 dL_dmeans3D=np.zeros((P, 3), np.float32), dL_dcov3D=np.zeros((P, 6), np.float32),
                 dL_dsh=np.zeros((P, M, 3), np.float32), dL_dscales=np.zeros((P, 3), np.float32),
                 dL_drotations=np.zeros((P, 4), np.float32))
        dc = _np(dL_dcolor)
        di = _np(dL_dinvdepth)
        lib().gsr_oracle_set_bwd_f64(ctypes.c_int(int(bool(f64))))
        lib().gsr_oracle_set_bwd_tile_sums(ctypes.c_int(int(bool(tile_sums))))
        lib().gsr_oracle_set_shared_exp(ctypes.c_int(int(self.shared_exp)))
        rc = lib().gsr_oracle_backward(
            ctypes.c_void_p(self.h), _p(a["bg"]), _p(a["means3D"]), _p(a["shs"]), _p(a["colors"]),
            _p(a["opacities"]), _p(a["scales"]), ctypes.c_float(self.scale_modifier), _p(a["rots"]),
            _p(a["cov3D"]), _p(a["view"]), _p(a["proj"]), _p(a["campos"]), ctypes.c_float(self.tanfovx),
            ctypes.c_float(self.tanfovy), _p(dc), _p(di), _p(g["dL_dmean2D"]), _p(g["dL_dconic"]),
            _p(g["dL_dopacity"]), _p(g["dL_dcolors"]), _p(g["dL_dmeans3D"]), _p(g["dL_dcov3D"]),
            _p(g["dL_dsh"]) if M else None, _p(g["dL_dscales"]), _p(g["dL_drotations"]),
            ctypes.c_int(self.nthreads))
        lib().gsr_oracle_set_bwd_f64(ctypes.c_int(0))
        lib().gsr_oracle_set_bwd_tile_sums(ctypes.c_int(0))
        lib().gsr_oracle_set_shared_exp(ctypes.c_int(0))
        if rc != 0:
            raise RuntimeError("oracle backward failed")
        return g

    def near_threshold(self, rel=1e-5, gaussians=False):
        """bool (H, W): pixels whose walk takes a blend decision within `rel` of its threshold
        (gsr_oracle_near_threshold) -- candidates for a decision the GPU's float32 order takes the
        other way below the image tolerance; with gaussians=True also bool (P,): the Gaussians
        whose decisions those are.  Test infrastructure."""
        out = np.zeros((self.H, self.W), np.uint8)
        g = np.zeros((max(self.P, 1),), np.uint8)
        if out.size:
            lib().gsr_oracle_set_shared_exp(ctypes.c_int(int(self.shared_exp)))
            lib().gsr_oracle_near_threshold(ctypes.c_void_p(self.h), ctypes.c_float(rel),
                                            out.ctypes.data_as(ctypes.c_void_p), g.ctypes.data_as(ctypes.c_void_p))
            lib().gsr_oracle_set_shared_exp(ctypes.c_int(0))
        return (out.astype(bool), g[:self.P].astype(bool)) if gaussians else out.astype(bool)

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib is not None:
                _lib.gsr_oracle_free(ctypes.c_void_p(self.h))
                self.h = None
        except Exception:
            pass


def mark_visible(means3D, viewmatrix, projmatrix):
    m = _np(means3D)
    out = np.zeros((m.shape[0],), np.uint8)
    lib().gsr_oracle_mark_visible(ctypes.c_int(m.shape[0]), _p(m), _p(_np(viewmatrix)), _p(_np(projmatrix)),
                                  out.ctypes.data_as(ctypes.c_void_p))
    return out.astype(bool)


def knn_dist2(points, nthreads=8):
    """simple-knn distCUDA2 restated (knn_oracle.c): mean squared distance to the 3 nearest others."""
    p = _np(points).reshape(-1, 3)
    out = np.zeros((p.shape[0],), np.float32)
    if p.shape[0]:
        lib().gsr_oracle_knn_dist2(ctypes.c_int(p.shape[0]), _p(p), out.ctypes.data_as(ctypes.c_void_p),
                                   ctypes.c_int(nthreads))
    return out


def higher_msb(n):
    return int(lib().gsr_oracle_higher_msb(ctypes.c_uint32(n)))
