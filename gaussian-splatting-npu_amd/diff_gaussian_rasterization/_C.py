"""Host binding of libgsr_hip.so (include/gsr.h) behind the reference's `_C` op surface.

Mirrors the three ops the reference's torch glue exposes
(diff-gaussian-rasterization-npu/rasterize_points.cu:35-244, bound in ext.cpp:15-19):
``rasterize_gaussians``, ``rasterize_gaussians_backward`` and ``mark_visible`` -- same
argument order, same returned tuples, same shape errors.  PyTorch only provides device
memory and the current HIP stream; all compute runs in the HIP library.  There is no
CPU fallback: a missing library, a non-GPU tensor or a HIP failure raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgsr_hip.so")

_vp, _i, _f, _b, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_bool, ctypes.c_size_t


def _load(path=LIB_PATH):
    """The C ABI of the HIP library at `path` with its ctypes signatures.  The package loads only
    LIB_PATH; tests/test_ref_alpha_exact.py passes its test-only GSR_REF_ALPHA build here."""
    if not os.path.exists(path):
        raise ImportError(
            f"diff_gaussian_rasterization: native library {path} is missing; build it with "
            "`make -C gaussian-splatting-npu_amd` (or __graft_entry__.build()). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    lib.gsr_last_error.restype = ctypes.c_char_p
    lib.gsr_version.restype = ctypes.c_char_p
    for n in ("gsr_geometry_buffer_size", "gsr_binning_buffer_size"):
        getattr(lib, n).restype = _sz
        getattr(lib, n).argtypes = [_i]
    lib.gsr_image_buffer_size.restype = _sz
    lib.gsr_image_buffer_size.argtypes = [_i, _i]
    lib.gsr_mark_visible.argtypes = [_i, _vp, _vp, _vp, _vp, _vp]
    lib.gsr_forward_geometry.argtypes = [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp,
                                         _vp, _vp, _f, _f, _b, _b, _vp, _b, _vp, ctypes.POINTER(_i)]
    lib.gsr_forward_render.argtypes = [_vp, _vp, _vp, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _b, _vp]
    lib.gsr_forward_prealloc.argtypes = [_vp, _vp, _vp, _sz, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _vp,
                                         _vp, _vp, _vp, _vp, _f, _f, _b, _b, _vp, _vp, _vp, _b, _vp,
                                         ctypes.POINTER(_i), ctypes.POINTER(_i)]
    lib.gsr_backward.argtypes = [_i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp,
                                 _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                 _vp, _b, _b, _vp]
    lib.gsr_forward_prealloc_dc.argtypes = [_vp, _vp, _vp, _sz, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _f, _vp, _vp, _vp, _vp, _vp, _f, _f, _b, _b, _vp, _vp, _vp, _b, _vp,
                                            ctypes.POINTER(_i), ctypes.POINTER(_i)]
    lib.gsr_backward_dc.argtypes = [_i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp,
                                    _vp, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _b, _b, _vp]
    lib.gsr_backward_dc_acc.argtypes = lib.gsr_backward_dc.argtypes[:-1] + [ctypes.c_uint, _vp]
    lib.gsr_backward_views.argtypes = [_i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp,
                                       _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _vp, _vp, _vp, _b, _b, ctypes.c_uint, _vp]
    lib.gsr_backward_render.argtypes = [_i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _b, _vp]
    lib.gsr_backward_preprocess_views.argtypes = [_i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _f,
                                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _b, _vp, _vp,
                                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _b, _b, ctypes.c_uint, _vp]
    lib.gsr_backward_preprocess_views_range.argtypes = lib.gsr_backward_preprocess_views.argtypes[:-1] + [_i, _i, _vp]
    lib.gsr_backward_render_views.argtypes = [_i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _b, _vp]
    lib.gsr_forward_views.argtypes = [_i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp,
                                      _vp, _vp, _vp, _vp, _b, _b, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _b, _vp, _vp,
                                      _vp]
    lib.gsr_adam_update.argtypes = [_vp, _vp, _vp, _vp, _vp, _f, _f, _f, _f, _i, _i, _vp]
    lib.gsr_adam_update_multi.argtypes = [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _vp]
    lib.gsr_debug_sorted_keys.argtypes = [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp]
    lib.gsr_debug_depth_sort_workspace_size.argtypes = [_i]
    lib.gsr_debug_depth_sort_workspace_size.restype = _sz
    lib.gsr_debug_depth_sort.argtypes = [_vp, _i, _vp, _vp, _vp]
    if hasattr(lib, "gsr_debug_set_depth_wide"):  # (test hooks; absent from libraries built before them)
        lib.gsr_debug_depth_wide.argtypes = []
        lib.gsr_debug_set_depth_wide.argtypes = [_i]
    if hasattr(lib, "gsr_debug_last_depth_passes"):
        lib.gsr_debug_last_depth_passes.argtypes = [_i]
    for n in ("gsr_geometry_layout", "gsr_binning_layout"):
        getattr(lib, n).argtypes = [_i, ctypes.POINTER(_sz), _i]
    lib.gsr_image_layout.argtypes = [_i, _i, ctypes.POINTER(_sz), _i]
    return lib


lib = _load()


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"diff_gaussian_rasterization (HIP): {lib.gsr_last_error().decode()} [status {rc}]")


_contig_cache = {}  # small non-contiguous inputs (the transposed view matrices) -> contiguous copy
# Per device: the last forward's num_rendered.  The next forward pre-allocates its binning buffer
# from it (+25 % and 64K instances of headroom), so the native forward can run emission, sorts and
# render straight after the num_rendered read-back instead of returning to Python to allocate
# (the reference's binningBuffer resize lambda, rasterize_points.cu:27-33, rasterizer_impl.cu:286).
_binning_hint = {}
_binning_hint_views = {}  # per device: the last view batch's num_rendered per view
views_reruns = 0  # batched forwards that outgrew their binning buffers and ran a second time


def _contiguous(t):
    """t.contiguous(), memoised for small tensors: the reference's camera matrices are
    transposed views (scene/cameras.py:86-88) that every call would otherwise copy with a
    separate kernel launch.  Keyed on storage, layout and the in-place version counter."""
    if t.is_contiguous():
        return t
    if t.numel() > 64:
        return t.contiguous()
    key = (t.data_ptr(), t.shape, t.stride(), t._version, t.device)
    hit = _contig_cache.get(key)
    if hit is None:
        if len(_contig_cache) > 256:
            _contig_cache.clear()
        # the entry keeps `t` alive, so its storage cannot be recycled under the same key
        hit = _contig_cache[key] = (t, t.contiguous())
    return hit[1]


def _ptr(t, name, device):
    """Device pointer of a float32 tensor, or None for an absent (empty) input -- the
    reference passes `.data<float>()` of `torch.Tensor([])`, i.e. nullptr."""
    if t is None or t.numel() == 0:
        return None, None
    if t.device != device:
        raise RuntimeError(f"{name} must be on {device}, got {t.device}")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32, got {t.dtype}")
    t = _contiguous(t)
    return t.data_ptr(), t


def _stream(device):
    return torch.cuda.current_stream(device).cuda_stream


def _require_gpu(t):
    if t.device.type != "cuda":
        raise RuntimeError("diff_gaussian_rasterization runs on the GPU only (HIP); got a tensor on "
                           f"{t.device}. There is no CPU path.")


def _sh_split(sh, dc):
    """(M, has_dc): M = sh.size(1) -- with dc, the number of REST coefficients (0 if sh is empty)."""
    M = sh.size(1) if sh is not None and sh.numel() != 0 and sh.size(0) != 0 else 0
    has_dc = dc is not None and dc.numel() != 0
    return M, has_dc


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, antialiasing, debug, dc=None, out=None):
    """RasterizeGaussiansNPU (rasterize_points.cu:35-124).  `dc` (P,1,3): the separate-DC form of
    the accelerated upstream op (coefficient 0 apart from the rest in `sh`), selected by train.py
    together with SparseGaussianAdam (train.py:37-41, gaussian_renderer/__init__.py:82-100).
    `out` (color (3,H,W), radii (P,), invdepth (1,H,W)): caller-provided outputs, e.g. slices of a
    multi-view batch (MultiViewRasterizer) -- written in full."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _require_gpu(means3D)
    dev = means3D.device
    P, H, W = means3D.size(0), int(image_height), int(image_width)
    empty = lambda: torch.empty((0,), dtype=torch.uint8, device=dev)  # noqa: E731
    if P == 0:
        radii = torch.zeros((P,), dtype=torch.int32, device=dev)
        out_invdepth = torch.zeros((1, H, W), dtype=torch.float32, device=dev)
        out_color = torch.zeros((3, H, W), dtype=torch.float32, device=dev)
        return 0, out_color, radii, empty(), empty(), empty(), out_invdepth

    # every element of these is written by the HIP forward (radii by preprocess, pixels by render)
    if out is not None:
        out_color, radii, out_invdepth = out
        for t, shape, dt in ((out_color, (3, H, W), torch.float32), (radii, (P,), torch.int32),
                             (out_invdepth, (1, H, W), torch.float32)):
            if tuple(t.shape) != shape or t.dtype != dt or t.device != dev or not t.is_contiguous():
                raise RuntimeError(f"out: expected a contiguous {dt} tensor of shape {shape} on {dev}")
    else:
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        out_invdepth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
        out_color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
    M, has_dc = _sh_split(sh, dc)
    if has_dc and (dc.dim() != 3 or dc.size(0) != P or dc.size(1) != 1 or dc.size(2) != 3):
        raise RuntimeError("dc must have dimensions (num_points, 1, 3)")
    keep = []

    def p(t, name):
        ptr, tt = _ptr(t, name, dev)
        keep.append(tt)
        return ptr

    geom = torch.empty((lib.gsr_geometry_buffer_size(P),), dtype=torch.uint8, device=dev)
    img = torch.empty((lib.gsr_image_buffer_size(W, H),), dtype=torch.uint8, device=dev)
    stream = _stream(dev)
    nr = ctypes.c_int(0)
    rendered = ctypes.c_int(0)
    hint = _binning_hint.get(dev)
    cap = lib.gsr_binning_buffer_size(min(int(hint * 1.25) + 65536, 0x7FFFFFFF)) if hint is not None else 0
    binning = torch.empty((cap,), dtype=torch.uint8, device=dev) if cap else None
    bg_p, means_p = p(background, "bg"), p(means3D, "means3D")
    colors_p, op_p = p(colors, "colors_precomp"), p(opacity, "opacities")
    sc_p, rot_p, cov_p = p(scales, "scales"), p(rotations, "rotations"), p(cov3D_precomp, "cov3D_precomp")
    vm_p, pm_p = p(viewmatrix, "viewmatrix"), p(projmatrix, "projmatrix")
    sh_p, cam_p = p(sh, "sh"), p(campos, "campos")
    dc_p = p(dc, "dc") if has_dc else None
    _check(lib.gsr_forward_prealloc_dc(
        geom.data_ptr(), img.data_ptr(), binning.data_ptr() if cap else None, cap, P, int(degree), M, bg_p, W, H,
        means_p, dc_p, sh_p, colors_p, op_p, sc_p, float(scale_modifier), rot_p, cov_p, vm_p, pm_p, cam_p,
        float(tan_fovx), float(tan_fovy), bool(prefiltered), bool(antialiasing), out_color.data_ptr(),
        out_invdepth.data_ptr(), radii.data_ptr(), bool(debug), stream, ctypes.byref(nr), ctypes.byref(rendered)))
    L = nr.value
    _binning_hint[dev] = L
    need = lib.gsr_binning_buffer_size(L)
    if rendered.value:
        binning = binning[:need]  # a view: the backward re-derives the layout from num_rendered
    else:  # first call on this device, or the scene grew past the headroom
        binning = torch.empty((need,), dtype=torch.uint8, device=dev)
        _check(lib.gsr_forward_render(geom.data_ptr(), binning.data_ptr(), img.data_ptr(), P, L, bg_p, W, H,
                                      colors_p, out_color.data_ptr(), out_invdepth.data_ptr(), radii.data_ptr(),
                                      bool(debug), stream))
    return L, out_color, radii, geom, binning, img, out_invdepth


def rasterize_gaussians_views(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                              cov3D_precomp, viewmatrices, projmatrices, tan_fovx, tan_fovy, image_height,
                              image_width, sh, degree, campos, prefiltered, antialiasing, debug, dc=None, out=None):
    """rasterize_gaussians over a batch of V views of the same Gaussians (gsr_forward_views: every
    stage of the views' binning prefix and their render as one launch per stage, grid.y = view).  Per-view lists of camera
    arguments; `out` = (colors (V,3,H,W), radii (V,P), invdepths (V,1,H,W)) -- written in full.
    Returns per-view lists (num_rendered, geomBuffer, binningBuffer, imageBuffer); each view's
    results are bit-identical to rasterize_gaussians on that view."""
    _require_gpu(means3D)
    dev = means3D.device
    P, H, W = means3D.size(0), int(image_height), int(image_width)
    V = len(viewmatrices)
    colors_out, radii_out, inv_out = out
    for t, shape, dt in ((colors_out, (V, 3, H, W), torch.float32), (radii_out, (V, P), torch.int32),
                         (inv_out, (V, 1, H, W), torch.float32)):
        if tuple(t.shape) != shape or t.dtype != dt or t.device != dev or not t.is_contiguous():
            raise RuntimeError(f"out: expected a contiguous {dt} tensor of shape {shape} on {dev}")
    if P == 0:
        colors_out.zero_()
        radii_out.zero_()
        inv_out.zero_()
        e = torch.empty((0,), dtype=torch.uint8, device=dev)
        return [0] * V, [e] * V, [e] * V, [e] * V
    M, has_dc = _sh_split(sh, dc)
    if has_dc and (dc.dim() != 3 or dc.size(0) != P or dc.size(1) != 1 or dc.size(2) != 3):
        raise RuntimeError("dc must have dimensions (num_points, 1, 3)")
    keep = []

    def p(t, name):
        ptr, tt = _ptr(t, name, dev)
        keep.append(tt)
        return ptr

    def cont(ts, name):
        res = []
        for t in ts:
            _, tt = _ptr(t, name, dev)
            keep.append(tt)
            res.append(tt)
        return res

    gsz, isz = lib.gsr_geometry_buffer_size(P), lib.gsr_image_buffer_size(W, H)
    geoms = [torch.empty((gsz,), dtype=torch.uint8, device=dev) for _ in range(V)]
    imgs = [torch.empty((isz,), dtype=torch.uint8, device=dev) for _ in range(V)]
    # every view's capacity from the LARGEST num_rendered of the previous batch on this device (+25 %
    # and 64K instances): the hint is not keyed by camera, and a training loop deals different
    # cameras to the batch's slots every step, so a per-slot hint would overflow (and rerun the
    # whole batch) whenever a slot's new view renders more than its old one did
    hints = _binning_hint_views.get(dev)
    h = max(hints) if hints else _binning_hint.get(dev)
    caps = [lib.gsr_binning_buffer_size(min(int(h * 1.25) + 65536, 0x7FFFFFFF))] * V if h is not None else [0] * V
    bins = [torch.empty((c,), dtype=torch.uint8, device=dev) if c else None for c in caps]
    bg_p, means_p = p(background, "bg"), p(means3D, "means3D")
    colors_p, op_p = p(colors, "colors_precomp"), p(opacity, "opacities")
    sc_p, rot_p, cov_p = p(scales, "scales"), p(rotations, "rotations"), p(cov3D_precomp, "cov3D_precomp")
    sh_p = p(sh, "sh")
    dc_p = p(dc, "dc") if has_dc else None
    views, projs, cams = cont(viewmatrices, "viewmatrix"), cont(projmatrices, "projmatrix"), cont(campos, "campos")
    stream = _stream(dev)
    nr = (_i * V)()
    rendered = (_i * V)()

    def run(caps):
        _check(lib.gsr_forward_views(
            V, P, int(degree), M, bg_p, W, H, means_p, dc_p, sh_p, colors_p, op_p, sc_p, float(scale_modifier), rot_p,
            cov_p, _ptr_array(views), _ptr_array(projs), _ptr_array(cams), (_f * V)(*[float(t) for t in tan_fovx]),
            (_f * V)(*[float(t) for t in tan_fovy]), bool(prefiltered), bool(antialiasing), _ptr_array(geoms),
            _ptr_array(imgs), _ptr_array(bins), (_sz * V)(*caps), _ptr_array([colors_out[v] for v in range(V)]),
            _ptr_array([inv_out[v] for v in range(V)]), _ptr_array([radii_out[v] for v in range(V)]), bool(debug),
            stream, nr, rendered))

    run(caps)
    Ls = [int(nr[v]) for v in range(V)]
    _binning_hint[dev] = max(Ls)
    _binning_hint_views[dev] = Ls
    if all(rendered[v] for v in range(V)):
        bins = [bins[v][:lib.gsr_binning_buffer_size(Ls[v])] for v in range(V)]  # views: the backward re-derives
    else:  # first call on this device, or the scene grew past the headroom: the batch again, exact buffers
        global views_reruns
        views_reruns += 1
        bins = [torch.empty((lib.gsr_binning_buffer_size(L),), dtype=torch.uint8, device=dev) for L in Ls]
        run([b.numel() for b in bins])
        if not all(rendered[v] for v in range(V)) or [int(nr[v]) for v in range(V)] != Ls:
            raise RuntimeError("diff_gaussian_rasterization (HIP): the repeated batch did not reproduce num_rendered")
    return Ls, geoms, bins, imgs


# accumulate= keys -> gsr.h GSR_ACC_* bits
ACC_BITS = {"means3D": 1, "dc": 2, "sh": 4, "opacities": 8, "scales": 16, "rotations": 32, "cov3D_precomp": 64,
            "colors_precomp": 128}


def rasterize_gaussians_backward(background, means3D, radii, colors, opacities, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color,
                                 dL_dout_invdepth, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                                 antialiasing, debug, dc=None, accumulate=None):
    """RasterizeGaussiansBackwardNPU (rasterize_points.cu:126-223).  With `dc` (the separate-DC
    form) the result carries dL_ddc (P,1,3) before dL_dsh, as the accelerated upstream op returns
    it: (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_ddc, dL_dsh, dL_dscales,
    dL_drotations).

    accumulate: optional {ACC_BITS key: tensor} -- the kernel ADDS that input's gradient into the
    given contiguous float32 tensor of the input's size (gsr_backward_dc_acc) and the result holds
    None in its place."""
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    M, has_dc = _sh_split(sh, dc)
    # Render-pass gradients (one allocation): mean2D 3 | colors 3 | conic 4 | invdepth 1.
    # The HIP backward writes every element (no atomics, no pre-zeroing needed).
    rbuf = torch.empty((P * 11,), dtype=torch.float32, device=dev)
    dL_dmeans2D = rbuf[0:3 * P].view(P, 3)
    dL_dcolors = rbuf[3 * P:6 * P].view(P, 3)
    dL_dconic = rbuf[6 * P:10 * P].view(P, 2, 2)
    has_inv = dL_dout_invdepth is not None and dL_dout_invdepth.numel() != 0 and dL_dout_invdepth.size(0) != 0
    dL_dinvdepths = rbuf[10 * P:11 * P].view(P, 1)
    # Parameter gradients, fully written by the HIP kernel (zeros for culled Gaussians), in ONE
    # buffer laid out as multiview.PARAM_ORDER (means3D | sh | opacity | scales | rotations) then
    # cov3D: autograd keeps these views as the leaves' .grad, so a multi-GPU step all-reduces the
    # buffer in place instead of gathering and scattering 236 B per Gaussian around the collective.
    # With dc, its gradient sits between means3D and the rest (multiview.PARAM_ORDER_DC).
    acc = dict(accumulate or {})
    for k, t in acc.items():
        n = {"means3D": 3 * P, "dc": 3 * P, "sh": 3 * M * P, "opacities": P, "scales": 3 * P, "rotations": 4 * P,
             "cov3D_precomp": 6 * P, "colors_precomp": 3 * P}.get(k)
        if n is None:
            raise RuntimeError(f"accumulate: unknown gradient {k!r}")
        if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != n:
            raise RuntimeError(f"accumulate[{k!r}] must be a contiguous float32 tensor of {n} elements on {dev}")
    if "dc" in acc and not has_dc:
        raise RuntimeError("accumulate['dc'] given without dc")
    sizes = [0 if "means3D" in acc else 3 * P, 3 * P if has_dc and "dc" not in acc else 0,
             0 if "sh" in acc else 3 * M * P, 0 if "opacities" in acc else P, 0 if "scales" in acc else 3 * P,
             0 if "rotations" in acc else 4 * P, 0 if "cov3D_precomp" in acc else 6 * P]
    parts = torch.split(torch.empty((sum(sizes),), dtype=torch.float32, device=dev), sizes)
    dL_dmeans3D = acc.get("means3D", parts[0]).view(P, 3)
    dL_ddc = acc.get("dc", parts[1]).view(P, 1, 3) if has_dc else None
    dL_dsh = acc.get("sh", parts[2]).view(P, M, 3)
    dL_dopacity = acc.get("opacities", parts[3]).view(P, 1)
    dL_dscales = acc.get("scales", parts[4]).view(P, 3)
    dL_drotations = acc.get("rotations", parts[5]).view(P, 4)
    dL_dcov3D = acc.get("cov3D_precomp", parts[6]).view(P, 6)
    if "colors_precomp" in acc:
        dL_dcolors = acc["colors_precomp"].view(P, 3)

    def result():
        r = {"means3D": dL_dmeans3D, "dc": dL_ddc, "sh": dL_dsh, "opacities": dL_dopacity, "scales": dL_dscales,
             "rotations": dL_drotations, "cov3D_precomp": dL_dcov3D, "colors_precomp": dL_dcolors}
        r = {k: (None if k in acc else v) for k, v in r.items()}
        if has_dc:
            return (dL_dmeans2D, r["colors_precomp"], r["opacities"], r["means3D"], r["cov3D_precomp"], r["dc"],
                    r["sh"], r["scales"], r["rotations"])
        return (dL_dmeans2D, r["colors_precomp"], r["opacities"], r["means3D"], r["cov3D_precomp"], r["sh"],
                r["scales"], r["rotations"])

    if P == 0:
        return result()

    keep = []

    def p(t, name):
        ptr, tt = _ptr(t, name, dev)
        keep.append(tt)
        return ptr

    dpix = p(dL_dout_color, "dL_dout_color")
    dinv = p(dL_dout_invdepth, "dL_dout_invdepth") if has_inv else None
    mask = 0
    for k in acc:
        mask |= ACC_BITS[k]
    _check(lib.gsr_backward_dc_acc(
        P, int(degree), M, int(R), p(background, "bg"), W, H, p(means3D, "means3D"),
        p(dc, "dc") if has_dc else None, p(sh, "sh"),
        p(colors, "colors_precomp"), p(opacities, "opacities"), p(scales, "scales"), float(scale_modifier),
        p(rotations, "rotations"), p(cov3D_precomp, "cov3D_precomp"), p(viewmatrix, "viewmatrix"),
        p(projmatrix, "projmatrix"), p(campos, "campos"), float(tan_fovx), float(tan_fovy), radii.data_ptr(),
        geomBuffer.data_ptr(), binningBuffer.data_ptr() if binningBuffer.numel() else None, imageBuffer.data_ptr(),
        dpix, dinv, dL_dmeans2D.data_ptr(), dL_dconic.data_ptr(), dL_dopacity.data_ptr(), dL_dcolors.data_ptr(),
        dL_dinvdepths.data_ptr() if has_inv else None, dL_dmeans3D.data_ptr(), dL_dcov3D.data_ptr(),
        dL_ddc.data_ptr() if has_dc else None, dL_dsh.data_ptr() if M else None, dL_dscales.data_ptr(),
        dL_drotations.data_ptr(), bool(antialiasing), bool(debug), mask, _stream(dev)))
    return result()


def _ptr_array(ts):
    return (_vp * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


def _views_grads(P, M, V, has_dc, accumulate, dev):
    """Outputs of a multi-view backward: (V,P,3) screen-space gradients and the summed parameter
    gradients (fresh buffers, or the caller's `accumulate` targets), plus the GSR_ACC_* mask."""
    acc = dict(accumulate or {})
    for k, t in acc.items():
        n = {"means3D": 3 * P, "dc": 3 * P, "sh": 3 * M * P, "opacities": P, "scales": 3 * P, "rotations": 4 * P,
             "cov3D_precomp": 6 * P, "colors_precomp": 3 * P}.get(k)
        if n is None:
            raise RuntimeError(f"accumulate: unknown gradient {k!r}")
        if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != n:
            raise RuntimeError(f"accumulate[{k!r}] must be a contiguous float32 tensor of {n} elements on {dev}")
    dL_dmeans2D = torch.empty((V, P, 3), dtype=torch.float32, device=dev)
    sizes = [0 if "means3D" in acc else 3 * P, 3 * P if has_dc and "dc" not in acc else 0,
             0 if "sh" in acc else 3 * M * P, 0 if "opacities" in acc else P, 0 if "scales" in acc else 3 * P,
             0 if "rotations" in acc else 4 * P, 0 if "cov3D_precomp" in acc else 6 * P,
             0 if "colors_precomp" in acc else 3 * P]
    parts = torch.split(torch.empty((sum(sizes),), dtype=torch.float32, device=dev), sizes)
    r = {"means3D": acc.get("means3D", parts[0]).view(P, 3),
         "dc": acc.get("dc", parts[1]).view(P, 1, 3) if has_dc else None,
         "sh": acc.get("sh", parts[2]).view(P, M, 3), "opacities": acc.get("opacities", parts[3]).view(P, 1),
         "scales": acc.get("scales", parts[4]).view(P, 3), "rotations": acc.get("rotations", parts[5]).view(P, 4),
         "cov3D_precomp": acc.get("cov3D_precomp", parts[6]).view(P, 6),
         "colors_precomp": acc.get("colors_precomp", parts[7]).view(P, 3)}
    mask = 0
    for k in acc:
        mask |= ACC_BITS[k]
    return dL_dmeans2D, r, acc, mask


def _views_result(dL_dmeans2D, r, acc, has_dc):
    r = {k: (None if k in acc else v) for k, v in r.items()}
    if has_dc:
        return (dL_dmeans2D, r["colors_precomp"], r["opacities"], r["means3D"], r["cov3D_precomp"], r["dc"], r["sh"],
                r["scales"], r["rotations"])
    return (dL_dmeans2D, r["colors_precomp"], r["opacities"], r["means3D"], r["cov3D_precomp"], r["sh"],
            r["scales"], r["rotations"])


def _preprocess_views_chunks(on_chunk, V, P, degree, M, Rs, W, H, means_p, dc_p, sh_p, colors_p, op_p, sc_p,
                             scale_modifier, rot_p, cov_p, views, projs, cams, tan_fovx, tan_fovy, radii, geomBuffers,
                             binningBuffers, has_inv, dL_dmeans2D, r, has_dc, antialiasing, debug, mask, acc, dev):
    """gsr_backward_preprocess_views_range over `chunks` Gaussian ranges (multiples of 256, the
    batched kernel's workgroup width), fn(g0, g1, grads) after each."""
    chunks, fn = on_chunk
    step = max(256, -(-P // max(1, int(chunks)) // 256) * 256)
    grads = {k: t for k, t in r.items() if t is not None}
    for g0 in range(0, P, step):
        g1 = min(P, g0 + step)
        _check(lib.gsr_backward_preprocess_views_range(
            V, P, int(degree), M, (_i * V)(*[int(x) for x in Rs]), int(W), int(H), means_p, dc_p, sh_p, colors_p,
            op_p, sc_p, float(scale_modifier), rot_p, cov_p, _ptr_array(views), _ptr_array(projs), _ptr_array(cams),
            (_f * V)(*[float(x) for x in tan_fovx]), (_f * V)(*[float(x) for x in tan_fovy]), _ptr_array(radii),
            _ptr_array(geomBuffers), _ptr_array([b if b.numel() else None for b in binningBuffers]), bool(has_inv),
            _ptr_array([dL_dmeans2D[v] for v in range(V)]), r["colors_precomp"].data_ptr(),
            r["opacities"].data_ptr(), r["means3D"].data_ptr(), r["cov3D_precomp"].data_ptr(),
            r["dc"].data_ptr() if has_dc else None, r["sh"].data_ptr() if M else None, r["scales"].data_ptr(),
            r["rotations"].data_ptr(), bool(antialiasing), bool(debug), mask, g0, g1, _stream(dev)))
        fn(g0, g1, grads)


def rasterize_gaussians_backward_views(background, means3D, radii, colors, opacities, scales, rotations,
                                       scale_modifier, cov3D_precomp, viewmatrices, projmatrices, tan_fovx, tan_fovy,
                                       dL_dout_colors, dL_dout_invdepths, sh, degree, campos, geomBuffers, Rs,
                                       binningBuffers, imageBuffers, antialiasing, debug, dc=None, accumulate=None,
                                       on_chunk=None):
    """Backward of a batch of V views (gsr_backward_views): per-view lists of the forward's state
    (radii (P,), camera, buffers, num_rendered) and dL_dout_colors (V,3,H,W), dL_dout_invdepths
    (V,1,H,W) or None.  Returns (dL_dmeans2D (V,P,3), dL_dcolors, dL_dopacity, dL_dmeans3D,
    dL_dcov3D, [dL_ddc,] dL_dsh, dL_dscales, dL_drotations): the screen-space gradient per view,
    everything else summed over the views; `accumulate` as in rasterize_gaussians_backward.
    on_chunk = (chunks, fn): the BACKWARD::preprocess runs as `chunks` launches over Gaussian ranges
    (gsr_backward_render_views, then gsr_backward_preprocess_views_range per range) and fn(g0, g1,
    grads) is called after each launch is enqueued, grads = {input name: its gradient tensor (P,...)}
    (the caller's accumulate targets or the fresh buffers): rows [g0, g1) are final from then on in
    stream order (multiview.overlapped_allreduce)."""
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    V = len(geomBuffers)
    H, W = dL_dout_colors.size(2), dL_dout_colors.size(3)
    M, has_dc = _sh_split(sh, dc)
    has_inv = dL_dout_invdepths is not None and dL_dout_invdepths.numel() != 0
    if dL_dout_colors.shape != (V, 3, H, W) or (has_inv and dL_dout_invdepths.shape != (V, 1, H, W)):
        raise RuntimeError("dL_dout_colors must be (V,3,H,W) and dL_dout_invdepths (V,1,H,W)")
    dL_dmeans2D, r, acc, mask = _views_grads(P, M, V, has_dc, accumulate, dev)
    keep = []

    def p(t, name):
        ptr, tt = _ptr(t, name, dev)
        keep.append(tt)
        return ptr

    def cont(ts, name):
        out = []
        for t in ts:
            ptr, tt = _ptr(t, name, dev)
            keep.append(tt)
            out.append(tt)
        return out

    views = cont(viewmatrices, "viewmatrix")
    projs = cont(projmatrices, "projmatrix")
    cams = cont(campos, "campos")
    dpix = [dL_dout_colors[v].contiguous() for v in range(V)]
    dinv = [dL_dout_invdepths[v].contiguous() for v in range(V)] if has_inv else None
    keep.extend(dpix)
    if on_chunk is not None:
        _check(lib.gsr_backward_render_views(
            V, P, (_i * V)(*[int(x) for x in Rs]), p(background, "bg"), W, H, _ptr_array(geomBuffers),
            _ptr_array([b if b.numel() else None for b in binningBuffers]), _ptr_array(imageBuffers),
            _ptr_array(dpix), _ptr_array(dinv) if has_inv else None, bool(debug), _stream(dev)))
        _preprocess_views_chunks(on_chunk, V, P, degree, M, Rs, W, H, p(means3D, "means3D"),
                                 p(dc, "dc") if has_dc else None, p(sh, "sh"), p(colors, "colors_precomp"),
                                 p(opacities, "opacities"), p(scales, "scales"), scale_modifier,
                                 p(rotations, "rotations"), p(cov3D_precomp, "cov3D_precomp"), views, projs, cams,
                                 tan_fovx, tan_fovy, radii, geomBuffers, binningBuffers, has_inv, dL_dmeans2D, r,
                                 has_dc, antialiasing, debug, mask, acc, dev)
        return _views_result(dL_dmeans2D, r, acc, has_dc)
    _check(lib.gsr_backward_views(
        V, P, int(degree), M, (_i * V)(*[int(x) for x in Rs]), p(background, "bg"), W, H, p(means3D, "means3D"),
        p(dc, "dc") if has_dc else None, p(sh, "sh"), p(colors, "colors_precomp"), p(opacities, "opacities"),
        p(scales, "scales"), float(scale_modifier), p(rotations, "rotations"), p(cov3D_precomp, "cov3D_precomp"),
        _ptr_array(views), _ptr_array(projs), _ptr_array(cams), (_f * V)(*[float(x) for x in tan_fovx]),
        (_f * V)(*[float(x) for x in tan_fovy]), _ptr_array(radii), _ptr_array(geomBuffers),
        _ptr_array([b if b.numel() else None for b in binningBuffers]), _ptr_array(imageBuffers),
        _ptr_array(dpix), _ptr_array(dinv) if has_inv else None, _ptr_array([dL_dmeans2D[v] for v in range(V)]),
        r["colors_precomp"].data_ptr(), r["opacities"].data_ptr(), r["means3D"].data_ptr(),
        r["cov3D_precomp"].data_ptr(), r["dc"].data_ptr() if has_dc else None, r["sh"].data_ptr() if M else None,
        r["scales"].data_ptr(), r["rotations"].data_ptr(), bool(antialiasing), bool(debug), mask, _stream(dev)))
    return _views_result(dL_dmeans2D, r, acc, has_dc)


def rasterize_gaussians_render_backward(background, P, R, geomBuffer, binningBuffer, imageBuffer, dL_dout_color,
                                        dL_dout_invdepth, debug):
    """BACKWARD::render of one view (gsr_backward_render): its per-(tile, Gaussian) gradient
    records into binningBuffer, for rasterize_gaussians_preprocess_backward_views later."""
    dev = dL_dout_color.device
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    has_inv = dL_dout_invdepth is not None and dL_dout_invdepth.numel() != 0
    bg_p, bg = _ptr(background, "bg", dev)
    dpix, dpix_t = _ptr(dL_dout_color, "dL_dout_color", dev)
    dinv, dinv_t = _ptr(dL_dout_invdepth, "dL_dout_invdepth", dev) if has_inv else (None, None)
    _check(lib.gsr_backward_render(int(P), int(R), bg_p, W, H, geomBuffer.data_ptr(),
                                   binningBuffer.data_ptr() if binningBuffer.numel() else None,
                                   imageBuffer.data_ptr(), dpix, dinv, bool(debug), _stream(dev)))
    return has_inv


def rasterize_gaussians_preprocess_backward_views(means3D, radii, colors, opacities, scales, rotations,
                                                  scale_modifier, cov3D_precomp, viewmatrices, projmatrices,
                                                  tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                                                  geomBuffers, Rs, binningBuffers, has_invdepth, antialiasing, debug,
                                                  dc=None, accumulate=None, on_chunk=None):
    """BACKWARD::preprocess of V views whose render backward already ran
    (gsr_backward_preprocess_views); returns what rasterize_gaussians_backward_views returns;
    on_chunk as there."""
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    V = len(geomBuffers)
    M, has_dc = _sh_split(sh, dc)
    dL_dmeans2D, r, acc, mask = _views_grads(P, M, V, has_dc, accumulate, dev)
    keep = []

    def p(t, name):
        ptr, tt = _ptr(t, name, dev)
        keep.append(tt)
        return ptr

    def cont(ts, name):
        out = []
        for t in ts:
            _, tt = _ptr(t, name, dev)
            keep.append(tt)
            out.append(tt)
        return out

    views, projs, cams = cont(viewmatrices, "viewmatrix"), cont(projmatrices, "projmatrix"), cont(campos, "campos")
    if on_chunk is not None:
        _preprocess_views_chunks(on_chunk, V, P, degree, M, Rs, image_width, image_height, p(means3D, "means3D"),
                                 p(dc, "dc") if has_dc else None, p(sh, "sh"), p(colors, "colors_precomp"),
                                 p(opacities, "opacities"), p(scales, "scales"), scale_modifier,
                                 p(rotations, "rotations"), p(cov3D_precomp, "cov3D_precomp"), views, projs, cams,
                                 tan_fovx, tan_fovy, radii, geomBuffers, binningBuffers, has_invdepth, dL_dmeans2D, r,
                                 has_dc, antialiasing, debug, mask, acc, dev)
        return _views_result(dL_dmeans2D, r, acc, has_dc)
    _check(lib.gsr_backward_preprocess_views(
        V, P, int(degree), M, (_i * V)(*[int(x) for x in Rs]), int(image_width), int(image_height),
        p(means3D, "means3D"), p(dc, "dc") if has_dc else None, p(sh, "sh"), p(colors, "colors_precomp"),
        p(opacities, "opacities"), p(scales, "scales"), float(scale_modifier), p(rotations, "rotations"),
        p(cov3D_precomp, "cov3D_precomp"), _ptr_array(views), _ptr_array(projs), _ptr_array(cams),
        (_f * V)(*[float(x) for x in tan_fovx]), (_f * V)(*[float(x) for x in tan_fovy]), _ptr_array(radii),
        _ptr_array(geomBuffers), _ptr_array([b if b.numel() else None for b in binningBuffers]), bool(has_invdepth),
        _ptr_array([dL_dmeans2D[v] for v in range(V)]), r["colors_precomp"].data_ptr(), r["opacities"].data_ptr(),
        r["means3D"].data_ptr(), r["cov3D_precomp"].data_ptr(), r["dc"].data_ptr() if has_dc else None,
        r["sh"].data_ptr() if M else None, r["scales"].data_ptr(), r["rotations"].data_ptr(), bool(antialiasing),
        bool(debug), mask, _stream(dev)))
    return _views_result(dL_dmeans2D, r, acc, has_dc)


def _adam_check(param, param_grad, exp_avg, exp_avg_sq, N, M, dev):
    for name, t in (("param", param), ("param_grad", param_grad), ("exp_avg", exp_avg), ("exp_avg_sq", exp_avg_sq)):
        if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"adamUpdate: {name} must be a contiguous float32 tensor on {dev}")
        if t.numel() != int(N) * int(M):
            raise RuntimeError(f"adamUpdate: {name} has {t.numel()} elements, expected N*M = {int(N) * int(M)}")


def adam_update_groups(groups, visible, b1, b2, N):
    """One launch for several (param, grad, exp_avg, exp_avg_sq, lr, eps) groups sharing the
    visibility mask of N Gaussians (SparseGaussianAdam.step); M = param.numel() // N per group."""
    if not groups:
        return
    dev = groups[0][0].device
    _require_gpu(groups[0][0])
    if visible.device != dev or visible.dtype != torch.bool or visible.numel() != int(N):
        raise RuntimeError(f"adamUpdate: visible must be a bool tensor of N = {int(N)} flags on {dev}")
    visible = visible.contiguous()
    n = len(groups)
    Ms = [g[0].numel() // int(N) if int(N) else 0 for g in groups]
    for (p, gr, m, v, _, _), M in zip(groups, Ms):
        _adam_check(p, gr, m, v, N, M, dev)
    ptrs = [(_vp * n)(*[g[k].data_ptr() for g in groups]) for k in range(4)]
    _check(lib.gsr_adam_update_multi(n, *ptrs, (_i * n)(*Ms), (_f * n)(*[float(g[4]) for g in groups]),
                                     (_f * n)(*[float(g[5]) for g in groups]), visible.data_ptr(), float(b1),
                                     float(b2), int(N), _stream(dev)))


def adamUpdate(param, param_grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M):
    """The accelerated upstream's `_C.adamUpdate` (called by SparseGaussianAdam.step): Adam on the
    rows of the N Gaussians with visible[i] set (M elements each), in place; no bias correction."""
    _require_gpu(param)
    dev = param.device
    _adam_check(param, param_grad, exp_avg, exp_avg_sq, N, M, dev)
    if visible.device != dev or visible.dtype != torch.bool or visible.numel() != int(N):
        raise RuntimeError(f"adamUpdate: visible must be a bool tensor of N = {int(N)} flags on {dev}")
    visible = visible.contiguous()
    _check(lib.gsr_adam_update(param.data_ptr(), param_grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                               visible.data_ptr(), float(lr), float(b1), float(b2), float(eps), int(N), int(M),
                               _stream(dev)))


def mark_visible(means3D, viewmatrix, projmatrix):
    """markVisible (rasterize_points.cu:225-244)."""
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    present = torch.zeros((P,), dtype=torch.bool, device=dev)
    if P != 0:
        m, mt = _ptr(means3D, "means3D", dev)
        v, vt = _ptr(viewmatrix, "viewmatrix", dev)
        pr, pt = _ptr(projmatrix, "projmatrix", dev)
        _check(lib.gsr_mark_visible(P, m, v, pr, present.data_ptr(), _stream(dev)))
    return present


# ---- parity/debug introspection (tests only) -------------------------------------------------
def _layout(fn, *args, n=64):
    offs = (_sz * n)()
    cnt = fn(*args, offs, n)
    return [offs[i] for i in range(cnt + 1)]


def geometry_layout(P):
    return _layout(lib.gsr_geometry_layout, P)


def image_layout(W, H):
    return _layout(lib.gsr_image_layout, W, H)


def binning_layout(L):
    return _layout(lib.gsr_binning_layout, L)


def sorted_keys(geomBuffer, binningBuffer, imgBuffer, P, L, W, H):
    """Sorted tile|depth keys, sorted Gaussian ids and per-tile ranges of the last forward."""
    dev = geomBuffer.device
    T = ((W + 15) // 16) * ((H + 15) // 16)
    keys = torch.empty((max(L, 0),), dtype=torch.int64, device=dev)
    vals = torch.empty((max(L, 0),), dtype=torch.int32, device=dev)
    ranges = torch.empty((T, 2), dtype=torch.int32, device=dev)
    _check(lib.gsr_debug_sorted_keys(geomBuffer.data_ptr(), binningBuffer.data_ptr() if L else None,
                                     imgBuffer.data_ptr(), P, L, W, H, keys.data_ptr() if L else None,
                                     vals.data_ptr() if L else None, ranges.data_ptr(), _stream(dev)))
    return keys, vals, ranges


def depth_sort(keys):
    """The forward's depth sort on its own (parity helper): the stable order of the u32 keys
    (int32 tensor of bit patterns; -1 = culled, sorted last)."""
    n = keys.numel()
    ids = torch.empty((n,), dtype=torch.int32, device=keys.device)
    if n == 0:
        return ids
    ws = torch.empty((lib.gsr_debug_depth_sort_workspace_size(n),), dtype=torch.uint8, device=keys.device)
    keys = keys.contiguous()
    _check(lib.gsr_debug_depth_sort(keys.data_ptr(), n, ids.data_ptr(), ws.data_ptr(),
                                    _stream(keys.device)))
    return ids


def depth_wide():
    """Test hook: True while this host thread's depth sorts are forced to four 8-bit passes
    (set_depth_wide).  Forwards never set it: a too-wide depth range re-runs that call's sort only."""
    return bool(lib.gsr_debug_depth_wide())


def set_depth_wide(on):
    """Test hook: force (True) or release (False) the four-pass depth sort for this host thread."""
    _check(lib.gsr_debug_set_depth_wide(1 if on else 0))


def grad_record_floats():
    """Floats per per-instance gradient record (GSR_GRAD_REC of the library build; diagnostics)."""
    return int(lib.gsr_debug_grad_record_floats())


def last_depth_passes(view=0):
    """Test hook: the passes of the final depth sort of view `view` in this thread's last forward (3,
    or 4 when its visible depth range was too wide for three and the sort was re-run)."""
    return int(lib.gsr_debug_last_depth_passes(int(view)))


def fusedssim(C1, C2, img1, img2):
    """The dr_aa extension's SSIM-map op that utils/loss_utils.py:17-30 imports: ssim_map."""
    import fused_ssim
    return fused_ssim.fusedssim(C1, C2, img1, img2, train=False)[0]


def fusedssim_backward(C1, C2, img1, img2, opt_grad):
    """dL/dimg1 of the SSIM map for upstream opt_grad (utils/loss_utils.py:32-37)."""
    import fused_ssim
    _, a, b, c = fused_ssim.fusedssim(C1, C2, img1, img2, train=True)
    return fused_ssim.fusedssim_backward(C1, C2, img1, img2, opt_grad, a, b, c)
