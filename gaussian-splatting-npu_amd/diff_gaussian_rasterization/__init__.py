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
           "accumulate_grads_in_place", "deferred_backward", "MultiViewRasterizer", "rasterize_views",
           "grad_chunk_hook"]

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


@contextlib.contextmanager
def grad_chunk_hook(chunks, fn, done):
    """Batched backward passes (MultiViewRasterizer, deferred_backward's flush) run inside this
    context split their BACKWARD::preprocess into `chunks` launches over Gaussian ranges and call
    fn(g0, g1, grads) after each (grads: {input name: the gradient tensor that input receives},
    rows [g0, g1) final in stream order), then done() before the backward returns -- the hook
    multiview.overlapped_allreduce uses to reduce each range while the next one computes.
    Process-wide, not per thread: autograd runs a CUDA backward on its own device thread."""
    global _grad_chunks
    prev = _grad_chunks
    _grad_chunks = (int(chunks), fn, done)
    try:
        yield
    finally:
        _grad_chunks = prev


_grad_chunks = None  # the active grad_chunk_hook (process-wide)


_hook_busy = threading.Lock()  # one hooked backward in flight at a time (collective order)


def _chunk_hook(wanted):
    """(on_chunk for _C, finish) from the active grad_chunk_hook, restricted to the gradients of
    the inputs in `wanted` (names); (None, None) outside the context.  finish() runs the hook's
    done() once -- the caller calls it in a `finally`, so a backward that fails after issuing
    collectives still waits for them -- and releases the hook for the next backward.  A second
    hooked backward while one is in flight (another thread or device of this process) would issue
    collectives in an order the other ranks do not match: it raises instead."""
    h = _grad_chunks
    if h is None or not wanted:
        return None, None
    chunks, fn, done = h
    if not _hook_busy.acquire(blocking=False):
        raise RuntimeError("grad_chunk_hook: a hooked batched backward is already in flight in this process; "
                           "concurrent hooked backward passes would issue collectives out of order across ranks")
    finished = []

    def on(g0, g1, grads):
        fn(g0, g1, {k: t for k, t in grads.items() if k in wanted and t.numel()})

    def finish():
        if finished:
            return
        finished.append(True)
        try:
            done()
        finally:
            _hook_busy.release()
    return (chunks, on), finish


# Per device: an event recorded after the last backward run inside accumulate_grads_in_place.
# Views rendered on different HIP streams (forward of one view overlapping the backward of the
# previous) add into the same .grad buffers; each in-place accumulating backward first makes its
# stream wait for this event, so the additions stay ordered.
_acc_fence = {}


def _accumulation_target(t):
    """t's existing .grad, if the backward may add into it in place."""
    if t is None or t.numel() == 0 or not t.requires_grad or not t.is_leaf or t._backward_hooks \
            or getattr(t, "_post_accumulate_grad_hooks", None):
        return None
    g = t.grad
    if g is None or g.dtype != torch.float32 or g.device != t.device or g.shape != t.shape or not g.is_contiguous():
        return None
    return g


class _DeferredBatch:
    """Views rendered inside deferred_backward: their render backward has run, their
    BACKWARD::preprocess waits for flush()."""

    def __init__(self):
        self.views = []
        self.closed = False
        self.lock = threading.Lock()

    def add(self, view):
        """Queue a view for the batched launch at the context's exit; a view whose backward runs
        after that exit (its forward was inside the context, its loss.backward() outside) gets its
        BACKWARD::preprocess right away, alone, so its gradients are never dropped."""
        with self.lock:
            if not self.closed:
                self.views.append(view)
                return
        self._launch([view])

    def flush(self):
        with self.lock:
            views, self.views = self.views, []
            self.closed = True
        # views share one set of Gaussian inputs and image/flag settings per batched launch
        groups = []
        for v in views:
            key = v["key"]
            if groups and groups[-1][0] == key and len(groups[-1][1]) < 16:
                groups[-1][1].append(v)
            else:
                groups.append((key, [v]))
        for _, g in groups:
            self._launch(g)

    @staticmethod
    def _launch(views):
        v0 = views[0]
        s0 = v0["settings"]
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, sh, opacities, dc) = v0["inputs"]
        (c_col, c_m3, c_sc, c_rot, c_cov, c_sh, c_op, c_dc) = v0["caller_inputs"]
        dev = means3D.device
        stream = torch.cuda.current_stream(dev)
        for v in views:  # each view's render backward ran on its forward's stream
            stream.wait_event(v["event"])
            # the batched kernel reads each view's state buffers on THIS stream: keep their memory
            # out of the caching allocator's reuse on their own streams until it has run
            for t in (v["geom"], v["binning"], v["radii"]):
                t.record_stream(stream)
        inputs = {"means3D": c_m3, "dc": c_dc, "sh": c_sh, "opacities": c_op, "scales": c_sc, "rotations": c_rot,
                  "cov3D_precomp": c_cov, "colors_precomp": c_col}
        on_chunk, done = _chunk_hook({k for k, t in inputs.items()
                                      if t is not None and t.numel() and t.requires_grad})
        try:
            # under a chunk hook (overlapped all-reduce) the gradients go into FRESH buffers, which the
            # hook reduces, and reach an existing .grad by autograd's add below: adding into a .grad
            # that already holds reduced gradients (an earlier launch group, a late view) and then
            # reducing it again would multiply those by the world size
            accumulate = {} if on_chunk is not None else {
                k: g for k, g in ((k, _accumulation_target(t)) for k, t in inputs.items()) if g is not None}
            if "dc" in accumulate and (dc is None or dc.numel() == 0):
                del accumulate["dc"]
            fence = _acc_fence.get(dev)
            if accumulate and fence is not None:
                stream.wait_event(fence)
            for g in accumulate.values():
                g.record_stream(stream)
            grads = _C.rasterize_gaussians_preprocess_backward_views(
                means3D, [v["radii"] for v in views], colors_precomp, opacities, scales, rotations,
                s0.scale_modifier, cov3Ds_precomp, [v["settings"].viewmatrix for v in views],
                [v["settings"].projmatrix for v in views], [v["settings"].tanfovx for v in views],
                [v["settings"].tanfovy for v in views], s0.image_height, s0.image_width, sh, s0.sh_degree,
                [v["settings"].campos for v in views], [v["geom"] for v in views], [v["num_rendered"] for v in views],
                [v["binning"] for v in views], any(v["has_inv"] for v in views), s0.antialiasing, s0.debug, dc=dc,
                accumulate=accumulate, on_chunk=on_chunk)
        finally:
            if done is not None:
                done()
        ev = torch.cuda.Event()
        ev.record(stream)
        _acc_fence[dev] = ev
        if len(grads) == 9:
            g2d, g_col, g_op, g_m3, g_cov, g_dc, g_sh, g_sc, g_rot = grads
        else:
            g2d, g_col, g_op, g_m3, g_cov, g_sh, g_sc, g_rot = grads
            g_dc = None
        # A leaf without a .grad (and without hooks) takes its gradient buffer as .grad, as autograd's
        # AccumulateGrad would (the parameter gradients stay views of ONE buffer: multiview's
        # in-place all-reduce); the rest goes through autograd: activations (exp, sigmoid,
        # normalize, cat) between the parameters and the rasterizer inputs, leaves with hooks.
        tensors, gts = [], []
        pairs = [(c_m3, g_m3), (c_sh, g_sh), (c_col, g_col), (c_op, g_op), (c_sc, g_sc), (c_rot, g_rot),
                 (c_cov, g_cov), (c_dc, g_dc)]
        pairs += [(v["means2D"], g2d[j]) for j, v in enumerate(views)]
        for t, g in pairs:
            if g is None or t is None or t.numel() == 0 or not t.requires_grad:
                continue
            g = g.view(t.shape)
            if t.is_leaf and t.grad is None and not t._backward_hooks and \
                    not getattr(t, "_post_accumulate_grad_hooks", None) and g.device == t.device:
                t.grad = g
            else:
                tensors.append(t)
                gts.append(g)
        if tensors:
            torch.autograd.backward(tensors, gts)


@contextlib.contextmanager
def deferred_backward():
    """Rasterizer calls (GaussianRasterizer) whose forward runs inside this context defer the
    per-Gaussian half of their backward: a view's backward runs only its BACKWARD::render (the
    per-(tile, Gaussian) records, gsr_backward_render) as soon as its image gradient exists, and
    when the context exits ONE BACKWARD::preprocess pass over the Gaussians
    (gsr_backward_preprocess_views) produces the gradients of all the views at once, summed --
    the multi-view step of MultiViewRasterizer with the views' forward and backward passes still
    free to interleave (view v's render backward beside view v+1's forward on another stream).
    The summed gradients reach the inputs at exit: added in place to an existing .grad of a leaf
    input (as accumulate_grads_in_place), otherwise through autograd (activations between the
    parameters and the rasterizer, means2D's screen-space gradient per view).  Until then the
    inputs' .grad (and means2D.grad) do not hold these views' contributions.  Equal to the views'
    ordinary backward passes up to fp32 summation order."""
    batch = _DeferredBatch()
    prev = getattr(_state, "deferred", None)
    _state.deferred = batch
    try:
        yield batch
    finally:
        _state.deferred = prev
    batch.flush()


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
    batch = getattr(_state, "deferred", None)
    inputs = (means3D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, dc)
    if batch is not None and torch.is_grad_enabled() and any(
            t is not None and t.requires_grad for t in inputs + (means2D,)):
        # deferred_backward: the autograd node sees detached Gaussian inputs (its backward returns
        # nothing for them, and the graph behind them -- activations -- stays untouched until the
        # batch's exit runs it once); means2D (or a stand-in) carries the view's backward call
        anchor = means2D if means2D.requires_grad else torch.zeros((0,), requires_grad=True)
        det = [None if t is None else t.detach() for t in inputs]
        return _RasterizeGaussians.apply(det[0], anchor, det[1], det[2], det[3], det[4], det[5], det[6],
                                         raster_settings, det[7], (batch, inputs, means2D))
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings, dc)


class _RasterizeGaussians(torch.autograd.Function):
    """Forward returns (color (3,H,W), radii int32 (P), invdepth (1,H,W)); backward returns the
    input gradients in input order, with d(means2D) = the screen-space gradient (P,3)
    that the caller's densification statistics read (scene/gaussian_model.py:471-473).  The last
    input, ``dc`` (None unless the separate-DC surface is used), gets its own gradient."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, dc=None, deferred=None):
        s = raster_settings
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer, invdepths = _C.rasterize_gaussians(
            s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered, s.antialiasing, s.debug, dc=dc)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.deferred = deferred  # (batch, the caller's inputs, the caller's means2D): deferred_backward
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
        if ctx.deferred is not None:  # deferred_backward: the records now, the rest at the context's exit
            dev = means3D.device
            has_inv = _C.rasterize_gaussians_render_backward(
                s.bg, means3D.size(0), ctx.num_rendered, geomBuffer, binningBuffer, imgBuffer, grad_out_color,
                grad_out_depth, s.debug)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            batch, caller_inputs, i_m2 = ctx.deferred
            (i_m3, i_sh, i_col, i_op, i_sc, i_rot, i_cov, i_dc) = caller_inputs
            ctx.deferred = None
            # views batched into one launch: the same Gaussian tensors (of the caller) and settings
            key = (tuple(None if t is None or t.numel() == 0 else id(t) for t in caller_inputs), means3D.data_ptr(),
                   sh.data_ptr(),
                   colors_precomp.data_ptr(), opacities.data_ptr(), scales.data_ptr(), rotations.data_ptr(),
                   cov3Ds_precomp.data_ptr(), None if dc is None else dc.data_ptr(), s.image_height, s.image_width,
                   float(s.scale_modifier), s.sh_degree, bool(s.antialiasing), bool(s.debug))
            batch.add({"key": key, "settings": s, "num_rendered": ctx.num_rendered, "radii": radii,
                       "geom": geomBuffer, "binning": binningBuffer, "event": ev, "has_inv": has_inv, "means2D": i_m2,
                       "inputs": (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, sh, opacities, dc),
                       "caller_inputs": (i_col, i_m3, i_sc, i_rot, i_cov, i_sh, i_op, i_dc)})
            return (None,) * 11
        accumulate = None
        if ctx.acc_inputs is not None:
            accumulate = {k: g for k, g in ((k, _accumulation_target(t)) for k, t in ctx.acc_inputs.items())
                          if g is not None}
            if "dc" in accumulate and (dc is None or dc.numel() == 0):
                del accumulate["dc"]
            dev = means3D.device
            stream = torch.cuda.current_stream(dev)
            fence = _acc_fence.get(dev)
            if accumulate and fence is not None:
                stream.wait_event(fence)
            for g in accumulate.values():
                g.record_stream(stream)  # may have been allocated on another view's stream
        grads = _C.rasterize_gaussians_backward(
            s.bg, means3D, radii, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, grad_out_depth, sh, s.sh_degree,
            s.campos, geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, s.antialiasing, s.debug, dc=dc,
            accumulate=accumulate)
        if ctx.acc_inputs is not None:
            ev = torch.cuda.Event()
            ev.record(stream)
            _acc_fence[dev] = ev
        if len(grads) == 9:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_dc, grad_sh,
             grad_scales, grad_rotations) = grads
        else:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
             grad_scales, grad_rotations) = grads
            grad_dc = None
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                grad_rotations, grad_cov3Ds_precomp, None, grad_dc, None)


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


def _check_inputs(shs, colors_precomp, scales, rotations, cov3D_precomp, dc):
    """The reference's argument rules (diff_gaussian_rasterization/__init__.py:178-182)."""
    if (shs is None) == (colors_precomp is None) or (dc is not None and colors_precomp is not None):
        raise Exception('Please provide excatly one of either SHs or precomputed colors!')
    if ((scales is None or rotations is None) and cov3D_precomp is None) or \
            ((scales is not None or rotations is not None) and cov3D_precomp is not None):
        raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')


def rasterize_views(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                    raster_settings, dc=None):
    return _RasterizeViews.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                 cov3Ds_precomp, tuple(raster_settings), dc)


class _RasterizeViews(torch.autograd.Function):
    """A batch of V camera views of the same Gaussians as ONE autograd node (the
    views of a data-parallel step).  Forward: _C.rasterize_gaussians_views (the single-view kernels
    per view, bit-identical outputs, the views' binning prefixes overlapped) into (V,3,H,W) / (V,P)
    / (V,1,H,W) outputs.
    Backward: _C.rasterize_gaussians_backward_views -- every view's BACKWARD::render, then one
    pass of BACKWARD::preprocess that reads each Gaussian's parameters once and writes their
    gradients summed over the views, where V single-view backward passes would read and write the
    236 B/Gaussian V times.  means2D is (V,P,3): its gradient is each view's screen-space gradient
    (what train.py's densification statistics read, gaussian_model.py:471-473)."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, dc=None):
        V = len(raster_settings)
        s0 = raster_settings[0]
        H, W, P = s0.image_height, s0.image_width, means3D.size(0)
        dev = means3D.device
        colors = torch.empty((V, 3, H, W), dtype=torch.float32, device=dev)
        radii = torch.empty((V, P), dtype=torch.int32, device=dev)
        invdepths = torch.empty((V, 1, H, W), dtype=torch.float32, device=dev)
        # gsr_forward_views: the views' binning prefixes (preprocess, sorts, scans: short
        # latency-bound launch chains) run side by side on the library's internal streams, the
        # renders on the caller's stream
        Ls, geoms, bins, imgs = _C.rasterize_gaussians_views(
            s0.bg, means3D, colors_precomp, opacities, scales, rotations, s0.scale_modifier, cov3Ds_precomp,
            [s.viewmatrix for s in raster_settings], [s.projmatrix for s in raster_settings],
            [s.tanfovx for s in raster_settings], [s.tanfovy for s in raster_settings], H, W, sh, s0.sh_degree,
            [s.campos for s in raster_settings], s0.prefiltered, s0.antialiasing, s0.debug, dc=dc,
            out=(colors, radii, invdepths))
        state = list(zip(Ls, geoms, bins, imgs))
        ctx.raster_settings = raster_settings
        ctx.num_rendered = [st[0] for st in state]
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, dc,
                              *[t for st in state for t in st[1:]])
        ctx.acc_inputs = None
        if getattr(_state, "accumulate", False):
            ctx.acc_inputs = {"means3D": means3D, "dc": dc, "sh": sh, "opacities": opacities, "scales": scales,
                              "rotations": rotations, "cov3D_precomp": cov3Ds_precomp,
                              "colors_precomp": colors_precomp}
        return colors, radii, invdepths

    @staticmethod
    def backward(ctx, grad_colors, _grad_radii, grad_invdepths):
        ss = ctx.raster_settings
        s0 = ss[0]
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, dc,
         *bufs) = ctx.saved_tensors
        V = len(ss)
        if grad_colors is None:
            grad_colors = torch.zeros((V, 3, s0.image_height, s0.image_width), dtype=torch.float32,
                                      device=means3D.device)
        # inputs of forward(): means3D 0, sh 2, colors_precomp 3, opacities 4, scales 5, rotations 6,
        # cov3D_precomp 7, dc 9
        names = {0: "means3D", 2: "sh", 3: "colors_precomp", 4: "opacities", 5: "scales", 6: "rotations",
                 7: "cov3D_precomp", 9: "dc"}
        on_chunk, done = _chunk_hook({n for i, n in names.items() if ctx.needs_input_grad[i]})
        accumulate = None
        # no in-place accumulation under a chunk hook: the hook reduces what the kernel writes, and an
        # existing .grad may already hold reduced gradients (see _DeferredBatch._launch)
        if ctx.acc_inputs is not None and on_chunk is None:
            accumulate = {k: g for k, g in ((k, _accumulation_target(t)) for k, t in ctx.acc_inputs.items())
                          if g is not None}
            if "dc" in accumulate and (dc is None or dc.numel() == 0):
                del accumulate["dc"]
            dev = means3D.device
            stream = torch.cuda.current_stream(dev)
            fence = _acc_fence.get(dev)
            if accumulate and fence is not None:
                stream.wait_event(fence)
            for g in accumulate.values():
                g.record_stream(stream)
        try:
            grads = _C.rasterize_gaussians_backward_views(
                s0.bg, means3D, [radii[v] for v in range(V)], colors_precomp, opacities, scales, rotations,
                s0.scale_modifier, cov3Ds_precomp, [s.viewmatrix for s in ss], [s.projmatrix for s in ss],
                [s.tanfovx for s in ss], [s.tanfovy for s in ss], grad_colors, grad_invdepths, sh, s0.sh_degree,
                [s.campos for s in ss], bufs[0::3], ctx.num_rendered, bufs[1::3], bufs[2::3], s0.antialiasing,
                s0.debug, dc=dc, accumulate=accumulate, on_chunk=on_chunk)
        finally:
            if done is not None:
                done()
        if accumulate is not None:
            ev = torch.cuda.Event()
            ev.record(stream)
            _acc_fence[dev] = ev
        if len(grads) == 9:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_dc, grad_sh,
             grad_scales, grad_rotations) = grads
        else:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
             grad_scales, grad_rotations) = grads
            grad_dc = None
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                grad_rotations, grad_cov3Ds_precomp, None, grad_dc)


class MultiViewRasterizer(nn.Module):
    """GaussianRasterizer over a batch of V <= 16 views of the same Gaussians (one settings tuple
    per view; image size, background, scale modifier, SH degree and flags shared).  forward takes
    GaussianRasterizer's inputs with means2D of shape (V,P,3) and returns (colors (V,3,H,W), radii
    (V,P), invdepths (V,1,H,W)); each view's outputs are bit-identical to GaussianRasterizer's, the
    parameter gradients are the sums over the views (see _RasterizeViews)."""

    def __init__(self, raster_settings_list):
        super().__init__()
        ss = tuple(raster_settings_list)
        if not 1 <= len(ss) <= 16:
            raise ValueError("MultiViewRasterizer takes 1 to 16 views")
        s0 = ss[0]
        for s in ss[1:]:
            if (s.image_height, s.image_width, float(s.scale_modifier), s.sh_degree, bool(s.prefiltered),
                    bool(s.debug), bool(s.antialiasing)) != (s0.image_height, s0.image_width, float(s0.scale_modifier),
                                                             s0.sh_degree, bool(s0.prefiltered), bool(s0.debug),
                                                             bool(s0.antialiasing)) or not torch.equal(s.bg, s0.bg):
                raise ValueError("the views of a MultiViewRasterizer must share image size, bg, scale_modifier, "
                                 "sh_degree and flags")
        self.raster_settings = ss

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, dc=None):
        _check_inputs(shs, colors_precomp, scales, rotations, cov3D_precomp, dc)
        absent = torch.Tensor([])
        return rasterize_views(
            means3D, means2D,
            absent if shs is None else shs,
            absent if colors_precomp is None else colors_precomp,
            opacities,
            absent if scales is None else scales,
            absent if rotations is None else rotations,
            absent if cov3D_precomp is None else cov3D_precomp,
            self.raster_settings, dc)


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
    def step(self, visibility, N, rows=None):
        """rows = (g0, g1): update only Gaussians [g0, g1) (visibility and every parameter restricted
        to those rows) -- the multi-GPU trainer steps each Gaussian range as soon as its gradient
        all-reduce has landed (multiview.DataParallelTrainer.reduce_and_step)."""
        if rows is not None:
            g0, g1 = int(rows[0]), int(rows[1])
            if not 0 <= g0 <= g1 <= int(N):
                raise RuntimeError(f"rows {rows} outside [0, {int(N)})")
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
            ts = (param, param.grad, state["exp_avg"], state["exp_avg_sq"])
            if rows is not None:  # the rows of Gaussians [g0, g1): contiguous slices of each tensor
                ts = tuple(t.view(int(N), -1)[g0:g1] for t in ts)
            batch.append(ts + (lr, eps))
        if rows is None:
            _C.adam_update_groups(batch, visibility, 0.9, 0.999, N)
        elif g1 > g0:
            _C.adam_update_groups(batch, visibility[g0:g1], 0.9, 0.999, g1 - g0)
