"""Multi-view data parallelism over the rasterizer.

One process per GPU; the Gaussian parameters are replicated, camera views are dealt out
round-robin (view v goes to rank v mod world), every rank runs forward+backward of its own
views and accumulates the parameter gradients locally, and ONE all_reduce(SUM) of a flat
fp32 bucket holding every parameter gradient (236 B per Gaussian at SH degree 3) makes the
replicas agree.  The densification statistics (screen-space gradient norms and visit counts:
SUM; max screen radius: MAX) are accumulated per view and reduced the same way.  The reference trains on one view per step on one GPU (train.py:97-111);
this is the multi-view form of that step, the only exchange the path has.

Backend-agnostic: "nccl" (RCCL over xGMI) on the GPU box, "gloo" in the CPU tests.
"""
import contextlib

import torch
import torch.distributed as dist

# parameter order of the bucket (xyz, features, opacity, scaling, rotation)
PARAM_ORDER = ("means3D", "shs", "opacities", "scales", "rotations")
# the same with the separate-DC surface (features_dc apart from features_rest)
PARAM_ORDER_DC = ("means3D", "dc", "shs", "opacities", "scales", "rotations")


def views_for_rank(rank, world, views_per_rank=1, n_views=8):
    """Views this rank renders: rank, rank + world, ... (mod n_views)."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return [(rank + i * world) % n_views for i in range(views_per_rank)]


def views_of_batch(rank, world, views_total=8):
    """Views this rank renders when a step is a fixed batch of `views_total` views dealt
    round-robin (strong scaling): v = rank, rank + world, ... < views_total."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    if views_total < world:
        raise ValueError(f"{views_total} views cannot occupy {world} ranks")
    return list(range(rank, views_total, world))


def grad_bucket(params, order=PARAM_ORDER):
    """Flat fp32 view of every parameter gradient (a fresh contiguous buffer)."""
    return torch.cat([params[k].grad.reshape(-1) for k in order])


def flat_grad_view(params, order=PARAM_ORDER):
    """The one buffer holding every parameter gradient, if the .grad tensors are consecutive
    views of a single storage in `order` (as the HIP backward allocates them and autograd hands
    them to the leaves); otherwise None."""
    gs = [params[k].grad for k in order]
    g0 = gs[0]
    if any(g is None for g in gs):
        return None
    if any(not g.is_contiguous() or g.dtype != g0.dtype or g.device != g0.device for g in gs):
        return None
    base = g0.untyped_storage().data_ptr()
    off = g0.storage_offset()
    for g in gs:
        if g.untyped_storage().data_ptr() != base or g.storage_offset() != off:
            return None
        off += g.numel()
    return g0.as_strided((off - g0.storage_offset(),), (1,), g0.storage_offset())


def allreduce_grads(params, order=PARAM_ORDER, group=None):
    """SUM every parameter gradient across ranks with one collective on a flat bucket.  When the
    gradients already live in one buffer (flat_grad_view) it is reduced in place; otherwise they
    are gathered into a bucket and scattered back.  Returns the number of bytes reduced per rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return 0
    flat = flat_grad_view(params, order)
    if flat is not None:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        return flat.numel() * flat.element_size()
    flat = grad_bucket(params, order)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for k in order:
        g = params[k].grad
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n
    return flat.numel() * flat.element_size()


@contextlib.contextmanager
def overlapped_allreduce(group=None, chunks=4):
    """The gradient all-reduce overlapped with the backward ("overlap it with the last
    view's backward"): batched backward passes run inside this context (MultiViewRasterizer, the
    flush of deferred_backward) compute their parameter gradients in `chunks` Gaussian ranges, and
    each range's rows of every parameter gradient go to an asynchronous all_reduce(SUM) as soon as
    its launch is enqueued -- the collective of range k runs while range k+1 computes.  The backward
    waits for its collectives before it returns, so the gradients it hands to autograd are already
    the sums over the ranks; the caller then skips allreduce_grads.  Chunks over [0, P) write
    exactly the rows one full launch writes, so the reduced gradients equal allreduce_grads after an
    unchunked backward bit for bit (for leaf inputs; activations between the parameters and the
    rasterizer are back-propagated from the reduced gradients afterwards).  Only for the one batched
    backward of a step: each backward inside reduces what its inputs' gradients hold then.  Yields
    a dict counting the collectives issued; a no-op (yields None) without a process group of more
    than one rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        yield None
        return
    import diff_gaussian_rasterization as dgr
    works, stats = [], {"collectives": 0, "chunks": 0, "bytes": 0}

    def fn(g0, g1, grads):
        stats["chunks"] += 1
        for t in grads.values():
            part = t[g0:g1]
            works.append(dist.all_reduce(part, op=dist.ReduceOp.SUM, group=group, async_op=True))
            stats["collectives"] += 1
            stats["bytes"] += part.numel() * part.element_size()

    def done():
        for w in works:
            w.wait()
        works.clear()
    with dgr.grad_chunk_hook(chunks, fn, done):
        yield stats


def densification_stats(P, device=None):
    """Per-rank densification accumulators, shaped as GaussianModel keeps them
    (scene/gaussian_model.py: xyz_gradient_accum (P,1), denom (P,1), max_radii2D (P,)).
    accum and denom are two columns of ONE (P,2) buffer so their SUM is one collective."""
    sums = torch.zeros((P, 2), dtype=torch.float32, device=device)
    return {"xyz_gradient_accum": sums[:, 0:1], "denom": sums[:, 1:2], "_sums": sums,
            "max_radii2D": torch.zeros((P,), dtype=torch.float32, device=device)}


@torch.no_grad()
def add_view_stats(stats, viewspace_grad, radii):
    """One view's contribution, before any reduction: train.py:166 (running max of radii over
    the visible Gaussians) and gaussian_model.py:471-473 (the norm of that view's screen-space
    gradient, taken per view, and a visit count).  viewspace_grad is the view's means2D.grad
    (P,3); radii the view's int32 radii (P,)."""
    vis = radii > 0
    mr = stats["max_radii2D"]
    mr[vis] = torch.max(mr[vis], radii[vis].to(mr.dtype))
    stats["xyz_gradient_accum"][vis] += torch.norm(viewspace_grad[vis, :2], dim=-1, keepdim=True)
    stats["denom"][vis] += 1


def allreduce_densification_stats(stats, group=None):
    """SUM of (xyz_gradient_accum, denom) in one collective on their shared (P,2) buffer, MAX of
    max_radii2D in a second: afterwards every replica holds the statistics of all
    views of the step, so densify_and_prune makes the same decision on every rank.  Returns the
    bytes reduced per rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return 0
    sums, mr = stats["_sums"], stats["max_radii2D"]
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(mr, op=dist.ReduceOp.MAX, group=group)
    return sums.numel() * sums.element_size() + mr.numel() * mr.element_size()


def max_over_ranks(seconds, device=None, group=None):
    """The slowest rank's wall time (the bench's timed region)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


# ---- train.py's iteration as a data-parallel step ------------------------
# GaussianModel's parameter groups, in its optimizer order (scene/gaussian_model.py:186-193)
TRAIN_GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
# train.py's learning rates at iteration 1 (arguments/__init__.py:74-100; xyz is scaled by the
# scene's spatial_lr_scale and decays with get_expon_lr_func -- the caller's update_learning_rate)
TRAIN_LR = {"xyz": 0.00016, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005,
            "rotation": 0.001}


def expon_lr(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py get_expon_lr_func (:29-63): log-linear decay from lr_init to
    lr_final over max_steps, with an optional sine-eased delay."""
    import math

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * math.sin(0.5 * math.pi * min(max(step / lr_delay_steps,
                                                                                               0.0), 1.0))
        else:
            delay_rate = 1.0
        t = min(max(step / max_steps, 0.0), 1.0)
        return delay_rate * math.exp(math.log(lr_init) * (1 - t) + math.log(lr_final) * t)
    return helper


def build_rotation(r):
    """utils/general_utils.py build_rotation (:78-99): normalised wxyz quaternions -> (N,3,3)."""
    q = r / torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.zeros((q.size(0), 3, 3), device=r.device, dtype=r.dtype)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def inverse_sigmoid(x):
    """utils/general_utils.py inverse_sigmoid (:18-19)."""
    return torch.log(x / (1 - x))


def view_from_camera(cam, bg, sh_degree=3, scale_modifier=1.0, debug=False, antialiasing=False, cam_index=None,
                     device=None):
    """One training view for DataParallelTrainer from a reference camera (scene/cameras.py Camera,
    or MiniCam plus `original_image`): (GaussianRasterizationSettings, ground-truth image, extras),
    the settings exactly as gaussian_renderer/__init__.py:32-50 builds them (tan of half the FoV,
    int image size, world_view_transform / full_proj_transform / camera_center, prefiltered False),
    and the extras train.py:113-141 reads from the camera: `alpha_mask` (the image is multiplied by
    it), `invdepth` + `depth_mask` only when `depth_reliable` (the depth L1 term), and `cam` =
    `cam_index` for the per-camera exposure.  `bg` (3,) on the device, as train.py's background."""
    import math
    import diff_gaussian_rasterization as dgr
    dev = device if device is not None else bg.device
    settings = dgr.GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width), tanfovx=math.tan(cam.FoVx * 0.5),
        tanfovy=math.tan(cam.FoVy * 0.5), bg=bg, scale_modifier=scale_modifier,
        viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev), sh_degree=sh_degree,
        campos=cam.camera_center.to(dev), prefiltered=False, debug=debug, antialiasing=antialiasing)
    extras = {}
    alpha = getattr(cam, "alpha_mask", None)
    if alpha is not None:
        extras["alpha_mask"] = alpha.to(dev)
    if getattr(cam, "depth_reliable", False) and getattr(cam, "invdepthmap", None) is not None:
        extras["invdepth"] = cam.invdepthmap.to(dev)
        extras["depth_mask"] = cam.depth_mask.to(dev)
    if cam_index is not None:
        extras["cam"] = cam_index
    return settings, cam.original_image.to(dev), extras


def views_from_cameras(cameras, bg, sh_degree=3, **kw):
    """view_from_camera over a Scene's train cameras (scene.getTrainCameras()), the camera's index
    in the list as its exposure index (train.py's `vind`, gaussian_model.py:175-176)."""
    return [view_from_camera(c, bg, sh_degree, cam_index=i, **kw) for i, c in enumerate(cameras)]


class OptimizationDefaults:
    """The densification / schedule fields of arguments/__init__.py OptimizationParams (:74-100)
    that train.py's iteration reads."""
    iterations = 30_000
    position_lr_init = 0.00016
    position_lr_final = 0.0000016
    position_lr_delay_mult = 0.01
    position_lr_max_steps = 30_000
    percent_dense = 0.01
    lambda_dssim = 0.2
    densification_interval = 100
    opacity_reset_interval = 3000
    densify_from_iter = 500
    densify_until_iter = 15_000
    densify_grad_threshold = 0.0002
    depth_l1_weight_init = 1.0
    depth_l1_weight_final = 0.01
    exposure_lr_init = 0.01
    exposure_lr_final = 0.001
    exposure_lr_delay_steps = 0
    exposure_lr_delay_mult = 0.0


class DataParallelTrainer:
    """train.py's iteration (train.py:97-186) over G ranks, one process per GPU.

    The reference trains on one random view per iteration on one GPU.  Here one step takes a
    batch of views; every rank holds a full replica of the Gaussians and renders its share of the
    batch (view v on rank v mod G, `views_of_batch`), and:

    1. renders its views -- as ONE MultiViewRasterizer batch (the default; `batched=False`: one
       GaussianRasterizer call per view) -- with train.py's inputs
       (activations of gaussian_model.py:40-48,102-135; the separate-DC surface train.py selects
       with SparseGaussianAdam, gaussian_renderer/__init__.py:82-100; the per-camera exposure
       when `exposures` is given, :112-115; image clamped to [0, 1], :119), loss = (1 - lambda_dssim)
       L1 + lambda_dssim (1 - fused SSIM) (train.py:119-124) + the inverse-depth L1 term for views
       with a depth target (train.py:128-141), backward; the per-view losses of the batch add up,
       so the step's gradient is the SUM of its views' gradients;
    2. keeps train.py's densification statistics per view, locally (train.py:166,
       gaussian_model.py:471-473: max screen radius, norm of that view's screen-space gradient,
       visit count);
    3. all-reduces (SUM) ONE flat fp32 buffer: every parameter gradient (236 B per Gaussian at SH
       degree 3; the parameters' .grad are views into it, so autograd accumulates into it in place
       and the collective runs in place) plus one visibility count per Gaussian (and the exposure
       gradients), so the same collective tells every rank which Gaussians some view of the step saw;
    4. steps the same optimizer on every rank: SparseGaussianAdam on the Gaussians visible in the
       step (train.py:180-183) or torch Adam (the default optimizer_type); identical reduced inputs
       keep the replicas bit-identical without a broadcast.

    Densification (train.py:164-174) runs on every rank from the statistics of ALL views of ALL
    ranks since the last densification (`reduced_densification_stats`: SUM of accum/denom, MAX of
    max_radii2D, reduced once at that point): `densify_and_prune` / `reset_opacity` follow
    gaussian_model.py:258-261,315-469, rebuild the flat buffer, the parameters and the optimizer
    state (Adam / sparse-Adam moments: cat_tensors_to_optimizer, _prune_optimizer,
    replace_tensor_to_optimizer) for the new P, identically on every rank (the split's random
    samples come from a generator seeded identically everywhere).  `iteration()` is train.py's
    loop body with that gating, the learning-rate schedule and the optimizer step.
    Backend-agnostic: RCCL ("nccl") on MI355X nodes, gloo in the tests.
    """

    def __init__(self, raw, lr=None, optimizer="sparse_adam", lambda_dssim=0.2, bg=None, group=None, batched=True,
                 seed=0, exposures=None, spatial_lr_scale=None, opt=None, pipeline_chunks=4):
        import diff_gaussian_rasterization as dgr
        self._dgr = dgr
        # > 1 (sparse Adam, several ranks): the gradient all-reduce and the optimizer step pipelined
        # over this many Gaussian ranges (reduce_and_step) in iterations without densification
        self.pipeline_chunks = pipeline_chunks
        dev = raw["xyz"].device
        self.device = dev
        self.group = group
        self.batched = batched  # a rank's views as one MultiViewRasterizer batch (one launch per stage)
        self.lambda_dssim = lambda_dssim
        self.opt = opt or OptimizationDefaults()
        self.bg = bg if bg is not None else torch.zeros(3, device=dev)
        self.lr = dict(TRAIN_LR, **(lr or {}))
        # xyz schedule (gaussian_model.py:184,203-206): position_lr_* x spatial_lr_scale; only when
        # the caller names the scene's spatial_lr_scale (else lr["xyz"] stays fixed)
        self.xyz_schedule = None if spatial_lr_scale is None else expon_lr(
            self.opt.position_lr_init * spatial_lr_scale, self.opt.position_lr_final * spatial_lr_scale,
            lr_delay_mult=self.opt.position_lr_delay_mult, max_steps=self.opt.position_lr_max_steps)
        self.depth_l1_weight = expon_lr(self.opt.depth_l1_weight_init, self.opt.depth_l1_weight_final,
                                        max_steps=self.opt.iterations)
        # the split's normal samples (gaussian_model.py:418): same seed on every rank -> same samples
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        self.sparse = optimizer == "sparse_adam"
        self.optimizer = None
        # per-camera 3x4 exposure (gaussian_model.py:175-176,201), optional (train_test_exp)
        self.exposures = None
        self.exposure_optimizer = None
        if exposures is not None:
            self.exposures = torch.nn.Parameter(exposures.detach().to(dev, torch.float32).contiguous().clone())
            self.exposure_optimizer = torch.optim.Adam([self.exposures])
            self.exposure_schedule = expon_lr(self.opt.exposure_lr_init, self.opt.exposure_lr_final,
                                              lr_delay_steps=self.opt.exposure_lr_delay_steps,
                                              lr_delay_mult=self.opt.exposure_lr_delay_mult,
                                              max_steps=self.opt.iterations)
        self._skip_step = set()
        self._install({k: raw[k].detach().to(dev, torch.float32).contiguous().clone() for k in TRAIN_GROUPS})
        groups = [{"params": [self.params[k]], "lr": self.lr[k], "name": k} for k in TRAIN_GROUPS]
        self.optimizer = (dgr.SparseGaussianAdam(groups, lr=0.0, eps=1e-15) if self.sparse
                          else torch.optim.Adam(groups, lr=0.0, eps=1e-15))

    def _install(self, tensors, states=None):
        """(Re)builds, for P = tensors["xyz"].shape[0]: the flat buffer [gradients of every group |
        visibility count per Gaussian | exposure gradients], the parameters (their .grad views of
        it), the densification statistics (zero), and -- after the first call -- the optimizer's
        groups and state, moved onto the new parameters (`states`: group name -> state dict)."""
        dev = self.device
        P = tensors["xyz"].shape[0]
        self.P = P
        sizes = [tensors[k].numel() for k in TRAIN_GROUPS]
        n_exp = self.exposures.numel() if self.exposures is not None else 0
        self.flat = torch.zeros(sum(sizes) + P + n_exp, dtype=torch.float32, device=dev)
        params = {}
        off = 0
        for k, n in zip(TRAIN_GROUPS, sizes):
            p = torch.nn.Parameter(tensors[k].contiguous())
            p.grad = self.flat[off:off + n].view_as(p)
            params[k] = p
            off += n
        self.visible_count = self.flat[off:off + P]
        off += P
        if self.exposures is not None:
            self.exposures.grad = self.flat[off:off + n_exp].view_as(self.exposures)
        if self.optimizer is not None:
            for group in self.optimizer.param_groups:
                old = group["params"][0]
                st = self.optimizer.state.pop(old, None)
                new = params[group["name"]]
                group["params"][0] = new
                st = states.get(group["name"], st) if states is not None else st
                if st:
                    self.optimizer.state[new] = st
        self.params = params
        self.stats = densification_stats(P, dev)

    def activations(self):
        """GaussianModel.get_* (gaussian_model.py:102-135)."""
        p = self.params
        return {"means3D": p["xyz"], "dc": p["f_dc"], "shs": p["f_rest"],
                "opacities": torch.sigmoid(p["opacity"]), "scales": torch.exp(p["scaling"]),
                "rotations": torch.nn.functional.normalize(p["rotation"])}

    def zero_grad(self):
        self.flat.zero_()

    def _expose(self, img, cam_index):
        """gaussian_renderer/__init__.py:112-115: rendered = (img^T E[:3,:3])^T + E[:3,3]."""
        if self.exposures is None or cam_index is None:
            return img
        e = self.exposures[cam_index]
        return torch.matmul(img.permute(1, 2, 0), e[:3, :3]).permute(2, 0, 1) + e[:3, 3, None, None]

    def render(self, settings, act=None, cam_index=None):
        """gaussian_renderer.render with separate_sh=True: (clamped image, screen-space points, radii,
        inverse depth)."""
        act = act or self.activations()
        means2D = torch.zeros_like(act["means3D"], requires_grad=True)
        means2D.retain_grad()
        img, radii, inv = self._dgr.GaussianRasterizer(settings)(
            means3D=act["means3D"], means2D=means2D, dc=act["dc"], shs=act["shs"], colors_precomp=None,
            opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"], cov3D_precomp=None)
        return self._expose(img, cam_index).clamp(0, 1), means2D, radii, inv

    def render_views(self, settings_list, act=None):
        """render() for a batch of views in one MultiViewRasterizer call: (images (V,3,H,W) before
        exposure and clamp, screen-space points (V,P,3), radii (V,P), inverse depths (V,1,H,W))."""
        act = act or self.activations()
        means2D = torch.zeros((len(settings_list),) + tuple(act["means3D"].shape), dtype=act["means3D"].dtype,
                              device=act["means3D"].device, requires_grad=True)
        means2D.retain_grad()
        imgs, radii, inv = self._dgr.MultiViewRasterizer(settings_list)(
            means3D=act["means3D"], means2D=means2D, dc=act["dc"], shs=act["shs"], colors_precomp=None,
            opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"], cov3D_precomp=None)
        return imgs, means2D, radii, inv

    def _view_loss(self, img, inv, view, depth_weight):
        """train.py:115-141 for one view: alpha mask, L1 + D-SSIM, the inverse-depth L1 term."""
        from fused_ssim import fused_ssim
        gt = view[1]
        extra = view[2] if len(view) > 2 and view[2] is not None else {}
        if extra.get("alpha_mask") is not None:
            img = img * extra["alpha_mask"]
        l1 = (img - gt).abs().mean()
        loss = (1.0 - self.lambda_dssim) * l1 + self.lambda_dssim * (1.0 - fused_ssim(img[None], gt[None]))
        if depth_weight > 0 and extra.get("invdepth") is not None:
            mask = extra.get("depth_mask")
            d = (inv - extra["invdepth"]) if mask is None else (inv - extra["invdepth"]) * mask
            loss = loss + depth_weight * d.abs().mean()
        return loss

    def render_and_backward(self, views, depth_weight=0.0, track_stats=True):
        """Step 1-2 for this rank's views: [(GaussianRasterizationSettings, gt image (3,H,W)[, extras])]
        with extras an optional dict: "invdepth" / "depth_mask" (train.py:130-141, weighted by
        `depth_weight`), "alpha_mask" (:115-117), "cam" (the view's exposure index).  Gradients
        accumulate into the flat buffer; returns the per-view losses.  With `batched` (the default)
        the views are one MultiViewRasterizer batch: each view's image is the one
        GaussianRasterizer renders, bit for bit, and the parameter gradients are the sum over the
        views up to fp32 summation order.  `track_stats`: train.py keeps densification statistics
        only before densify_until_iter (train.py:164-167)."""
        def cam_of(view):
            return view[2].get("cam") if len(view) > 2 and view[2] is not None else None
        if self.batched and len(views) > 1:
            with self._dgr.accumulate_grads_in_place():
                imgs, means2D, radii, invs = self.render_views([v[0] for v in views])
            losses = [self._view_loss(self._expose(imgs[j], cam_of(v)).clamp(0, 1), invs[j], v, depth_weight)
                      for j, v in enumerate(views)]
            torch.stack(losses).sum().backward()
            with torch.no_grad():
                for j in range(len(views)):
                    if track_stats:
                        add_view_stats(self.stats, means2D.grad[j], radii[j])
                    self.visible_count += (radii[j] > 0).to(self.visible_count.dtype)
            return [l.detach() for l in losses]
        losses = []
        for v in views:
            # xyz, f_dc, f_rest enter the rasterizer as leaves whose .grad are views of the flat
            # buffer: the backward kernel adds into them directly (no separate accumulation pass)
            with self._dgr.accumulate_grads_in_place():
                img, means2D, radii, inv = self.render(v[0], cam_index=cam_of(v))
            loss = self._view_loss(img, inv, v, depth_weight)
            loss.backward()
            with torch.no_grad():
                if track_stats:
                    add_view_stats(self.stats, means2D.grad, radii)
                self.visible_count += (radii > 0).to(self.visible_count.dtype)
            losses.append(loss.detach())
        return losses

    def reduce(self):
        """Step 3: one in-place all_reduce(SUM) of gradients + visibility counts.  Returns bytes."""
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return 0
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        return self.flat.numel() * self.flat.element_size()

    @torch.no_grad()
    def optimizer_step(self):
        """Step 4 (train.py:176-183).  Parameters replaced by a densification or an opacity reset in
        this iteration are new tensors without a gradient in the reference, so its optimizer skips
        them (Adam skips parameters whose grad is None): the same here."""
        if self.exposure_optimizer is not None:
            self.exposure_optimizer.step()
        skip = [self.params[k] for k in self._skip_step]
        held = [p.grad for p in skip]
        for p in skip:
            p.grad = None
        try:
            if self.sparse:
                self.optimizer.step(self.visible_count > 0, self.P)
            else:
                self.optimizer.step()
        finally:
            for p, g in zip(skip, held):
                p.grad = g
            self._skip_step = set()

    def update_learning_rate(self, iteration):
        """gaussian_model.py:213-223: the exposure and xyz schedules."""
        if self.exposure_optimizer is not None:
            for g in self.exposure_optimizer.param_groups:
                g["lr"] = self.exposure_schedule(iteration)
        if self.xyz_schedule is None:
            return None
        for g in self.optimizer.param_groups:
            if g["name"] == "xyz":
                g["lr"] = self.xyz_schedule(iteration)
                return g["lr"]

    def _pipelined(self):
        return (self.sparse and self.pipeline_chunks > 1 and not self._skip_step and dist.is_initialized()
                and dist.get_world_size(self.group) > 1)

    @torch.no_grad()
    def reduce_and_step(self, chunks=None):
        """Steps 3 + 4 pipelined over Gaussian ranges: every range's
        rows of each gradient and of the visibility counts go to an asynchronous all_reduce(SUM) at
        once; then, range by range, the optimizer waits for that range's collectives only and runs
        SparseGaussianAdam on its rows -- range k's update runs while range k+1 is still being
        reduced.  With 2 ranks this is bit-identical to reduce() + optimizer_step() (a + b commutes;
        tests/test_dp_train.py).  With more ranks a ring all-reduce adds each element's terms in an
        order that depends on how the buffer is split across the ring, so reducing range by range can
        round differently from one flat reduction: the result is then identical on every rank (the
        replicas stay in sync) but not bit-identical to the unpipelined path -- not pinned by a test.
        (Iterations that densify or reset opacities keep the unpipelined order: the reference
        densifies between the reduction and the step.)"""
        P = self.P
        chunks = max(1, min(chunks or self.pipeline_chunks, P))
        bounds = [(P * k // chunks, P * (k + 1) // chunks) for k in range(chunks)]
        works = []
        for g0, g1 in bounds:
            w = [dist.all_reduce(self.params[k].grad.view(P, -1)[g0:g1], op=dist.ReduceOp.SUM, group=self.group,
                                 async_op=True) for k in TRAIN_GROUPS]
            w.append(dist.all_reduce(self.visible_count[g0:g1], op=dist.ReduceOp.SUM, group=self.group,
                                     async_op=True))
            works.append(w)
        if self.exposures is not None:
            dist.all_reduce(self.exposures.grad, op=dist.ReduceOp.SUM, group=self.group)
            self.exposure_optimizer.step()
        visible = torch.empty((P,), dtype=torch.bool, device=self.device)  # (each range's rows after its reduction)
        for (g0, g1), w in zip(bounds, works):
            for x in w:
                x.wait()
            visible[g0:g1] = self.visible_count[g0:g1] > 0
            self.optimizer.step(visible, P, rows=(g0, g1))

    def step(self, views, depth_weight=0.0):
        self.zero_grad()
        losses = self.render_and_backward(views, depth_weight)
        if self._pipelined():
            self.reduce_and_step()
            return losses
        self.reduce()
        self.optimizer_step()
        return losses

    def iteration(self, iteration, views, extent, white_background=False):
        """train.py's loop body (train.py:93-186) for one data-parallel step: learning rates, render +
        loss (with the depth term's schedule, :64,130), backward, the gradient all-reduce, the
        densification gating (:164-174) and the optimizer step.  Returns the per-view losses and a
        dict of what densification did (None when it did not run)."""
        o = self.opt
        self.update_learning_rate(iteration)
        self.zero_grad()
        track = iteration < o.densify_until_iter
        losses = self.render_and_backward(views, self.depth_l1_weight(iteration), track_stats=track)
        densify = track and ((iteration > o.densify_from_iter and iteration % o.densification_interval == 0) or
                             iteration % o.opacity_reset_interval == 0 or
                             (white_background and iteration == o.densify_from_iter))
        if not densify and self._pipelined():
            self.reduce_and_step()
            return losses, None
        self.reduce()
        did = None
        if track:
            if iteration > o.densify_from_iter and iteration % o.densification_interval == 0:
                size_threshold = 20 if iteration > o.opacity_reset_interval else None
                did = self.densify_and_prune(o.densify_grad_threshold, 0.005, extent, size_threshold)
            if iteration % o.opacity_reset_interval == 0 or (white_background and iteration == o.densify_from_iter):
                self.reset_opacity()
        self.optimizer_step()
        return losses, did

    def reduced_densification_stats(self):
        """Copies of the densification statistics of every view of every rank since the last
        reset (what GaussianModel.densify_and_prune reads): SUM of xyz_gradient_accum and denom,
        MAX of max_radii2D.  The local accumulators are left as they are."""
        out = densification_stats(self.P, self.device)
        out["_sums"].copy_(self.stats["_sums"])
        out["max_radii2D"].copy_(self.stats["max_radii2D"])
        allreduce_densification_stats(out, self.group)
        return out

    def reset_densification_stats(self):
        self.stats["_sums"].zero_()
        self.stats["max_radii2D"].zero_()

    # ---- densification (gaussian_model.py:315-469), identically on every rank ----------------
    def _tensors_and_states(self):
        T = {k: p.detach() for k, p in self.params.items()}
        S = {k: dict(self.optimizer.state.get(p, {})) for k, p in self.params.items()}
        return T, S

    @staticmethod
    def _cat(T, S, new):
        """cat_tensors_to_optimizer (gaussian_model.py:364-384): append rows, zero moments for them."""
        for k in TRAIN_GROUPS:
            T[k] = torch.cat((T[k], new[k]), dim=0)
            st = S[k]
            if st:
                st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(new[k])), dim=0)
                st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(new[k])), dim=0)

    @staticmethod
    def _keep(T, S, mask):
        """_prune_optimizer (gaussian_model.py:331-347): keep the rows of `mask`, moments too."""
        for k in TRAIN_GROUPS:
            T[k] = T[k][mask]
            st = S[k]
            if st:
                st["exp_avg"] = st["exp_avg"][mask]
                st["exp_avg_sq"] = st["exp_avg_sq"][mask]

    @torch.no_grad()
    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, stats=None, N=2):
        """GaussianModel.densify_and_prune (gaussian_model.py:452-469) on the reduced statistics
        (`stats`: the reduced statistics to use instead, e.g. a single process emulating ranks):
        clone the small high-gradient Gaussians (:425-440), split the large ones into N samples
        (:402-423), then prune the split originals, the transparent ones and -- with
        max_screen_size -- the world-space large ones.  As in the reference, densification_postfix
        zeroes max_radii2D before the prune reads it (:399), so the screen-space test never fires.
        Rebuilds buffers, parameters and optimizer state for the new P; returns the counts."""
        pd = self.opt.percent_dense
        st = stats if stats is not None else self.reduced_densification_stats()
        grads = st["xyz_gradient_accum"] / st["denom"]
        grads[grads.isnan()] = 0.0
        T, S = self._tensors_and_states()
        P0 = T["xyz"].shape[0]
        # clone (densify_and_clone)
        sel = torch.norm(grads, dim=-1) >= max_grad
        sel = torch.logical_and(sel, torch.exp(T["scaling"]).max(dim=1).values <= pd * extent)
        n_clone = int(sel.sum())
        self._cat(T, S, {k: T[k][sel] for k in TRAIN_GROUPS})
        # split (densify_and_split)
        n_init = T["xyz"].shape[0]
        padded = torch.zeros((n_init,), device=self.device)
        padded[:grads.shape[0]] = grads.squeeze()
        scaling = torch.exp(T["scaling"])
        sel = padded >= max_grad
        sel = torch.logical_and(sel, scaling.max(dim=1).values > pd * extent)
        n_split = int(sel.sum())
        stds = scaling[sel].repeat(N, 1)
        samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=self.device), std=stds, generator=self.gen)
        rots = build_rotation(T["rotation"][sel]).repeat(N, 1, 1)
        new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + T["xyz"][sel].repeat(N, 1),
               "scaling": torch.log(scaling[sel].repeat(N, 1) / (0.8 * N)),
               "rotation": T["rotation"][sel].repeat(N, 1),
               "f_dc": T["f_dc"][sel].repeat(N, 1, 1), "f_rest": T["f_rest"][sel].repeat(N, 1, 1),
               "opacity": T["opacity"][sel].repeat(N, 1)}
        self._cat(T, S, new)
        prune_filter = torch.cat((sel, torch.zeros(N * n_split, device=self.device, dtype=torch.bool)))
        self._keep(T, S, ~prune_filter)
        # prune (max_radii2D is all zero here, see the docstring)
        prune = (torch.sigmoid(T["opacity"]) < min_opacity).squeeze(-1)
        if max_screen_size:
            big_ws = torch.exp(T["scaling"]).max(dim=1).values > 0.1 * extent
            prune = torch.logical_or(prune, big_ws)
        n_prune = int(prune.sum())
        self._keep(T, S, ~prune)
        self._install(T, S)
        self._skip_step = set(TRAIN_GROUPS)  # every parameter is a new tensor without a gradient
        return {"P_before": P0, "cloned": n_clone, "split": n_split, "pruned": n_prune, "P_after": self.P}

    @torch.no_grad()
    def reset_opacity(self):
        """GaussianModel.reset_opacity (gaussian_model.py:258-261) + replace_tensor_to_optimizer
        (:315-329): opacities capped at 0.01, their moments zeroed, the step count kept."""
        p = self.params["opacity"]
        p.copy_(inverse_sigmoid(torch.min(torch.sigmoid(p), torch.ones_like(p) * 0.01)))
        st = self.optimizer.state.get(p)
        if st:
            st["exp_avg"] = torch.zeros_like(p)
            st["exp_avg_sq"] = torch.zeros_like(p)
        self._skip_step.add("opacity")
