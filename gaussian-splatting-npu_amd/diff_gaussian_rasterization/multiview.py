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


class DataParallelTrainer:
    """train.py's iteration (train.py:97-183) over G ranks, one process per GPU.

    The reference trains on one random view per iteration on one GPU.  Here one step takes a
    batch of views; every rank holds a full replica of the Gaussians and renders its share of the
    batch (view v on rank v mod G, `views_of_batch`), and:

    1. renders its views -- as ONE MultiViewRasterizer batch (the default; `batched=False`: one
       GaussianRasterizer call per view) -- with train.py's inputs
       (activations of gaussian_model.py:40-48,102-135; the separate-DC surface train.py selects
       with SparseGaussianAdam, gaussian_renderer/__init__.py:82-100; image clamped to [0, 1],
       :119), loss = (1 - lambda_dssim) L1 + lambda_dssim (1 - fused SSIM) (train.py:119-124),
       backward; the per-view losses of the batch add up, so the step's gradient is the SUM of its
       views' gradients;
    2. keeps train.py's densification statistics per view, locally (train.py:166,
       gaussian_model.py:471-473: max screen radius, norm of that view's screen-space gradient,
       visit count);
    3. all-reduces (SUM) ONE flat fp32 buffer: every parameter gradient (236 B per Gaussian at SH
       degree 3; the parameters' .grad are views into it, so autograd accumulates into it in place
       and the collective runs in place) plus one visibility count per Gaussian, so the same
       collective tells every rank which Gaussians some view of the step saw;
    4. steps the same optimizer on every rank: SparseGaussianAdam on the Gaussians visible in the
       step (train.py:180-183) or torch Adam (the default optimizer_type); identical reduced inputs
       keep the replicas bit-identical without a broadcast.

    Densification itself stays with the caller (GaussianModel.densify_and_prune); before it runs,
    `reduced_densification_stats()` gives every rank the statistics of ALL views since the last
    reset (SUM of accum/denom, MAX of max_radii2D) -- reduced once at that point, not per step, so
    nothing is counted twice.  Backend-agnostic: RCCL ("nccl") on MI355X nodes, gloo in the tests.
    """

    def __init__(self, raw, lr=None, optimizer="sparse_adam", lambda_dssim=0.2, bg=None, group=None, batched=True):
        import diff_gaussian_rasterization as dgr
        self._dgr = dgr
        dev = raw["xyz"].device
        self.device = dev
        self.P = P = raw["xyz"].shape[0]
        self.group = group
        self.batched = batched  # a rank's views as one MultiViewRasterizer batch (one launch per stage)
        self.lambda_dssim = lambda_dssim
        self.bg = bg if bg is not None else torch.zeros(3, device=dev)
        lr = dict(TRAIN_LR, **(lr or {}))
        sizes = [raw[k].numel() for k in TRAIN_GROUPS]
        # [gradients of every group | visibility count per Gaussian]
        self.flat = torch.zeros(sum(sizes) + P, dtype=torch.float32, device=dev)
        self.params = {}
        off = 0
        for k, n in zip(TRAIN_GROUPS, sizes):
            p = torch.nn.Parameter(raw[k].detach().to(dev, torch.float32).contiguous().clone())
            p.grad = self.flat[off:off + n].view_as(p)
            self.params[k] = p
            off += n
        self.visible_count = self.flat[off:off + P]
        groups = [{"params": [self.params[k]], "lr": lr[k], "name": k} for k in TRAIN_GROUPS]
        self.sparse = optimizer == "sparse_adam"
        self.optimizer = (dgr.SparseGaussianAdam(groups, lr=0.0, eps=1e-15) if self.sparse
                          else torch.optim.Adam(groups, lr=0.0, eps=1e-15))
        self.stats = densification_stats(P, dev)

    def activations(self):
        """GaussianModel.get_* (gaussian_model.py:102-135)."""
        p = self.params
        return {"means3D": p["xyz"], "dc": p["f_dc"], "shs": p["f_rest"],
                "opacities": torch.sigmoid(p["opacity"]), "scales": torch.exp(p["scaling"]),
                "rotations": torch.nn.functional.normalize(p["rotation"])}

    def zero_grad(self):
        self.flat.zero_()

    def render(self, settings, act=None):
        """gaussian_renderer.render with separate_sh=True: (clamped image, screen-space points, radii)."""
        act = act or self.activations()
        means2D = torch.zeros_like(act["means3D"], requires_grad=True)
        means2D.retain_grad()
        img, radii, _ = self._dgr.GaussianRasterizer(settings)(
            means3D=act["means3D"], means2D=means2D, dc=act["dc"], shs=act["shs"], colors_precomp=None,
            opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"], cov3D_precomp=None)
        return img.clamp(0, 1), means2D, radii

    def render_views(self, settings_list, act=None):
        """render() for a batch of views in one MultiViewRasterizer call: (clamped images (V,3,H,W),
        screen-space points (V,P,3), radii (V,P))."""
        act = act or self.activations()
        means2D = torch.zeros((len(settings_list),) + tuple(act["means3D"].shape), dtype=act["means3D"].dtype,
                              device=act["means3D"].device, requires_grad=True)
        means2D.retain_grad()
        imgs, radii, _ = self._dgr.MultiViewRasterizer(settings_list)(
            means3D=act["means3D"], means2D=means2D, dc=act["dc"], shs=act["shs"], colors_precomp=None,
            opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"], cov3D_precomp=None)
        return imgs.clamp(0, 1), means2D, radii

    def render_and_backward(self, views):
        """Step 1-2 for this rank's views: [(GaussianRasterizationSettings, gt image (3,H,W))].
        Gradients accumulate into the flat buffer; returns the per-view losses.  With `batched`
        (the default) the views are one MultiViewRasterizer batch: each view's image is the one
        GaussianRasterizer renders, bit for bit, and the parameter gradients are the sum over the
        views up to fp32 summation order."""
        from fused_ssim import fused_ssim
        if self.batched and len(views) > 1:
            with self._dgr.accumulate_grads_in_place():
                imgs, means2D, radii = self.render_views([s for s, _ in views])
            losses = []
            for v, (_, gt) in enumerate(views):
                l1 = (imgs[v] - gt).abs().mean()
                losses.append((1.0 - self.lambda_dssim) * l1 +
                              self.lambda_dssim * (1.0 - fused_ssim(imgs[v][None], gt[None])))
            torch.stack(losses).sum().backward()
            with torch.no_grad():
                for v in range(len(views)):
                    add_view_stats(self.stats, means2D.grad[v], radii[v])
                    self.visible_count += (radii[v] > 0).to(self.visible_count.dtype)
            return [l.detach() for l in losses]
        losses = []
        for settings, gt in views:
            # xyz, f_dc, f_rest enter the rasterizer as leaves whose .grad are views of the flat
            # buffer: the backward kernel adds into them directly (no separate accumulation pass)
            with self._dgr.accumulate_grads_in_place():
                img, means2D, radii = self.render(settings)
            l1 = (img - gt).abs().mean()
            loss = (1.0 - self.lambda_dssim) * l1 + self.lambda_dssim * (1.0 - fused_ssim(img[None], gt[None]))
            loss.backward()
            with torch.no_grad():
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
        """Step 4 (train.py:176-183)."""
        if self.sparse:
            self.optimizer.step(self.visible_count > 0, self.P)
        else:
            self.optimizer.step()

    def step(self, views):
        self.zero_grad()
        losses = self.render_and_backward(views)
        self.reduce()
        self.optimizer_step()
        return losses

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
