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
