"""Multi-view data-parallel step logic on CPU with gloo, world_size 2.

The GPU bench runs the same functions over RCCL; here each rank fabricates the gradients a
forward+backward of its views would leave in .grad and checks that the single bucketed
all_reduce(SUM) produces the sum over all views on every rank, and that the view deal-out
covers each of the 8 ring views exactly once at every supported GPU count.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-npu_amd"))

from diff_gaussian_rasterization import multiview  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_params(P, M, view):
    """Parameters plus the per-view gradient a fwd+bwd of `view` would accumulate."""
    g = torch.Generator().manual_seed(100 + view)
    shapes = {"means3D": (P, 3), "shs": (P, M, 3), "opacities": (P, 1), "scales": (P, 3), "rotations": (P, 4)}
    out = {}
    for k, shp in shapes.items():
        t = torch.zeros(shp, requires_grad=True)
        t.grad = torch.randn(shp, generator=g)
        out[k] = t
    return out


def _fake_params_flat(P, M, view):
    """As _fake_params, with the gradients as consecutive views of one buffer (the layout the
    HIP backward produces)."""
    p = _fake_params(P, M, view)
    flat = torch.cat([p[k].grad.reshape(-1) for k in multiview.PARAM_ORDER])
    off = 0
    for k in multiview.PARAM_ORDER:
        n = p[k].grad.numel()
        p[k].grad = flat[off:off + n].view_as(p[k])
        off += n
    return p


def _worker(rank, world, port, P, M, views_per_rank, q, flat=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        views = multiview.views_for_rank(rank, world, views_per_rank)
        params = None
        for v in views:  # local accumulation over this rank's views
            p = (_fake_params_flat if flat else _fake_params)(P, M, v)
            if params is None:
                params = p
            else:
                for k in params:
                    params[k].grad += p[k].grad
        assert (multiview.flat_grad_view(params) is not None) == flat
        nbytes = multiview.allreduce_grads(params)
        t = multiview.max_over_ranks(0.5 + rank)
        q.put((rank, views, {k: v.grad.numpy().copy() for k, v in params.items()}, nbytes, t))  # by value
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("flat", [False, True], ids=["bucketed", "in-place"])
@pytest.mark.parametrize("views_per_rank", [1, 4])
def test_allreduce_sums_all_views_world2(views_per_rank, flat):
    world, P, M = 2, 257, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, M, views_per_rank, q, flat))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    all_views = sorted(v for r in res for v in r[1])
    assert all_views == sorted(set(all_views)) and len(all_views) == world * views_per_rank
    expect = None
    for v in all_views:
        p = _fake_params(P, M, v)
        expect = {k: t.grad.clone() for k, t in p.items()} if expect is None else \
            {k: expect[k] + p[k].grad for k in expect}
    for rank, _, grads, nbytes, t in res:
        assert nbytes == 4 * P * (3 + 3 * M + 1 + 3 + 4)  # 236 B/Gaussian at M=16
        assert t == 0.5 + (world - 1)  # max over ranks
        for k in expect:
            torch.testing.assert_close(torch.from_numpy(grads[k]), expect[k], rtol=1e-6, atol=1e-6)
    # both replicas hold bit-identical gradients after the reduction
    for k in expect:
        assert (res[0][2][k] == res[1][2][k]).all()


def _fake_view(P, view):
    """A view's screen-space gradient (P,3) and int32 radii (about a third culled)."""
    g = torch.Generator().manual_seed(500 + view)
    grad = torch.randn((P, 3), generator=g)
    radii = torch.randint(0, 40, (P,), generator=g, dtype=torch.int32)
    radii[torch.rand((P,), generator=g) < 0.3] = 0
    return grad, radii


def _stats_worker(rank, world, port, P, views_per_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stats = multiview.densification_stats(P)
        for v in multiview.views_for_rank(rank, world, views_per_rank):
            multiview.add_view_stats(stats, *_fake_view(P, v))
        nbytes = multiview.allreduce_densification_stats(stats)
        q.put((rank, {k: stats[k].numpy().copy() for k in ("xyz_gradient_accum", "denom", "max_radii2D")},
               nbytes))
    finally:
        dist.destroy_process_group()


def _serial_stats(P, views):
    """train.py:166 + gaussian_model.py:471-473 applied view after view on one process."""
    accum = torch.zeros((P, 1))
    denom = torch.zeros((P, 1))
    max_radii2D = torch.zeros((P,))
    for v in views:
        grad, radii = _fake_view(P, v)
        visibility_filter = (radii > 0).nonzero()  # gaussian_renderer/__init__.py:123
        max_radii2D[visibility_filter] = torch.max(max_radii2D[visibility_filter], radii[visibility_filter])
        accum[visibility_filter] += torch.norm(grad[visibility_filter, :2], dim=-1, keepdim=True)
        denom[visibility_filter] += 1
    return {"xyz_gradient_accum": accum, "denom": denom, "max_radii2D": max_radii2D}


@pytest.mark.parametrize("views_per_rank", [1, 4])
def test_densification_stats_reduce_world2(views_per_rank):
    world, P = 2, 301
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, world, port, P, views_per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    views = sorted(v for r in range(world) for v in multiview.views_for_rank(r, world, views_per_rank))
    expect = _serial_stats(P, views)
    for rank, got, nbytes in res:
        assert nbytes == P * 2 * 4 + P * 4
        torch.testing.assert_close(torch.from_numpy(got["xyz_gradient_accum"]), expect["xyz_gradient_accum"],
                                   rtol=1e-6, atol=1e-6)
        assert torch.equal(torch.from_numpy(got["denom"]), expect["denom"])
        assert torch.equal(torch.from_numpy(got["max_radii2D"]), expect["max_radii2D"])
    for k in ("xyz_gradient_accum", "denom", "max_radii2D"):
        assert (res[0][1][k] == res[1][1][k]).all()


def test_view_stats_match_training_loop_single_process():
    P = 97
    stats = multiview.densification_stats(P)
    for v in (0, 3):
        multiview.add_view_stats(stats, *_fake_view(P, v))
    assert multiview.allreduce_densification_stats(stats) == 0
    expect = _serial_stats(P, (0, 3))
    for k in expect:
        torch.testing.assert_close(stats[k], expect[k], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_views_cover_the_ring(world):
    views = [v for r in range(world) for v in multiview.views_for_rank(r, world, 8 // world)]
    assert sorted(views) == list(range(8))


def test_single_process_is_a_noop():
    params = _fake_params(4, 16, 0)
    before = {k: v.grad.clone() for k, v in params.items()}
    assert multiview.allreduce_grads(params) == 0
    for k in params:
        assert torch.equal(params[k].grad, before[k])
    with pytest.raises(ValueError):
        multiview.views_for_rank(2, 2)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_views_of_batch_strong_scaling(world):
    """bench.py's default step: the same 8-view batch at every N, each view on exactly one rank."""
    per = [multiview.views_of_batch(r, world, 8) for r in range(world)]
    assert sorted(v for vs in per for v in vs) == list(range(8))
    assert all(len(vs) == 8 // world for vs in per)
    with pytest.raises(ValueError):
        multiview.views_of_batch(0, 16, 8)


# ---- densification surgery (DataParallelTrainer.densify_and_prune / reset_opacity) on CPU ------
def _ref_densify(raw, state, grads, max_grad, min_opacity, extent, max_screen_size, gen, pd=0.01, N=2, normal=None,
                 counts=None):
    """gaussian_model.py:315-469 step by step on dicts (the reference's own sequence: clone's
    postfix, split's postfix, split prune, final prune; tensors and Adam moments).  `normal(stds)`:
    the split's samples (default: torch.normal on `gen`); `counts`: a dict that receives the
    cloned / split / pruned counts."""
    names = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
    T = {k: raw[k].clone() for k in names}
    S = {k: {"exp_avg": state[k][0].clone(), "exp_avg_sq": state[k][1].clone()} for k in names}

    def cat(d):
        for k in names:
            T[k] = torch.cat((T[k], d[k]), 0)
            S[k]["exp_avg"] = torch.cat((S[k]["exp_avg"], torch.zeros_like(d[k])), 0)
            S[k]["exp_avg_sq"] = torch.cat((S[k]["exp_avg_sq"], torch.zeros_like(d[k])), 0)

    def prune(mask):
        keep = ~mask
        for k in names:
            T[k] = T[k][keep]
            S[k]["exp_avg"] = S[k]["exp_avg"][keep]
            S[k]["exp_avg_sq"] = S[k]["exp_avg_sq"][keep]
    # densify_and_clone
    sel = torch.where(torch.norm(grads, dim=-1) >= max_grad, True, False)
    sel = torch.logical_and(sel, torch.max(torch.exp(T["scaling"]), dim=1).values <= pd * extent)
    n_clone = int(sel.sum())
    cat({k: T[k][sel] for k in names})
    # densify_and_split
    n_init = T["xyz"].shape[0]
    padded = torch.zeros((n_init,))
    padded[:grads.shape[0]] = grads.squeeze()
    sel = torch.where(padded >= max_grad, True, False)
    sel = torch.logical_and(sel, torch.max(torch.exp(T["scaling"]), dim=1).values > pd * extent)
    stds = torch.exp(T["scaling"])[sel].repeat(N, 1)
    samples = normal(stds) if normal is not None else torch.normal(mean=torch.zeros((stds.size(0), 3)), std=stds,
                                                                    generator=gen)
    rots = multiview.build_rotation(T["rotation"][sel]).repeat(N, 1, 1)
    new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + T["xyz"][sel].repeat(N, 1),
           "scaling": torch.log(torch.exp(T["scaling"])[sel].repeat(N, 1) / (0.8 * N)),
           "rotation": T["rotation"][sel].repeat(N, 1), "f_dc": T["f_dc"][sel].repeat(N, 1, 1),
           "f_rest": T["f_rest"][sel].repeat(N, 1, 1), "opacity": T["opacity"][sel].repeat(N, 1)}
    cat(new)
    prune(torch.cat((sel, torch.zeros(N * int(sel.sum()), dtype=bool))))
    max_radii2D = torch.zeros((T["xyz"].shape[0],))  # densification_postfix zeroed it
    mask = (torch.sigmoid(T["opacity"]) < min_opacity).squeeze()
    if max_screen_size:
        mask = mask | (max_radii2D > max_screen_size) | (torch.exp(T["scaling"]).max(dim=1).values > 0.1 * extent)
    prune(mask)
    if counts is not None:
        counts.update(cloned=n_clone, split=int(sel.sum()), pruned=int(mask.sum()), P_after=int(T["xyz"].shape[0]))
    return T, S


def test_densify_and_prune_matches_reference_sequence():
    """DataParallelTrainer.densify_and_prune (one pass over the tensors and the optimizer state,
    rebuilding the flat gradient buffer) against the reference's step-by-step sequence, and
    reset_opacity against gaussian_model.py:258-261 -- on CPU tensors with torch Adam."""
    P, M = 400, 15
    g = torch.Generator().manual_seed(3)
    raw = {"xyz": torch.randn(P, 3, generator=g), "f_dc": torch.randn(P, 1, 3, generator=g),
           "f_rest": 0.1 * torch.randn(P, M, 3, generator=g),
           "opacity": torch.randn(P, 1, generator=g) * 3.0,
           "scaling": torch.log(0.003 + 0.02 * torch.rand(P, 3, generator=g)),
           "rotation": torch.randn(P, 4, generator=g)}
    tr = multiview.DataParallelTrainer(raw, optimizer="adam", seed=9)
    for p in tr.params.values():  # one optimizer step so the moments are non-trivial
        p.grad.copy_(torch.randn(p.shape, generator=g))
    tr.optimizer_step()
    state = {k: (tr.optimizer.state[p]["exp_avg"].clone(), tr.optimizer.state[p]["exp_avg_sq"].clone())
             for k, p in tr.params.items()}
    before = {k: p.detach().clone() for k, p in tr.params.items()}
    stats = multiview.densification_stats(P)
    stats["xyz_gradient_accum"].copy_(torch.rand(P, 1, generator=g) * 2e-3)
    stats["denom"].copy_(torch.randint(0, 3, (P, 1), generator=g).float())  # some 0/0 -> NaN -> 0
    stats["max_radii2D"].copy_(torch.rand(P, generator=g) * 40)
    did = tr.densify_and_prune(5e-4, 0.05, 1.3, 20, stats=stats)
    gen = torch.Generator().manual_seed(9)
    grads = stats["xyz_gradient_accum"] / stats["denom"]
    grads[grads.isnan()] = 0.0
    T, S = _ref_densify(before, state, grads, 5e-4, 0.05, 1.3, 20, gen)
    assert did["cloned"] > 0 and did["split"] > 0 and did["pruned"] > 0, did
    assert tr.P == T["xyz"].shape[0] == did["P_after"]
    for k, p in tr.params.items():
        assert torch.equal(p.detach(), T[k]), k
        assert torch.equal(tr.optimizer.state[p]["exp_avg"], S[k]["exp_avg"]), k
        assert torch.equal(tr.optimizer.state[p]["exp_avg_sq"], S[k]["exp_avg_sq"]), k
        # the gradients are views of the rebuilt flat buffer, zeroed
        assert p.grad.shape == p.shape and p.grad.untyped_storage().data_ptr() == tr.flat.untyped_storage().data_ptr()
    assert tr.stats["denom"].shape == (tr.P, 1) and float(tr.stats["_sums"].abs().sum()) == 0.0
    # the iteration's optimizer step skips the replaced parameters (the reference's have no grad)
    snap = {k: p.detach().clone() for k, p in tr.params.items()}
    tr.optimizer_step()
    assert all(torch.equal(snap[k], tr.params[k].detach()) for k in snap)
    # reset_opacity: min(sigmoid, 0.01) in logit space, moments zeroed, opacity not stepped this time
    op = tr.params["opacity"].detach().clone()
    tr.reset_opacity()
    want = multiview.inverse_sigmoid(torch.min(torch.sigmoid(op), torch.ones_like(op) * 0.01))
    assert torch.equal(tr.params["opacity"].detach(), want)
    assert float(tr.optimizer.state[tr.params["opacity"]]["exp_avg"].abs().sum()) == 0.0
    for p in tr.params.values():
        p.grad.copy_(torch.randn(p.shape, generator=g))
    tr.optimizer_step()
    assert torch.equal(tr.params["opacity"].detach(), want)
    assert not torch.equal(tr.params["xyz"].detach(), T["xyz"])


def test_expon_lr_matches_reference_formula():
    """utils/general_utils.py get_expon_lr_func: endpoints, log-linear midpoint, delay easing."""
    import math
    f = multiview.expon_lr(1e-2, 1e-4, max_steps=100)
    assert math.isclose(f(0), 1e-2) and math.isclose(f(100), 1e-4) and math.isclose(f(50), 1e-3)
    assert f(-1) == 0.0 and math.isclose(f(1000), 1e-4)
    d = multiview.expon_lr(1.0, 1.0, lr_delay_steps=10, lr_delay_mult=0.01)
    assert math.isclose(d(0), 0.01) and math.isclose(d(10), 1.0) and 0.01 < d(5) < 1.0


def _overlap_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_rasterization as dgr
        P, M = 1000, 15
        mine = _fake_params(P, M, rank)
        want = {k: t.grad.clone() for k, t in mine.items()}
        for t in want.values():
            dist.all_reduce(t)
        grads = {k: t.grad for k, t in mine.items()}
        with multiview.overlapped_allreduce(chunks=3) as st:
            chunks, fn, done = dgr._grad_chunks  # what a batched backward calls
            step = 384
            for g0 in range(0, P, step):
                fn(g0, min(P, g0 + step), grads)
            done()
        q.put((rank, all(torch.equal(grads[k], want[k]) for k in want), dict(st)))
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_chunks_sum_like_one_allreduce():
    """overlapped_allreduce's hook (what MultiViewRasterizer's backward calls per Gaussian range)
    reduces each range's rows of every gradient: together equal to one all_reduce per tensor, on
    gloo world 2 (CPU)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, st in res:
        assert ok, rank
        assert st == {"collectives": 15, "chunks": 3, "bytes": 4 * 1000 * (3 + 45 + 1 + 3 + 4)}, st
