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
