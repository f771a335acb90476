"""Data-parallel training mode: multiview.DataParallelTrainer on real
rasterizer gradients (needs an MI355X: -m gpu).

Two gloo ranks share the one GPU of the test box (the driver's multi-GPU nodes run the same code
over RCCL).  Each step is a batch of 4 of the 8 ring views, view j of the batch on rank j mod 2;
after ITERS steps of train.py's iteration (sparse Adam, L1 + D-SSIM, separate-DC render) the
parameters of both ranks must be bit-identical to each other AND to a single process that renders
the same views and sums the two ranks' gradient buffers itself (x0 + x1: a two-rank all-reduce adds
each element once, and float addition commutes), and the reduced densification statistics must
equal the single process's.  The ranks run the pipelined reduction (DataParallelTrainer.
reduce_and_step: each Gaussian range's all-reduce followed by its sparse-Adam rows), the single
process the unpipelined optimizer step: bit-identical.
"""
import contextlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

P, H, W, VIEWS, BATCH, ITERS, WORLD = 2000, 96, 128, 8, 4, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _collect(q, procs, timeout=240):
    """The workers' results; fails fast (instead of waiting out the timeout) when a worker dies --
    its peer may then wait in a collective forever, so every worker is terminated."""
    import queue
    import time
    res, t0 = [], time.monotonic()
    try:
        while len(res) < len(procs):
            try:
                res.append(q.get(timeout=2))
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                assert not dead, f"a worker failed (exit codes {[p.exitcode for p in procs]})"
                assert time.monotonic() - t0 < timeout, "workers timed out"
    finally:
        for p in procs:
            p.join(timeout=30 if len(res) == len(procs) else 1)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    return sorted(res, key=lambda r: r[0])


def _setup(dev):
    """Trainer (perturbed start of the seed-0 cloud), settings per view and ground-truth images."""
    import synthetic
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import multiview
    gt = synthetic.make_scene(P, seed=0)
    g = torch.Generator().manual_seed(5)
    raw = {"xyz": gt["means3D"] + 0.02 * torch.randn(P, 3, generator=g),
           "f_dc": gt["shs"][:, :1] + 0.3 * torch.randn(P, 1, 3, generator=g),
           "f_rest": gt["shs"][:, 1:].clone(),
           "opacity": torch.full((P, 1), -1.0),
           "scaling": torch.log(gt["scales"]) + 0.3 * torch.randn(P, 3, generator=g),
           "rotation": gt["rotations"] + 0.1 * torch.randn(P, 4, generator=g)}
    trainer = multiview.DataParallelTrainer({k: v.to(dev) for k, v in raw.items()}, lr={"xyz": 4.8e-4})
    settings = []
    for v in range(VIEWS):
        c = synthetic.Camera(W, H, view=v)
        settings.append(dgr.GaussianRasterizationSettings(
            H, W, c.tanfovx, c.tanfovy, torch.zeros(3, device=dev), 1.0, c.world_view_transform.to(dev),
            c.full_proj_transform.to(dev), 3, c.camera_center.to(dev), False, False, False))
    gt_t = {k: v.to(dev) for k, v in gt.items()}
    with torch.no_grad():
        targets = [dgr.GaussianRasterizer(s)(means3D=gt_t["means3D"], means2D=torch.zeros_like(gt_t["means3D"]),
                                             shs=gt_t["shs"], opacities=gt_t["opacities"], scales=gt_t["scales"],
                                             rotations=gt_t["rotations"])[0].clamp(0, 1) for s in settings]
    return trainer, settings, targets


def _rank_views(it, rank, settings, targets):
    from diff_gaussian_rasterization import multiview
    batch = [(BATCH * it + j) % VIEWS for j in range(BATCH)]
    return [(settings[batch[j]], targets[batch[j]]) for j in multiview.views_of_batch(rank, WORLD, BATCH)]


def _result(trainer):
    st = trainer.reduced_densification_stats()
    return ({k: p.detach().cpu().numpy() for k, p in trainer.params.items()},
            {k: st[k].cpu().numpy() for k in ("xyz_gradient_accum", "denom", "max_radii2D")})


def _worker(rank, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gaussian-splatting-npu_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        trainer, settings, targets = _setup(dev)
        for it in range(ITERS):
            trainer.step(_rank_views(it, rank, settings, targets))
        torch.cuda.synchronize()
        q.put((rank,) + _result(trainer))
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = _collect(q, procs)
    assert all(p.exitcode == 0 for p in procs)

    # the single-process run of the same step: both ranks' views, their buffers summed here
    dev = torch.device("cuda", 0)
    trainer, settings, targets = _setup(dev)
    start = {k: p.detach().clone() for k, p in trainer.params.items()}
    for it in range(ITERS):
        trainer.zero_grad()
        trainer.render_and_backward(_rank_views(it, 0, settings, targets))
        g0 = trainer.flat.clone()
        trainer.zero_grad()
        trainer.render_and_backward(_rank_views(it, 1, settings, targets))
        trainer.flat += g0
        trainer.optimizer_step()
    torch.cuda.synchronize()
    params, stats = _result(trainer)
    assert any(not torch.equal(start[k], trainer.params[k]) for k in start), "the step changed nothing"
    for rank, p_r, s_r in res:
        for k in params:
            np.testing.assert_array_equal(p_r[k], params[k], err_msg=f"rank {rank} {k}")
        np.testing.assert_array_equal(s_r["denom"], stats["denom"])
        np.testing.assert_array_equal(s_r["max_radii2D"], stats["max_radii2D"])
        np.testing.assert_allclose(s_r["xyz_gradient_accum"], stats["xyz_gradient_accum"], rtol=1e-5, atol=1e-9)
    assert stats["denom"].max() > 0


def test_batched_views_match_per_view_renders():
    """A rank's views as one MultiViewRasterizer batch (the trainer's default) against one
    GaussianRasterizer call per view: the per-view losses are bit-identical (same images), the
    summed gradient buffer equal up to fp32 summation order, the densification counts equal."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gaussian-splatting-npu_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dev = torch.device("cuda", 0)
    out = {}
    for batched in (False, True):
        trainer, settings, targets = _setup(dev)
        trainer.batched = batched
        trainer.zero_grad()
        losses = trainer.render_and_backward([(settings[v], targets[v]) for v in range(BATCH)])
        torch.cuda.synchronize()
        out[batched] = ([float(l) for l in losses], trainer.flat.clone().cpu().numpy(),
                        trainer.stats["denom"].clone().cpu().numpy())
    assert out[True][0] == out[False][0], (out[True][0], out[False][0])
    a, b = out[True][1], out[False][1]
    assert np.abs(a - b).max() <= 1e-5 * np.abs(b).max() + 1e-9, np.abs(a - b).max()
    np.testing.assert_array_equal(out[True][2], out[False][2])


# ---- densification across ranks -----------------------------------------
D_ITERS = 4  # train.py iterations 1..4: densify at 2 and 4, opacity reset at 3


def _densify_opt(threshold):
    from diff_gaussian_rasterization import multiview
    o = multiview.OptimizationDefaults()
    o.densify_from_iter, o.densification_interval, o.opacity_reset_interval = 0, 2, 3
    o.densify_until_iter, o.densify_grad_threshold = 100, threshold
    return o


EXTENT = 1.3  # percent_dense * extent = 0.013: about half the Gaussians clone, half split


def _dsetup(dev, threshold):
    import synthetic
    trainer, settings, targets = _setup(dev)
    raw = {k: p.detach().clone() for k, p in trainer.params.items()}
    raw["opacity"][::10] = -6.0  # below train.py's min_opacity 0.005: pruned at the first densification
    from diff_gaussian_rasterization import multiview
    trainer = multiview.DataParallelTrainer(raw, lr={"xyz": 4.8e-4}, opt=_densify_opt(threshold), seed=11)
    # inverse-depth targets (the ground-truth scene's own) so the depth L1 term is exercised
    import diff_gaussian_rasterization as dgr
    gt = {k: v.to(dev) for k, v in synthetic.make_scene(P, seed=0).items()}
    views = []
    with torch.no_grad():
        for s, t in zip(settings, targets):
            inv = dgr.GaussianRasterizer(s)(means3D=gt["means3D"], means2D=torch.zeros_like(gt["means3D"]),
                                            shs=gt["shs"], opacities=gt["opacities"], scales=gt["scales"],
                                            rotations=gt["rotations"])[2]
            views.append((s, t, {"invdepth": inv * 1.1, "depth_mask": (inv > 0).float()}))
    return trainer, views


def _drank_views(it, rank, views):
    from diff_gaussian_rasterization import multiview
    batch = [(BATCH * it + j) % VIEWS for j in range(BATCH)]
    return [views[batch[j]] for j in multiview.views_of_batch(rank, WORLD, BATCH)]


def _dworker(rank, port, threshold, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gaussian-splatting-npu_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        trainer, views = _dsetup(dev, threshold)
        did = []
        for it in range(1, D_ITERS + 1):
            did.append(trainer.iteration(it, _drank_views(it, rank, views), EXTENT)[1])
        torch.cuda.synchronize()
        q.put((rank, {k: p.detach().cpu().numpy() for k, p in trainer.params.items()},
               {k: trainer.optimizer.state[p]["exp_avg"].cpu().numpy() for k, p in trainer.params.items()}, did))
    finally:
        dist.destroy_process_group()


def _emulate(dev, threshold):
    """The same iterations in one process: both ranks' views rendered here, their gradient buffers
    and densification statistics combined as the collectives combine them (x0 + x1, max)."""
    from diff_gaussian_rasterization import multiview
    trainer, views = _dsetup(dev, threshold)
    o = trainer.opt
    stats = [trainer.stats, multiview.densification_stats(trainer.P, dev)]
    did = []
    for it in range(1, D_ITERS + 1):
        trainer.update_learning_rate(it)
        w = trainer.depth_l1_weight(it)
        trainer.zero_grad()
        trainer.stats = stats[0]
        trainer.render_and_backward(_drank_views(it, 0, views), w)
        g0 = trainer.flat.clone()
        trainer.zero_grad()
        trainer.stats = stats[1]
        trainer.render_and_backward(_drank_views(it, 1, views), w)
        trainer.flat += g0
        d = None
        if it > o.densify_from_iter and it % o.densification_interval == 0:
            red = multiview.densification_stats(trainer.P, dev)
            red["_sums"].copy_(stats[0]["_sums"] + stats[1]["_sums"])
            red["max_radii2D"].copy_(torch.max(stats[0]["max_radii2D"], stats[1]["max_radii2D"]))
            d = trainer.densify_and_prune(o.densify_grad_threshold, 0.005, EXTENT,
                                          20 if it > o.opacity_reset_interval else None, stats=red)
            stats = [trainer.stats, multiview.densification_stats(trainer.P, dev)]
        if it % o.opacity_reset_interval == 0:
            trainer.reset_opacity()
        trainer.optimizer_step()
        did.append(d)
    torch.cuda.synchronize()
    return trainer, did


def test_two_ranks_densify_and_reset_match_single_process():
    """train.py's iteration with densification (train.py:164-174) over 2 gloo ranks: two
    densify_and_prune calls (clone, split and prune each happen) and an opacity reset between
    them, plus the inverse-depth L1 term; afterwards both ranks' parameters and Adam moments are
    bit-identical to each other and to the single-process emulation."""
    dev = torch.device("cuda", 0)
    # a threshold that selects about half of the Gaussians: the median of the statistics the first
    # densification will see (a dry run of iterations 1-2 in one process)
    trainer, views = _dsetup(dev, 1.0)
    from diff_gaussian_rasterization import multiview
    for it in (1, 2):
        trainer.zero_grad()
        trainer.render_and_backward(_drank_views(it, 0, views), trainer.depth_l1_weight(it))
        trainer.render_and_backward(_drank_views(it, 1, views), trainer.depth_l1_weight(it))
    g = trainer.stats["xyz_gradient_accum"] / trainer.stats["denom"]
    threshold = float(torch.nan_to_num(g, 0.0).median())
    assert threshold > 0

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dworker, args=(r, port, threshold, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = _collect(q, procs)
    assert all(p.exitcode == 0 for p in procs)

    emu, did = _emulate(dev, threshold)
    d2, d4 = did[1], did[3]
    assert d2 is not None and d4 is not None and did[0] is None and did[2] is None
    assert d2["cloned"] > 0 and d2["split"] > 0 and d2["pruned"] > 0, d2
    assert d4["P_after"] != P, did
    for rank, params, moments, rdid in res:
        assert rdid == did, (rank, rdid, did)
        for k in params:
            np.testing.assert_array_equal(params[k], emu.params[k].detach().cpu().numpy(), err_msg=f"rank {rank} {k}")
            np.testing.assert_array_equal(moments[k], emu.optimizer.state[emu.params[k]]["exp_avg"].cpu().numpy(),
                                          err_msg=f"rank {rank} exp_avg {k}")


# ---- the gradient all-reduce overlapped with the batched backward ---------
O_P, O_H, O_W, O_VIEWS = 4000, 144, 176, 4


def _oworker(rank, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gaussian-splatting-npu_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import synthetic
        import diff_gaussian_rasterization as dgr
        from diff_gaussian_rasterization import multiview
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        scene = synthetic.make_scene(O_P, seed=0)
        mine = multiview.views_of_batch(rank, WORLD, O_VIEWS)
        settings, grads = [], []
        for v in mine:
            c = synthetic.Camera(O_W, O_H, view=v)
            settings.append(dgr.GaussianRasterizationSettings(
                O_H, O_W, c.tanfovx, c.tanfovy, torch.zeros(3, device=dev), 1.0, c.world_view_transform.to(dev),
                c.full_proj_transform.to(dev), 3, c.camera_center.to(dev), False, False, False))
            grads.append(tuple(g.to(dev) for g in synthetic.make_grads(O_H, O_W, seed=1 + v)))
        out = {}
        log = open(os.path.join(root, "gpurun_out", f"overlap_rank{rank}.log"), "w")
        for mode in ("plain", "overlap", "deferred_overlap", "deferred_overlap_18"):
            print(f"rank {rank} mode {mode} start", file=log, flush=True)
            params = {k: v.to(dev).clone().requires_grad_(True) for k, v in scene.items()}
            reps = 1
            if mode == "deferred_overlap_18":
                # 18 views per rank: two batched launches (16 + 2), into a .grad that already holds
                # gradients -- each launch's own contribution is reduced once
                reps = 9
                for p_ in params.values():
                    p_.grad = torch.full_like(p_, 0.5)
            ctx = multiview.overlapped_allreduce(chunks=3) if mode != "plain" else contextlib.nullcontext()
            with ctx as st:
                if mode.startswith("deferred_overlap"):
                    with dgr.deferred_backward():
                        for s, (gc, gi) in zip(settings * reps, grads * reps):
                            m2 = torch.zeros_like(params["means3D"], requires_grad=True)
                            c, _, i = dgr.GaussianRasterizer(s)(means2D=m2, **{
                                "means3D": params["means3D"], "shs": params["shs"], "opacities": params["opacities"],
                                "scales": params["scales"], "rotations": params["rotations"]})
                            torch.autograd.backward([c, i], [gc, gi])
                else:
                    m2 = torch.zeros((len(settings), O_P, 3), device=dev, requires_grad=True)
                    c, _, i = dgr.MultiViewRasterizer(settings)(
                        means3D=params["means3D"], means2D=m2, shs=params["shs"], opacities=params["opacities"],
                        scales=params["scales"], rotations=params["rotations"])
                    torch.autograd.backward([c, i], [torch.stack([g[0] for g in grads]),
                                                     torch.stack([g[1] for g in grads])])
            if mode == "plain":
                multiview.allreduce_grads(params)
            elif mode == "deferred_overlap_18":
                assert st["chunks"] == 6 and st["collectives"] == 30, st
            else:
                assert st["chunks"] == 3 and st["collectives"] == 15, st
            torch.cuda.synchronize()
            print(f"rank {rank} mode {mode} done {st}", file=log, flush=True)
            out[mode] = {k: p.grad.cpu().numpy() for k, p in params.items()}
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_equals_allreduce_after_backward():
    """multiview.overlapped_allreduce (the batched BACKWARD::preprocess in 3 Gaussian ranges, each
    range's gradient rows all-reduced while the next computes) against the unchunked backward
    followed by allreduce_grads: bitwise equal, on 2 gloo ranks, for a MultiViewRasterizer batch
    and for deferred_backward's flush; and equal on both ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.makedirs(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out"), exist_ok=True)
    procs = [ctx.Process(target=_oworker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = _collect(q, procs)
    assert all(p.exitcode == 0 for p in procs)
    ref = res[0][1]["plain"]
    for rank, out in res:
        for mode in ("plain", "overlap"):
            for k in ref:
                np.testing.assert_array_equal(out[mode][k], ref[k], err_msg=f"rank {rank} {mode} {k}")
        # the deferred flush sums the same views with the same kernel: bitwise too
        for k in ref:
            np.testing.assert_array_equal(out["deferred_overlap"][k], res[0][1]["deferred_overlap"][k],
                                          err_msg=f"rank {rank} deferred {k}")
            ok = np.abs(out["deferred_overlap"][k] - ref[k]).max() <= 1e-5 * np.abs(ref[k]).max() + 1e-9
            assert ok, f"rank {rank} deferred vs batch {k}"
            # 9 copies of the step's views in two launch groups on top of a .grad of 0.5: 0.5 + 9 x
            # the reduced gradient (not multiplied by the world size anywhere)
            want = 0.5 + 9.0 * ref[k].astype(np.float64)
            err = np.abs(out["deferred_overlap_18"][k] - want).max()
            assert err <= 1e-5 * np.abs(want).max() + 1e-6, f"rank {rank} 18 views {k}: {err}"
