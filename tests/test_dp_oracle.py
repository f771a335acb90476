"""The data-parallel trainer against a loop built only from oracles (needs an
MI355X: -m gpu).  VERDICT r03 item 3.

Two gloo ranks run multiview.DataParallelTrainer.iteration -- train.py's loop body
(train.py:93-186) over a batch of 4 of the 8 ring views per step, view j of the batch on rank
j mod 2, with SparseGaussianAdam, L1 + D-SSIM, densification at iterations 2 and 4 and an opacity
reset at 3 -- driven by reference-shaped cameras through multiview.views_from_cameras (the
scene/cameras.py Camera fields gaussian_renderer/__init__.py:32-50 reads).  The reference is a
single CPU process that never touches the HIP library: per view oracle/gsr_oracle.c forward and
backward, oracle/ssim_oracle.py, the gradients summed over the step's views, the densification
statistics of gaussian_model.py:471-473, the reference's step-by-step densify_and_prune
(test_multiview._ref_densify, gaussian_model.py:402-469), reset_opacity (:258-261) and
oracle/adam_oracle.py on the Gaussians some view of the step saw.

The densification thresholds and scene extents are chosen from the oracle loop's own statistics
in the widest gaps (the log-distance to the nearest value is recorded), so float32 differences
between the two loops cannot flip a decision; the split's normal samples come from a generator
seeded as the trainer's.  Asserts: every densification produces the same counts and P; both ranks
end bit-identical; the per-view PSNR of the trained clouds agrees within PSNR_TOL_DB.
"""
import math
import os
import types

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import adam_oracle
import oracle
import ssim_oracle
import synthetic
from test_dp_train import _collect, _free_port
from test_multiview import _ref_densify

pytestmark = pytest.mark.gpu

P, H, W, VIEWS, BATCH, WORLD, ITERS, SEED = 1500, 96, 128, 8, 4, 2, 40, 11
LR = {"xyz": 4.8e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20.0, "opacity": 2.5e-2, "scaling": 5e-3, "rotation": 1e-3}
NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
PSNR_TOL_DB = 0.01
PERCENT_DENSE = 0.01


def _opt():
    from diff_gaussian_rasterization import multiview
    o = multiview.OptimizationDefaults()
    # densify at 2 and 4 (it > from, it % interval == 0, it < until), opacity reset at 3
    o.densify_from_iter, o.densification_interval, o.opacity_reset_interval, o.densify_until_iter = 0, 2, 3, 5
    return o


def _start():
    gt = synthetic.make_scene(P, seed=0)
    g = torch.Generator().manual_seed(5)
    raw = {"xyz": gt["means3D"] + 0.02 * torch.randn(P, 3, generator=g),
           "f_dc": gt["shs"][:, :1] + 0.3 * torch.randn(P, 1, 3, generator=g),
           "f_rest": gt["shs"][:, 1:].clone(),
           "opacity": torch.full((P, 1), -1.0),
           "scaling": torch.log(gt["scales"]) + 0.3 * torch.randn(P, 3, generator=g),
           "rotation": gt["rotations"] + 0.1 * torch.randn(P, 4, generator=g)}
    raw["opacity"][::10] = -6.0  # below min_opacity 0.005: pruned at the first densification
    return gt, {k: v.contiguous().float() for k, v in raw.items()}


def _activate(raw):
    return {"means3D": raw["xyz"], "dc": raw["f_dc"], "rest": raw["f_rest"], "opacities": torch.sigmoid(raw["opacity"]),
            "scales": torch.exp(raw["scaling"]), "rotations": torch.nn.functional.normalize(raw["rotation"], dim=1)}


def _oracle_render(act, cam):
    shs = torch.cat([act["dc"], act["rest"]], dim=1).detach()
    return oracle.OracleRaster(act["means3D"].detach(), act["opacities"].detach(), torch.zeros(3),
                               cam.world_view_transform, cam.full_proj_transform, cam.camera_center,
                               math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), H, W, shs=shs, sh_degree=3, scales=act["scales"].detach(),
                               rotations=act["rotations"].detach(), nthreads=8)


def _reference_cameras(targets):
    """scene/cameras.py Camera stand-ins with the fields train.py / render() read."""
    cams = []
    for v in range(VIEWS):
        c = synthetic.Camera(W, H, view=v)
        cams.append(types.SimpleNamespace(
            FoVx=c.FoVx, FoVy=c.FoVy, image_width=W, image_height=H, world_view_transform=c.world_view_transform,
            full_proj_transform=c.full_proj_transform, camera_center=c.camera_center,
            original_image=targets[v], alpha_mask=torch.ones((1, H, W)), invdepthmap=None, depth_reliable=False))
    return cams


def _batch(it):
    return [(BATCH * it + j) % VIEWS for j in range(BATCH)]


def _gap_mid(values, lo=0.25, hi=0.75):
    """The geometric midpoint of the widest gap between the sorted positive values inside the
    [lo, hi] quantile band, and half that gap's log-width (the decision margin)."""
    v = np.sort(values[values > 0])
    band = np.log(v[int(lo * len(v)):int(hi * len(v)) + 1])
    gaps = np.diff(band)
    i = int(np.argmax(gaps))
    return float(math.exp(0.5 * (band[i] + band[i + 1]))), float(gaps[i] / 2)


def _choose(grads, raw, big_ws):
    """Threshold in the widest gap of the per-Gaussian mean gradient norms; extent such that the
    clone/split boundary (percent_dense * extent, on the selected Gaussians' largest scales) and,
    with big_ws, the world-space prune boundary (0.1 * extent, on every largest scale and its
    split child's) lie as far from every value as possible."""
    g = grads.squeeze(-1).numpy().astype(np.float64)
    thr, m_g = _gap_mid(g)
    ms = torch.exp(raw["scaling"]).max(dim=1).values.numpy().astype(np.float64)
    sel_ms = np.log(ms[g >= thr])
    all_ms = np.log(np.concatenate([ms, ms / 1.6]))
    best = (-1.0, None)
    for ext in np.exp(np.linspace(math.log(0.8), math.log(2.0), 2001)):
        m = np.abs(sel_ms - math.log(PERCENT_DENSE * ext)).min()
        if big_ws:
            m = min(m, np.abs(all_ms - math.log(0.1 * ext)).min())
        if m > best[0]:
            best = (float(m), float(ext))
    return thr, best[1], {"threshold": thr, "extent": best[1], "margin_grad": m_g, "margin_scale": best[0]}


def _cpu_loop(raw0, cams, targets, rng_device="cuda"):
    """train.py's iteration over the step's 4 views, oracles only (see the module docstring).
    Returns the final raw parameters, each densification's counts and the chosen decisions.
    rng_device: where the split's normal samples are drawn (the trainer's generator lives on the
    GPU; "cpu" only for a dry run without one)."""
    o_ = _opt()
    raw = {k: v.clone() for k, v in raw0.items()}
    S = {k: {"exp_avg": torch.zeros_like(v), "exp_avg_sq": torch.zeros_like(v)} for k, v in raw.items()}
    gen = torch.Generator(device=rng_device).manual_seed(SEED)  # the trainer's split samples (same seed)

    def normal(stds):
        return torch.normal(mean=torch.zeros((stds.size(0), 3), device=rng_device), std=stds.to(rng_device),
                            generator=gen).cpu()
    stats = None
    did, choices, snap = {}, {}, None
    for it in range(1, ITERS + 1):
        if it == o_.densify_until_iter:  # after the last densification and the opacity reset
            snap = {k: v.clone() for k, v in raw.items()}
        n = raw["xyz"].shape[0]
        if stats is None:
            stats = {"accum": torch.zeros((n, 1)), "denom": torch.zeros((n, 1)), "max_radii2D": torch.zeros(n)}
        params = {k: v.clone().requires_grad_(True) for k, v in raw.items()}
        act = _activate(params)
        track = it < o_.densify_until_iter
        vis_any = np.zeros(n, dtype=bool)
        for v in _batch(it):
            o = _oracle_render(act, cams[v])
            img = torch.from_numpy(o.color.copy()).requires_grad_(True)
            imgc = img.clamp(0, 1) * cams[v].alpha_mask  # render()'s clamp, train.py:115-117
            ssim = ssim_oracle.ssim_map(imgc[None], targets[v][None], dtype=torch.float32).mean()
            loss = 0.8 * (imgc - targets[v]).abs().mean() + 0.2 * (1.0 - ssim)
            loss.backward()
            g = o.backward(img.grad.numpy())
            dsh = torch.from_numpy(g["dL_dsh"])
            torch.autograd.backward(
                [act["means3D"], act["dc"], act["rest"], act["opacities"], act["scales"], act["rotations"]],
                [torch.from_numpy(g["dL_dmeans3D"]), dsh[:, :1], dsh[:, 1:], torch.from_numpy(g["dL_dopacity"]),
                 torch.from_numpy(g["dL_dscales"]), torch.from_numpy(g["dL_drotations"])], retain_graph=True)
            vis = o.radii > 0
            if track:  # train.py:166-167, gaussian_model.py:471-473
                vt = torch.from_numpy(vis)
                r = torch.from_numpy(o.radii.astype(np.float32))
                stats["max_radii2D"][vt] = torch.max(stats["max_radii2D"][vt], r[vt])
                m2 = torch.from_numpy(np.asarray(g["dL_dmean2D"]).reshape(n, 3))
                stats["accum"][vt] += torch.norm(m2[vt, :2], dim=-1, keepdim=True)
                stats["denom"][vt] += 1
            vis_any |= vis
        skip = set()
        if track and it > o_.densify_from_iter and it % o_.densification_interval == 0:
            grads = stats["accum"] / stats["denom"]
            grads[grads.isnan()] = 0.0
            size_threshold = 20 if it > o_.opacity_reset_interval else None
            thr, ext, choice = _choose(grads, raw, big_ws=bool(size_threshold))
            counts = {}
            raw, S = _ref_densify(raw, {k: (S[k]["exp_avg"], S[k]["exp_avg_sq"]) for k in NAMES}, grads, thr, 0.005,
                                  ext, size_threshold, None, normal=normal, counts=counts)
            counts["P_before"] = n
            did[it], choices[it] = counts, choice
            stats = None
            skip = set(NAMES)  # every parameter is a new tensor without a gradient (reference)
        if track and it % o_.opacity_reset_interval == 0:  # gaussian_model.py:258-261
            op = raw["opacity"]
            raw["opacity"] = torch.log(torch.min(torch.sigmoid(op), torch.ones_like(op) * 0.01) /
                                       (1 - torch.min(torch.sigmoid(op), torch.ones_like(op) * 0.01)))
            S["opacity"] = {"exp_avg": torch.zeros_like(op), "exp_avg_sq": torch.zeros_like(op)}
            skip.add("opacity")
        for k in NAMES:
            if k in skip:
                continue
            pa = raw[k].numpy().reshape(-1)  # shares storage with raw[k]
            adam_oracle.adam_update(pa, params[k].grad.numpy().reshape(-1).copy(),
                                    S[k]["exp_avg"].numpy().reshape(-1), S[k]["exp_avg_sq"].numpy().reshape(-1),
                                    vis_any, LR[k], 0.9, 0.999, 1e-15, n, raw[k].numel() // n)
    return raw, did, choices, snap


def _worker(rank, port, raw0, targets, choices, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "gaussian-splatting-npu_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from diff_gaussian_rasterization import multiview
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cams = _reference_cameras(targets)
        views = multiview.views_from_cameras(cams, torch.zeros(3, device=dev), sh_degree=3, device=dev)
        trainer = multiview.DataParallelTrainer({k: v.to(dev) for k, v in raw0.items()}, lr=LR, opt=_opt(), seed=SEED)
        did = {}
        for it in range(1, ITERS + 1):
            ext = 1.0
            if it in choices:
                trainer.opt.densify_grad_threshold = choices[it]["threshold"]
                ext = choices[it]["extent"]
            batch = _batch(it)
            mine = [views[batch[j]] for j in multiview.views_of_batch(rank, WORLD, BATCH)]
            _, d = trainer.iteration(it, mine, ext)
            if d is not None:
                did[it] = d
        torch.cuda.synchronize()
        # numpy copies: a torch CPU tensor crosses the queue as a shared-memory fd that dies with this
        # process (the parent then reads EOF)
        q.put((rank, {k: p.detach().cpu().numpy().copy() for k, p in trainer.params.items()}, did))
    finally:
        dist.destroy_process_group()


def _psnrs(raw, cams, targets):
    act = _activate(raw)
    out = []
    for c, t in zip(cams, targets):
        img = np.clip(_oracle_render(act, c).color, 0, 1).astype(np.float64)
        mse = float(((img - t.numpy().astype(np.float64)) ** 2).mean())
        out.append(20.0 * math.log10(1.0 / math.sqrt(mse)))
    return np.array(out)


def test_dp_trainer_matches_oracle_loop():
    import common
    gt, raw0 = _start()
    ring = [synthetic.Camera(W, H, view=v) for v in range(VIEWS)]
    gt_act = {"means3D": gt["means3D"], "dc": gt["shs"][:, :1], "rest": gt["shs"][:, 1:],
              "opacities": gt["opacities"], "scales": gt["scales"], "rotations": gt["rotations"]}
    targets = [torch.from_numpy(np.clip(_oracle_render(gt_act, c).color, 0, 1).astype(np.float32)) for c in ring]
    cams = _reference_cameras(targets)

    raw_cpu, did_cpu, choices, snap = _cpu_loop(raw0, cams, targets)
    assert sorted(did_cpu) == [2, 4], did_cpu
    assert did_cpu[2]["cloned"] > 0 and did_cpu[2]["split"] > 0 and did_cpu[2]["pruned"] > 0, did_cpu

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, raw0, targets, choices, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = _collect(q, procs, timeout=400)
    assert all(p.exitcode == 0 for p in procs)

    p0 = _psnrs(raw0, ring, targets)
    p_reset = _psnrs(snap, ring, targets)  # after the densifications and the opacity reset
    p_cpu = _psnrs(raw_cpu, ring, targets)
    (r0, params0, did0), (r1, params1, did1) = res
    params0 = {k: torch.from_numpy(v) for k, v in params0.items()}
    params1 = {k: torch.from_numpy(v) for k, v in params1.items()}
    for k in params0:
        assert torch.equal(params0[k], params1[k]), f"ranks differ in {k}"
    p_gpu = _psnrs(params0, ring, targets)
    common.PARITY_LOG.append({"name": "dp trainer vs oracle loop", "choices": {str(k): v for k, v in choices.items()},
                              "did_oracle": {str(k): v for k, v in did_cpu.items()},
                              "did_ranks": {str(k): v for k, v in did0.items()},
                              "psnr_start": p0.tolist(), "psnr_after_reset": p_reset.tolist(), "psnr_oracle": p_cpu.tolist(), "psnr_hip": p_gpu.tolist(),
                              "max_abs_psnr_diff_db": float(np.abs(p_gpu - p_cpu).max())})
    for it, want in did_cpu.items():
        got = did0.get(it)
        assert got is not None, f"iteration {it}: the trainer did not densify"
        for key in ("P_before", "cloned", "split", "pruned", "P_after"):
            assert got[key] == want[key], f"iteration {it} {key}: trainer {got} vs oracle loop {want} ({choices[it]})"
    assert sorted(did0) == sorted(did_cpu)
    assert params0["xyz"].shape[0] == raw_cpu["xyz"].shape[0]
    assert p_cpu.mean() > p_reset.mean() + 0.5, \
        f"the oracle loop does not train after the reset ({p_reset.mean():.2f} -> {p_cpu.mean():.2f} dB)"
    np.testing.assert_allclose(p_gpu, p_cpu, atol=PSNR_TOL_DB)
