""""PSNR vs ref" on reference-held real images: train.py on the NeRF-synthetic chair (needs an MI355X).

BASELINE's metric pairs the rasterizer's throughput with "PSNR vs ref".  The Mip-NeRF360 scenes of
configs 3/5 are absent offline; the reference does hold the NeRF-synthetic chair (points3d.ply and
its train / test images), so this test trains on those, the way train.py does, twice:
  * GPU: the drop-ins train.py takes with `--optimizer_type sparse_adam` -- GaussianRasterizer with
    dc= / shs= (gaussian_renderer/__init__.py:82-100), fused_ssim, SparseGaussianAdam -- all HIP;
  * CPU: the oracles -- oracle/gsr_oracle.c forward + backward, oracle/ssim_oracle.py,
    oracle/adam_oracle.py;
and evaluates both on held-out test views with training_report's PSNR (train.py:214-252,
utils/image_utils.py:17-19).

What is restated from the reference (not imported):
  * data: tests/golden/chair/chair_frames.npz (make_chair_images.py): 25 training and 8 test frames
    (the dataset's PNG files), loaded at `-r 4` (200 x 200) as loadCam / Camera / PILtoTorch do:
    original_image = the RGB channels of the resized RGBA frame, alpha_mask = its alpha
    (utils/camera_utils.py:20-66,
    scene/cameras.py:40-47); black background (ModelParams white_background default False);
  * initialisation: create_from_pcd on the dataset's points3d.ply (tests/golden/chair/
    nerf_chair.npz, gaussian_model.py:149-176): SH degree 3 stored, active degree 0 (it rises
    every 1000 iterations, train.py:95-96: never within this run);
  * the iteration (train.py:97-183): xyz learning rate from get_expon_lr_func (general_utils.py:
    29-60) with spatial_lr_scale = cameras_extent (gaussian_model.py:178-192,
    update_learning_rate), the camera picked by popping a random index from a refilled stack
    (train.py:101-107; random.Random(SEED) here, the same sequence for both loops), render,
    image *= alpha_mask, loss = 0.8 L1 + 0.2 (1 - SSIM), backward, SparseGaussianAdam.step(radii > 0,
    P) with betas (0.9, 0.999) and eps 1e-15.  Densification starts at iteration 500 (densify_from_iter)
    and is not reached; the exposure optimiser does not touch the render without train_test_exp.
Asserted: the oracle loop trains (masked test PSNR up by > 0.5 dB); the two loops' test PSNRs (each
loop's final parameters rendered by the oracle) agree within PSNR_TOL_DB on the mean over the test
views (the figure training_report prints) and within PSNR_VIEW_TOL_DB per view; the HIP render of
the GPU loop's parameters gives the same PSNR as the oracle's render of them within 0.01 dB.
Why a per-view bound above the mean's: 200 iterations of training amplify float32 rounding
differences (a chaotic trajectory), and the oracle loop is itself not reproducible -- its render
backward adds the tiles' sums into the per-Gaussian gradients with OpenMP atomics in whatever order
the threads reach them, as the reference's CUDA atomics do (backward.cu:593-635).  The test runs
the oracle loop twice and logs that run-to-run spread beside the HIP-vs-oracle differences.
The absolute PSNRs go to the parity statistics (gpurun_out/parity_stats.json).
"""
import math
import os
import random

import numpy as np
import pytest
import torch

import adam_oracle
import common
import nerf_synthetic as ns
import oracle
import ssim_oracle

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
HERE = os.path.dirname(os.path.abspath(__file__))
FRAMES = os.path.join(HERE, "golden", "chair", "chair_frames.npz")  # the dataset's PNG files + cameras
CLOUD = os.path.join(HERE, "golden", "chair", "nerf_chair.npz")
ITERS = 200
RES = 200        # train.py -r 4 (the oracle loop's cost grows with the pixels)
LONG_RES = 800   # the dataset's resolution (train.py's default -r for 800-pixel frames)
SEED = 0
SH_MAX, SH_ACTIVE = 3, 0
PSNR_TOL_DB = 0.05       # mean over the 8 test views
PSNR_VIEW_TOL_DB = 0.15  # any one view (see the module docstring)
THREADS = min(16, os.cpu_count() or 1)
# OptimizationParams (arguments/__init__.py:74-100)
POS_LR_INIT, POS_LR_FINAL, POS_LR_DELAY_MULT, POS_LR_MAX_STEPS = 0.00016, 0.0000016, 0.01, 30_000
LR = {"f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005, "rotation": 0.001}
LAMBDA_DSSIM = 0.2


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:29-60"""
    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        return delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
    return helper


class View:
    """A loaded camera (utils/camera_utils.py:20-66 loadCam at `-r 800 // res`, scene/cameras.py:40-47):
    the matrices from the fixture; original_image and alpha_mask from PILtoTorch of the PNG frame
    (utils/general_utils.py:21-27: PIL resize with its default filter, / 255)."""

    def __init__(self, f, split, i, res):
        import io
        from PIL import Image
        self.world_view_transform = torch.from_numpy(f[f"{split}_viewmatrix"][i].copy())
        self.full_proj_transform = torch.from_numpy(f[f"{split}_projmatrix"][i].copy())
        self.camera_center = torch.from_numpy(f[f"{split}_campos"][i].copy())
        self.tanfovx, self.tanfovy = (float(x) for x in f[f"{split}_tanfov"][i])
        o = f[f"{split}_png_offsets"]
        image = Image.open(io.BytesIO(f[f"{split}_png"][o[i]:o[i + 1]].tobytes()))
        rgba = torch.from_numpy(np.array(image.resize((res, res)))) / 255.0  # PILtoTorch
        rgba = rgba.permute(2, 0, 1)
        self.original_image = rgba[:3].clamp(0.0, 1.0).contiguous()
        self.alpha_mask = rgba[3:4].contiguous()
        self.H, self.W = self.original_image.shape[1:]


def _load(res):
    f = dict(np.load(FRAMES))
    c = dict(np.load(CLOUD))
    train = [View(f, "train", i, res) for i in range(len(f["train_frames"]))]
    test = [View(f, "test", i, res) for i in range(len(f["test_frames"]))]
    # create_from_pcd (gaussian_model.py:149-176), raw (pre-activation) parameters; the activated
    # scale / opacity as stored in the cloud fixture, so both loops start from the same bits
    scene = ns.initial_gaussians(c["xyz"], c["rgb"], c["dist2"], scale=c["scale"], opacity=c["opacity"])
    P = scene["means3D"].shape[0]
    raw = {"xyz": scene["means3D"].clone(), "f_dc": scene["shs"][:, :1].clone(),
           "f_rest": scene["shs"][:, 1:].clone(), "opacity": torch.logit(scene["opacities"]),
           "scaling": torch.log(scene["scales"]), "rotation": scene["rotations"].clone()}
    return train, test, {k: v.contiguous().float() for k, v in raw.items()}, float(f["extent"]), P


def _activate(raw):
    """gaussian_model.py:111-135 getters"""
    return {"means3D": raw["xyz"], "dc": raw["f_dc"], "rest": raw["f_rest"],
            "opacities": torch.sigmoid(raw["opacity"]), "scales": torch.exp(raw["scaling"]),
            "rotations": torch.nn.functional.normalize(raw["rotation"], dim=1)}


def _schedule(n_train):
    """train.py:101-107: pop a random index from a stack refilled with every training view."""
    rng = random.Random(SEED)
    stack, order = [], []
    for _ in range(ITERS):
        if not stack:
            stack = list(range(n_train))
        order.append(stack.pop(rng.randint(0, len(stack) - 1)))
    return order


def _oracle_render(act, v, sh_degree=SH_ACTIVE):
    shs = torch.cat([act["dc"], act["rest"]], dim=1).detach()
    return oracle.OracleRaster(act["means3D"].detach(), act["opacities"].detach(), torch.zeros(3),
                               v.world_view_transform, v.full_proj_transform, v.camera_center, v.tanfovx, v.tanfovy,
                               v.H, v.W, shs=shs, sh_degree=sh_degree, scales=act["scales"].detach(),
                               rotations=act["rotations"].detach(), nthreads=THREADS)


def _psnr(img, gt):
    """utils/image_utils.py:17-19 on clamp(render, 0, 1) vs clamp(original_image, 0, 1)"""
    a = np.clip(np.asarray(img, np.float64), 0, 1)
    b = np.clip(np.asarray(gt, np.float64), 0, 1)
    return 20.0 * math.log10(1.0 / math.sqrt(((a - b) ** 2).mean()))


def _test_psnrs(raw, test):
    """(training_report's PSNR of every test view, the PSNR of the render x alpha_mask -- the image the
    training loss compares, train.py:119-121 -- of every test view)"""
    act = _activate(raw)
    full, masked = [], []
    for v in test:
        c = _oracle_render(act, v).color
        full.append(_psnr(c, v.original_image.numpy()))
        masked.append(_psnr(c * v.alpha_mask.numpy(), v.original_image.numpy()))
    return np.array(full), np.array(masked)


def _train_cpu(raw, train, extent, P):
    xyz_lr = get_expon_lr_func(POS_LR_INIT * extent, POS_LR_FINAL * extent, lr_delay_mult=POS_LR_DELAY_MULT,
                               max_steps=POS_LR_MAX_STEPS)
    raw = {k: v.clone().requires_grad_(True) for k, v in raw.items()}
    state = {k: (np.zeros(v.numel(), np.float32), np.zeros(v.numel(), np.float32)) for k, v in raw.items()}
    for it, vi in enumerate(_schedule(len(train)), start=1):
        v = train[vi]
        lr = dict(LR, xyz=xyz_lr(it))
        act = _activate(raw)
        o = _oracle_render(act, v)
        img = torch.from_numpy(o.color.copy()).requires_grad_(True)
        image = img.clamp(0, 1) * v.alpha_mask  # gaussian_renderer/__init__.py:119, train.py:119-121
        ssim = ssim_oracle.ssim_map(image[None], v.original_image[None], dtype=torch.float32).mean()
        loss = (1.0 - LAMBDA_DSSIM) * (image - v.original_image).abs().mean() + LAMBDA_DSSIM * (1.0 - ssim)
        loss.backward()
        g = o.backward(img.grad.numpy(), tile_sums=True)
        dsh = torch.from_numpy(g["dL_dsh"]).reshape(P, (SH_MAX + 1) ** 2, 3)
        torch.autograd.backward(
            [act["means3D"], act["dc"], act["rest"], act["opacities"], act["scales"], act["rotations"]],
            [torch.from_numpy(g["dL_dmeans3D"]), dsh[:, :1], dsh[:, 1:], torch.from_numpy(g["dL_dopacity"]),
             torch.from_numpy(g["dL_dscales"]), torch.from_numpy(g["dL_drotations"])])
        vis = o.radii > 0
        with torch.no_grad():
            for k, p in raw.items():
                pa = p.detach().numpy().reshape(-1)  # shares storage with p
                m, s = state[k]
                adam_oracle.adam_update(pa, p.grad.numpy().reshape(-1).copy(), m, s, vis, lr[k], 0.9, 0.999, 1e-15,
                                        P, p.numel() // P)
                p.grad = None
    return {k: v.detach() for k, v in raw.items()}


def _settings(dgr, v, sh_degree=SH_ACTIVE):
    return dgr.GaussianRasterizationSettings(v.H, v.W, v.tanfovx, v.tanfovy, torch.zeros(3, device=DEV), 1.0,
                                             v.world_view_transform.to(DEV), v.full_proj_transform.to(DEV),
                                             sh_degree, v.camera_center.to(DEV), False, False, False)


def _train_gpu(raw, train, extent, P):
    import diff_gaussian_rasterization as dgr
    from fused_ssim import fused_ssim
    xyz_lr = get_expon_lr_func(POS_LR_INIT * extent, POS_LR_FINAL * extent, lr_delay_mult=POS_LR_DELAY_MULT,
                               max_steps=POS_LR_MAX_STEPS)
    raw = {k: torch.nn.Parameter(v.to(DEV).clone()) for k, v in raw.items()}
    opt = dgr.SparseGaussianAdam([{"params": [raw["xyz"]], "lr": xyz_lr(0), "name": "xyz"}] +
                                 [{"params": [raw[k]], "lr": LR[k], "name": k} for k in LR], lr=0.0, eps=1e-15)
    settings = [_settings(dgr, v) for v in train]
    gts = [v.original_image.to(DEV) for v in train]
    masks = [v.alpha_mask.to(DEV) for v in train]
    for it, vi in enumerate(_schedule(len(train)), start=1):
        for group in opt.param_groups:  # gaussian_model.update_learning_rate
            if group["name"] == "xyz":
                group["lr"] = xyz_lr(it)
        act = _activate(raw)
        means2D = torch.zeros_like(act["means3D"], requires_grad=True)
        img, radii, _ = dgr.GaussianRasterizer(settings[vi])(
            means3D=act["means3D"], means2D=means2D, dc=act["dc"], shs=act["rest"], colors_precomp=None,
            opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"], cov3D_precomp=None)
        image = img.clamp(0, 1) * masks[vi]
        gt = gts[vi]
        loss = (1.0 - LAMBDA_DSSIM) * (image - gt).abs().mean() + LAMBDA_DSSIM * (1.0 - fused_ssim(image[None],
                                                                                                 gt[None]))
        loss.backward()
        opt.step(radii > 0, P)
        opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    return {k: v.detach() for k, v in raw.items()}


def test_chair_training_psnr_matches_oracle_loop():
    import diff_gaussian_rasterization as dgr
    train, test, raw0, extent, P = _load(RES)
    assert len(train) == 25 and len(test) == 8 and P == 100_000
    (f0, m0) = _test_psnrs(raw0, test)
    raw_cpu = _train_cpu(raw0, train, extent, P)
    f_cpu, m_cpu = _test_psnrs(raw_cpu, test)
    f_cpu2, m_cpu2 = _test_psnrs(_train_cpu(raw0, train, extent, P), test)  # the oracle loop's own spread
    raw_gpu = _train_gpu(raw0, train, extent, P)
    f_gpu, m_gpu = _test_psnrs({k: v.cpu() for k, v in raw_gpu.items()}, test)
    # the HIP render of the GPU loop's parameters, as training_report would evaluate them
    f_hip, m_hip = _hip_test_psnrs(dgr, _activate(raw_gpu), test, SH_ACTIVE)
    stats = {"name": "chair training PSNR (8 test views, 200x200, 100k Gaussians)", "iterations": ITERS,
             "psnr_start": float(f0.mean()), "psnr_oracle_loop": float(f_cpu.mean()),
             "psnr_hip_loop": float(f_gpu.mean()), "psnr_hip_loop_hip_render": float(f_hip.mean()),
             "masked_psnr_start": float(m0.mean()), "masked_psnr_oracle_loop": float(m_cpu.mean()),
             "masked_psnr_hip_loop": float(m_gpu.mean()), "masked_psnr_hip_loop_hip_render": float(m_hip.mean()),
             "max_view_diff_db": float(max(np.abs(f_gpu - f_cpu).max(), np.abs(m_gpu - m_cpu).max())),
             "mean_diff_db": float(max(abs(f_gpu.mean() - f_cpu.mean()), abs(m_gpu.mean() - m_cpu.mean()))),
             "oracle_rerun_max_view_diff_db": float(max(np.abs(f_cpu2 - f_cpu).max(), np.abs(m_cpu2 - m_cpu).max())),
             "oracle_rerun_mean_diff_db": float(max(abs(f_cpu2.mean() - f_cpu.mean()),
                                                    abs(m_cpu2.mean() - m_cpu.mean()))),
             "per_view_oracle_loop": f_cpu.round(4).tolist(), "per_view_hip_loop": f_gpu.round(4).tolist(),
             "per_view_masked_oracle_loop": m_cpu.round(4).tolist(),
             "per_view_masked_hip_loop": m_gpu.round(4).tolist()}
    common.PARITY_LOG.append(stats)
    print(stats)
    # the loss only sees render x alpha_mask: the masked PSNR rises, training_report's unmasked one
    # need not in 200 iterations (the create_from_pcd haze outside the object gets no gradient)
    assert m_cpu.mean() > m0.mean() + 0.5, "the oracle loop does not train"
    assert abs(f_gpu.mean() - f_cpu.mean()) <= PSNR_TOL_DB
    assert abs(m_gpu.mean() - m_cpu.mean()) <= PSNR_TOL_DB
    np.testing.assert_allclose(f_gpu, f_cpu, atol=PSNR_VIEW_TOL_DB)
    np.testing.assert_allclose(m_gpu, m_cpu, atol=PSNR_VIEW_TOL_DB)
    np.testing.assert_allclose(f_hip, f_gpu, atol=0.01)
    np.testing.assert_allclose(m_hip, m_gpu, atol=0.01)


def _hip_test_psnrs(dgr, act, test, sh_degree):
    full, masked = [], []
    with torch.no_grad():
        for v in test:
            img, _, _ = dgr.GaussianRasterizer(_settings(dgr, v, sh_degree))(
                means3D=act["means3D"], means2D=torch.zeros_like(act["means3D"]), dc=act["dc"], shs=act["rest"],
                colors_precomp=None, opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"],
                cov3D_precomp=None)
            c = img.clamp(0, 1).cpu().numpy()
            full.append(_psnr(c, v.original_image.numpy()))
            masked.append(_psnr(c * v.alpha_mask.numpy(), v.original_image.numpy()))
    return np.array(full), np.array(masked)


LONG_ITERS = 7000  # train.py's first testing iteration (--test_iterations default 7000 30000)
REPORT_AT = (1000, 3000, 5000, 7000)


def test_chair_train_py_hip_long():
    """train.py's loop on the HIP drop-ins at the frames' 800 x 800 up to its first test iteration
    (multiview.DataParallelTrainer in one process: train.py:93-186 with densify_and_prune every 100
    iterations from 500, reset_opacity every 3000, oneupSHdegree every 1000): training_report's PSNR
    and the masked PSNR of the 8 test views at REPORT_AT go to the parity statistics.  No oracle loop
    (hours on the host); asserted: the masked PSNR rises and densification changes the model."""
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import multiview
    train, test, raw0, extent, P0 = _load(LONG_RES)
    trainer = multiview.DataParallelTrainer({k: v.to(DEV) for k, v in raw0.items()}, optimizer="sparse_adam",
                                            spatial_lr_scale=extent, seed=SEED)
    views_by_degree = {d: [(_settings(dgr, v, d), v.original_image.to(DEV), {"alpha_mask": v.alpha_mask.to(DEV)})
                           for v in train] for d in range(SH_MAX + 1)}
    with torch.no_grad():
        f_start, m_start = _hip_test_psnrs(dgr, _activate(trainer.params), test, 0)
    order = random.Random(SEED)
    stack, report = [], []
    for it in range(1, LONG_ITERS + 1):
        degree = min(it // 1000, SH_MAX)  # oneupSHdegree at every 1000th iteration, before its render
        if not stack:
            stack = list(range(len(train)))
        vi = stack.pop(order.randint(0, len(stack) - 1))
        trainer.iteration(it, [views_by_degree[degree][vi]], extent)
        if it in REPORT_AT:
            with torch.no_grad():
                f, m = _hip_test_psnrs(dgr, _activate(trainer.params), test, degree)
            report.append({"iteration": it, "P": int(trainer.P), "psnr": round(float(f.mean()), 4),
                           "masked_psnr": round(float(m.mean()), 4)})
    stats = {"name": "chair train.py loop on the HIP drop-ins (8 test views, 800x800)", "P_start": P0,
             "psnr_start": round(float(f_start.mean()), 4), "masked_psnr_start": round(float(m_start.mean()), 4),
             "report": report}
    common.PARITY_LOG.append(stats)
    print(stats)
    assert report[-1]["masked_psnr"] > stats["masked_psnr_start"] + 2.0
    assert report[-1]["P"] != P0  # densification ran
