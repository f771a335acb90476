"""Fused SSIM (the fused_ssim drop-in and diff_gaussian_rasterization._C.fusedssim*) against its
restatement.

The reference's fused-ssim submodule is not vendored; train.py:121-124 falls back to the
reference's PyTorch ssim (utils/loss_utils.py:56-86), which oracle/ssim_oracle.py restates.
CPU tests pin the restatement (SSIM(x, x) = 1, the closed form on constant images, autograd vs
central finite differences in float64); GPU tests compare the HIP map and dL/dimg1 with it
(float32 kernels vs the float64 restatement: mean SSIM within 2e-6, gradients within 1e-4 of
their largest element) on odd, batched and full-HD sizes with both paddings.  Parity with the
reference's own execution is unpinned.
"""
import numpy as np
import pytest
import torch

import ssim_oracle as so


def _pair(shape, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.rand(shape, generator=g)
    b = (a + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)
    return a, b


def test_window_is_the_reference_gaussian():
    w = so.window_1d().double()
    x = torch.arange(11, dtype=torch.float64) - 5
    ref = torch.exp(-x * x / 4.5)
    ref /= ref.sum()
    assert torch.allclose(w, ref, atol=1e-7) and abs(float(w.sum()) - 1.0) < 1e-6


def test_self_similarity_is_one():
    a, _ = _pair((3, 40, 50), 0)
    m = so.ssim_map(a, a)
    assert torch.allclose(m, torch.ones_like(m), atol=1e-12)


def test_constant_images_closed_form():
    a = torch.full((1, 40, 40), 0.3)
    b = torch.full((1, 40, 40), 0.7)
    m = so.ssim_map(a, b)[0, 10:30, 10:30]  # the window lies inside the image
    expect = (2 * 0.3 * 0.7 + so.C1) / (0.3 ** 2 + 0.7 ** 2 + so.C1)
    assert torch.allclose(m, torch.full_like(m, expect), atol=1e-5)


def test_gradient_matches_finite_differences():
    a, b = _pair((2, 24, 28), 1)
    a64 = a.double()
    _, g = so.ssim_and_grad(a64, b)
    rng = np.random.default_rng(0)
    eps = 1e-6
    for _ in range(16):
        c, y, x = int(rng.integers(0, 2)), int(rng.integers(0, 24)), int(rng.integers(0, 28))
        ap, am = a64.clone(), a64.clone()
        ap[c, y, x] += eps
        am[c, y, x] -= eps
        fd = float(so.ssim_map(ap, b).mean() - so.ssim_map(am, b).mean()) / (2 * eps)
        assert abs(fd - g[c, y, x]) <= 1e-4 * np.abs(g).max() + 1e-12


GPU_CASES = [((3, 64, 80), 2), ((1, 3, 50, 70), 3), ((3, 37, 29), 4), ((2, 3, 33, 65), 5)]


@pytest.mark.gpu
@pytest.mark.parametrize("padding", ["same", "valid"])
@pytest.mark.parametrize("shape,seed", GPU_CASES, ids=[str(c[0]) for c in GPU_CASES])
def test_hip_matches_oracle(shape, seed, padding):
    from fused_ssim import fused_ssim  # the reference's import (train.py:31-35)
    a, b = _pair(shape, seed)
    x = a.cuda().requires_grad_(True)
    v = fused_ssim(x, b.cuda(), padding=padding)
    v.backward()
    a64 = a.double().requires_grad_(True)
    m = so.ssim_map(a64, b)
    if padding == "valid":
        m = m[..., 5:-5, 5:-5]
    ref = m.mean()
    ref.backward()
    assert abs(float(v.detach()) - float(ref.detach())) < 2e-6
    g, r = x.grad.cpu().numpy(), a64.grad.numpy()
    assert np.abs(g - r).max() <= 1e-4 * np.abs(r).max() + 1e-12


@pytest.mark.gpu
def test_hip_full_hd_map_and_upstream_gradient():
    from fused_ssim import fusedssim, fusedssim_backward
    a, b = _pair((3, 1080, 1920), 6)
    up = torch.randn(a.shape, generator=torch.Generator().manual_seed(7))
    m, dA, dB, dC = fusedssim(so.C1, so.C2, a.cuda(), b.cuda(), True)
    grad = fusedssim_backward(so.C1, so.C2, a.cuda(), b.cuda(), up.cuda(), dA, dB, dC)
    ref_map = so.ssim_map(a, b)
    assert float((m.cpu().double() - ref_map).abs().max()) < 1e-5
    _, rg = so.ssim_and_grad(a, b, upstream=up)
    g = grad.cpu().numpy()
    assert np.abs(g - rg).max() <= 1e-4 * np.abs(rg).max() + 1e-12


@pytest.mark.gpu
def test_dr_aa_ops_and_train_loss():
    """utils/loss_utils.py:17-38 (fusedssim / fusedssim_backward from _C) and the train.py:121-126
    loss (1 - lambda) L1 + lambda (1 - fused_ssim(image, gt)) with lambda_dssim = 0.2."""
    import diff_gaussian_rasterization._C as C
    from fused_ssim import fused_ssim
    a, b = _pair((3, 70, 90), 8)
    ac, bc = a.cuda(), b.cuda()
    m = C.fusedssim(so.C1, so.C2, ac, bc)
    assert float((m.cpu().double() - so.ssim_map(a, b)).abs().max()) < 1e-5
    up = torch.ones_like(ac) / ac.numel()
    g = C.fusedssim_backward(so.C1, so.C2, ac, bc, up)
    _, rg = so.ssim_and_grad(a, b)
    assert np.abs(g.cpu().numpy() - rg).max() <= 1e-4 * np.abs(rg).max()
    img = ac.clone().requires_grad_(True)
    loss = 0.8 * (img - bc).abs().mean() + 0.2 * (1.0 - fused_ssim(img.unsqueeze(0), bc.unsqueeze(0)))
    loss.backward()
    a64 = a.double().requires_grad_(True)
    ref = 0.8 * (a64 - b.double()).abs().mean() + 0.2 * (1.0 - so.ssim_map(a64, b).mean())
    ref.backward()
    assert abs(float(loss.detach()) - float(ref.detach())) < 2e-6
    assert np.abs(img.grad.cpu().numpy() - a64.grad.numpy()).max() <= 1e-4 * np.abs(a64.grad.numpy()).max()


@pytest.mark.gpu
def test_hip_rejects_cpu_tensor():
    from fused_ssim import fused_ssim
    with pytest.raises(RuntimeError, match="GPU only"):
        fused_ssim(torch.zeros(1, 3, 8, 8), torch.zeros(1, 3, 8, 8))
