"""CPU restatement of the reference's SSIM (utils/loss_utils.py:46-86) -- TEST INFRASTRUCTURE
ONLY: imported by tests/ and bench.py's cpu_baseline leg, never by the product.

The reference's fused SSIM is an un-vendored submodule (fused-ssim), and train.py:121-124 falls
back to this PyTorch formulation when it is absent, so this is the definition the drop-in
(csrc/ssim.hip) must reproduce:
  * window: gaussian(11, 1.5) -- exp evaluated in double, stored as float32, normalised in
    float32 (:46-48); 2-D window = outer product in float32 (:50-54);
  * mu = conv2d(img, window, padding=5, groups=C) (zero padding) (:66-67);
  * sigma1_sq = conv2d(img1^2) - mu1^2, sigma2_sq likewise, sigma12 = conv2d(img1 img2) - mu1 mu2
    (:73-75);
  * map = ((2 mu1 mu2 + C1)(2 sigma12 + C2)) / ((mu1^2 + mu2^2 + C1)(sigma1_sq + sigma2_sq + C2)),
    C1 = 0.01^2, C2 = 0.03^2 (:77-80); the loss uses map.mean() (:82-83).
Gradients come from torch.autograd through this restatement (float64 by default).  Parity with
the reference's own execution is UNPINNED: importing the reference to generate fixtures was
refused in this round; tests/test_ssim.py pins this restatement by finite
differences and closed-form cases instead.
"""
from math import exp

import numpy as np
import torch
import torch.nn.functional as F

C1 = 0.01 ** 2
C2 = 0.03 ** 2


def window_1d(window_size=11, sigma=1.5):
    g = torch.tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)],
                     dtype=torch.float32)
    return g / g.sum()


def window_2d(window_size=11):
    w = window_1d(window_size).unsqueeze(1)
    return w.mm(w.t()).float()


def _t(x, dtype):
    return (x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))).to(dtype)


def ssim_map(img1, img2, dtype=torch.float64):
    """SSIM map of (..., H, W) images (numpy or torch), computed in `dtype` on the CPU."""
    a, b = _t(img1, dtype), _t(img2, dtype)
    shape = a.shape
    H, W = shape[-2], shape[-1]
    a4 = a.reshape(-1, 1, H, W)
    b4 = b.reshape(-1, 1, H, W)
    win = window_2d().to(dtype).view(1, 1, 11, 11)

    def conv(t):  # one plane per channel, zero padding
        return F.conv2d(t, win, padding=5)

    mu1, mu2 = conv(a4), conv(b4)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    s11 = conv(a4 * a4) - mu1_sq
    s22 = conv(b4 * b4) - mu2_sq
    s12 = conv(a4 * b4) - mu1_mu2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s11 + s22 + C2))
    return m.reshape(shape)


def ssim_and_grad(img1, img2, dtype=torch.float64, upstream=None):
    """(mean SSIM, d mean / d img1) -- or, with `upstream`, d <upstream, map> / d img1."""
    a = _t(img1, dtype).clone().requires_grad_(True)
    m = ssim_map(a, img2, dtype)
    loss = m.mean() if upstream is None else (m * _t(upstream, dtype)).sum()
    loss.backward()
    return float(m.detach().mean()), a.grad.numpy()
