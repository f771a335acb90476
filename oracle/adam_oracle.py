"""CPU restatement of the visibility-masked Adam step -- TEST INFRASTRUCTURE ONLY: imported by
tests/ and bench.py's cpu_baseline leg, never by the product.

The reference selects it in train.py:37-41 (``from diff_gaussian_rasterization import
SparseGaussianAdam``), builds it in scene/gaussian_model.py:194-196 (``SparseGaussianAdam(l,
lr=0.0, eps=1e-15)``) and steps it in train.py:180-183 (``optimizer.step(radii > 0,
radii.shape[0])``).  The class and its ``_C.adamUpdate`` kernel belong to the accelerated upstream
diff-gaussian-rasterization (graphdeco-inria, the "3dgs_accel" rasterizer the README's 2.7x
training-time claim refers to, README.md:496), which the reference does not vendor -- its own
rasterizer package has no such export.  Restated from that published algorithm:

    for each Gaussian i with visible[i], for each of its M elements j = i*M + k:
        m[j] = b1 m[j] + (1 - b1) g[j]
        v[j] = b2 v[j] + (1 - b2) g[j]^2
        p[j] = p[j] + (-lr m[j] / (sqrt(v[j]) + eps))
    (betas fixed at 0.9 / 0.999 by the Python wrapper; no bias correction; the ``step`` entry of
    the optimizer state is created but never advanced); rows of invisible Gaussians untouched.

No test or fixture in the reference exercises this path: parity is UNPINNED against the
reference's execution; tests/test_adam.py pins this restatement by closed-form first steps.
Arithmetic is float32 in the order written above, as the kernel (csrc/adam.hip) does it.
"""
import numpy as np


def adam_update(param, grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M):
    """In-place update of float32 numpy arrays of N*M elements; visible is a bool array of N."""
    f = np.float32
    lr, b1, b2, eps = f(lr), f(b1), f(b2), f(eps)
    rows = np.repeat(np.asarray(visible, dtype=bool), M)
    g = grad.reshape(-1)[rows]
    m = b1 * exp_avg.reshape(-1)[rows] + (f(1.0) - b1) * g
    v = b2 * exp_avg_sq.reshape(-1)[rows] + (f(1.0) - b2) * g * g
    step = -lr * m / (np.sqrt(v) + eps)
    param.reshape(-1)[rows] = param.reshape(-1)[rows] + step
    exp_avg.reshape(-1)[rows] = m
    exp_avg_sq.reshape(-1)[rows] = v
