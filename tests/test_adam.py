"""Visibility-masked Adam (SparseGaussianAdam / _C.adamUpdate).

CPU: the numpy restatement (oracle/adam_oracle.py) is pinned by closed-form first steps and by a
per-element scalar loop.  GPU (-m gpu): the HIP kernel through the drop-in surface against that
restatement (float32; the kernel and the oracle use the same operation order, so the tolerance
below only covers sqrt/division rounding), for element counts and alignments that take both the
16-byte and the scalar kernel path, plus the train.py usage (render with dc=, backward,
step(radii > 0, N)).  Parity with the reference's own execution is unpinned (no reference test or
fixture covers this path; see the oracle's header).
"""
import numpy as np
import pytest
import torch

import adam_oracle

RTOL = 2e-6  # relative, per element: sqrt / division rounding (fp32)
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _state(N, M, seed):
    r = np.random.default_rng(seed)
    p = r.standard_normal(N * M).astype(np.float32)
    g = r.standard_normal(N * M).astype(np.float32)
    m = (0.1 * r.standard_normal(N * M)).astype(np.float32)
    v = np.abs(0.01 * r.standard_normal(N * M)).astype(np.float32)
    vis = r.random(N) < 0.6
    return p, g, m, v, vis


def test_oracle_first_step_closed_form():
    # from zero moments: m = 0.1 g, v = 0.001 g^2, step = -lr * 0.1 g / (sqrt(0.001) |g| + eps)
    N, M = 5, 3
    g = np.array([1.0, -2.0, 0.5] * N, dtype=np.float32)
    p = np.zeros(N * M, np.float32)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    vis = np.array([True, False, True, True, False])
    adam_oracle.adam_update(p, g, m, v, vis, 0.01, 0.9, 0.999, 1e-15, N, M)
    rows = np.repeat(vis, M)
    expect = -0.01 * 0.1 * g / (np.sqrt(0.001) * np.abs(g))
    # 1 - float32(0.999) = 0.00100004673: the closed form holds to ~5e-5 in float32
    np.testing.assert_allclose(p[rows], expect[rows], rtol=1e-4)
    np.testing.assert_allclose(m[rows], 0.1 * g[rows], rtol=1e-6)
    np.testing.assert_allclose(v[rows], 0.001 * g[rows] ** 2, rtol=1e-4)
    assert not p[~rows].any() and not m[~rows].any() and not v[~rows].any()


def test_oracle_matches_scalar_loop():
    N, M = 37, 4
    p, g, m, v, vis = _state(N, M, 3)
    p0, m0, v0 = p.copy(), m.copy(), v.copy()
    adam_oracle.adam_update(p, g, m, v, vis, 1e-3, 0.9, 0.999, 1e-15, N, M)
    f = np.float32
    for i in range(N):
        for k in range(M):
            j = i * M + k
            if not vis[i]:
                assert p[j] == p0[j] and m[j] == m0[j] and v[j] == v0[j]
                continue
            mm = f(0.9) * m0[j] + (f(1) - f(0.9)) * g[j]
            vv = f(0.999) * v0[j] + (f(1) - f(0.999)) * g[j] * g[j]
            assert m[j] == mm and v[j] == vv
            assert p[j] == p0[j] + (-f(1e-3) * mm / (np.sqrt(vv) + f(1e-15)))


def _dgr():
    import diff_gaussian_rasterization as dgr
    return dgr


@pytest.mark.gpu
@pytest.mark.parametrize("N,M,offset", [(1000, 3, 0), (1000, 4, 0), (999, 45, 0), (1001, 1, 0), (257, 3, 1),
                                        (100003, 3, 0), (0, 3, 0)])
def test_adam_update_matches_oracle(N, M, offset):
    dgr = _dgr()
    p, g, m, v, vis = _state(N, M, N + M)

    def dev(a):  # `offset` floats into a buffer: a 4-byte-aligned start takes the scalar kernel path
        buf = torch.zeros(a.size + offset, dtype=torch.float32, device=DEV)
        t = buf[offset:]
        t.copy_(torch.from_numpy(a))
        return t

    tp, tg, tm, tv = dev(p), dev(g), dev(m), dev(v)
    tvis = torch.from_numpy(vis).to(DEV)
    for _ in range(3):
        dgr._C.adamUpdate(tp, tg, tm, tv, tvis, 1e-3, 0.9, 0.999, 1e-15, N, M)
        adam_oracle.adam_update(p, g, m, v, vis, 1e-3, 0.9, 0.999, 1e-15, N, M)
    torch.cuda.synchronize()
    for got, want in ((tp, p), (tm, m), (tv, v)):
        got = got.cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=RTOL, atol=1e-30)
    rows = np.repeat(~vis, M)
    assert np.array_equal(tp.cpu().numpy()[rows], p[rows])  # invisible rows: untouched, bit for bit


@pytest.mark.gpu
def test_adam_update_rejects_bad_shapes():
    dgr = _dgr()
    t = torch.zeros(12, device=DEV)
    vis = torch.ones(4, dtype=torch.bool, device=DEV)
    with pytest.raises(RuntimeError):
        dgr._C.adamUpdate(t, t, t, t, vis, 1e-3, 0.9, 0.999, 1e-15, 4, 4)  # 12 != 4*4
    with pytest.raises(RuntimeError):
        dgr._C.adamUpdate(t, t, t, t, vis.to(torch.uint8), 1e-3, 0.9, 0.999, 1e-15, 4, 3)


@pytest.mark.gpu
def test_sparse_adam_training_step():
    """train.py:111-183 with SparseGaussianAdam: render(separate_sh) with dc=, L1 loss, backward,
    optimizer.step(radii > 0, N).  Invisible Gaussians keep their parameters bit for bit; visible
    ones move by the oracle's update of their gradient."""
    import common
    dgr = _dgr()
    case = common.make_case(P=2000, H=128, W=160)
    cam, sc = case["cam"], case["scene"]
    params = {
        "xyz": sc["means3D"], "f_dc": sc["shs"][:, :1].contiguous(), "f_rest": sc["shs"][:, 1:].contiguous(),
        "opacity": sc["opacities"], "scaling": sc["scales"], "rotation": sc["rotations"]}
    params = {k: torch.nn.Parameter(v.to(DEV).clone()) for k, v in params.items()}
    lrs = {k: 1e-3 * (i + 1) for i, k in enumerate(params)}  # per-group rates, as the caller's schedule sets them
    opt = dgr.SparseGaussianAdam([{"params": [p], "lr": lrs[k], "name": k} for k, p in params.items()], lr=0.0,
                                 eps=1e-15)
    s = dgr.GaussianRasterizationSettings(case["H"], case["W"], cam.tanfovx, cam.tanfovy, case["bg"].to(DEV), 1.0,
                                          cam.world_view_transform.to(DEV), cam.full_proj_transform.to(DEV), 3,
                                          cam.camera_center.to(DEV), False, False, False)
    means2D = torch.zeros_like(params["xyz"], requires_grad=True)
    color, radii, _ = dgr.GaussianRasterizer(s)(
        means3D=params["xyz"], means2D=means2D, dc=params["f_dc"], shs=params["f_rest"],
        colors_precomp=None, opacities=params["opacity"], scales=params["scaling"], rotations=params["rotation"],
        cov3D_precomp=None)
    target = torch.rand_like(color)
    (color - target).abs().mean().backward()
    before = {k: p.detach().cpu().numpy().copy() for k, p in params.items()}
    grads = {k: p.grad.detach().cpu().numpy().copy() for k, p in params.items()}
    visible = radii > 0
    N = radii.shape[0]
    assert 0 < int(visible.sum()) < N
    opt.step(visible, N)
    opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    vis = visible.cpu().numpy()
    for k, p in params.items():
        M = p.numel() // N
        want = before[k].copy()
        adam_oracle.adam_update(want, grads[k], np.zeros_like(want), np.zeros_like(want), vis, lrs[k], 0.9, 0.999,
                                1e-15, N, M)
        got = p.detach().cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=RTOL, atol=1e-30, err_msg=k)
        assert np.array_equal(got.reshape(N, -1)[~vis], before[k].reshape(N, -1)[~vis]), k
        st = opt.state[p]
        assert set(st) == {"step", "exp_avg", "exp_avg_sq"}


@pytest.mark.gpu
def test_adam_update_groups_one_launch_matches_oracle():
    """Ten groups (more than one launch holds) of mixed widths, rates, epsilons and alignments
    through the multi-group entry point, against the per-group oracle."""
    dgr = _dgr()
    N = 3001
    r = np.random.default_rng(11)
    vis = r.random(N) < 0.5
    tvis = torch.from_numpy(vis).to(DEV)
    groups, host = [], []
    for i, M in enumerate([3, 3, 45, 1, 3, 4, 2, 7, 16, 5]):
        p, g, m, v, _ = _state(N, M, 100 + i)
        off = i % 3
        dev = []
        for a in (p, g, m, v):
            buf = torch.zeros(a.size + off, dtype=torch.float32, device=DEV)
            t = buf[off:]
            t.copy_(torch.from_numpy(a))
            dev.append(t)
        lr, eps = 1e-3 * (i + 1), 1e-15 * (i + 1)
        groups.append((*dev, lr, eps))
        host.append((p, g, m, v, lr, eps, M))
    for _ in range(2):
        dgr._C.adam_update_groups(groups, tvis, 0.9, 0.999, N)
        for p, g, m, v, lr, eps, M in host:
            adam_oracle.adam_update(p, g, m, v, vis, lr, 0.9, 0.999, eps, N, M)
    torch.cuda.synchronize()
    for (tp, _, tm, tv, _, _), (p, _, m, v, _, _, M) in zip(groups, host):
        for got, want in ((tp, p), (tm, m), (tv, v)):
            np.testing.assert_allclose(got.cpu().numpy(), want, rtol=RTOL, atol=1e-30, err_msg=f"M={M}")
