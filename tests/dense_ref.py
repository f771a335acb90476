"""Dense differentiable restatement of the rasterizer forward (torch, float64, CPU).

Used only to pin the oracle's analytic backward (backward.cu restated in gsr_oracle.c):
the per-pixel contributor sets (which list entries pass power<=0, alpha>=1/255 and the
T>=1e-4 stop rule) are frozen from the oracle's own float32 forward, then the forward is
re-expressed as a smooth function of the inputs and differentiated by torch.autograd.
Standard-math formulation (not the reference's GLM code), so agreement pins the formulas,
not a transcription:
    cov3D = R S^2 R^T,  cov2D = (J W) cov3D (J W)^T + 0.3 I,  conic = cov2D^-1,
    pixel = ((ndc + 1) * size - 1) / 2,  rgb = max(SH(dir) + 0.5, 0),
    C = sum_k c_k a_k T_k + T_final * bg,  invdepth = sum_k a_k T_k / z_k.
"""
import numpy as np
import torch

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435]


def sh_to_rgb(deg, sh, dirs):
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    r = C0 * sh[:, 0]
    if deg > 0:
        r = r - C1 * y * sh[:, 1] + C1 * z * sh[:, 2] - C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + C2[0] * xy * sh[:, 4] + C2[1] * yz * sh[:, 5] + C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + C2[3] * xz * sh[:, 7] + C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + C3[0] * y * (3 * xx - yy) * sh[:, 9] + C3[1] * xy * z * sh[:, 10]
             + C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + C3[5] * z * (xx - yy) * sh[:, 14]
             + C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return torch.clamp_min(r + 0.5, 0.0)


def quat_to_R(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)


class RefAAScale(torch.autograd.Function):
    """h = sqrt(max(2.5e-5, det(cov2D) / det(cov2D + 0.3 I))) with the reference's backward.

    The reference differentiates det/det' with the textbook formula but evaluates it at the
    already-dilated entries (backward.cu:213-214 add h_var, then :235-245 use them as x, y).
    That is not the exact derivative of its own forward; the oracle restates the reference,
    so the dense pin reproduces the same rule here (the exact derivative would use the
    undilated entries)."""

    @staticmethod
    def forward(ctx, cxx, cyy, cxy):
        det0 = cxx * cyy - cxy * cxy
        det1 = (cxx + 0.3) * (cyy + 0.3) - cxy * cxy
        ratio = det0 / det1
        h = torch.sqrt(torch.clamp_min(ratio, 0.000025))
        ctx.save_for_backward(cxx, cyy, cxy, ratio, h)
        return h

    @staticmethod
    def backward(ctx, gh):
        cxx, cyy, cxy, ratio, h = ctx.saved_tensors
        d_inside_root = torch.where(ratio <= 0.000025, torch.zeros_like(h), gh / (2 * h))
        x, y, z, w = cxx + 0.3, cyy + 0.3, cxy, 0.3
        denom_f = d_inside_root / (w * w + w * (x + y) + x * y - z * z) ** 2
        return (w * (w * y + y * y + z * z) * denom_f, w * (w * x + x * x + z * z) * denom_f,
                -2.0 * w * z * (w + x + y) * denom_f)


def frozen_contributors(o):
    """Per pixel, the ordered Gaussian ids that the oracle blended (float32 decisions)."""
    means2D = o.get("means2D")
    conic = o.get("conic_opacity")
    vals = o.get("vals")
    ranges = o.get("ranges")
    n_contrib = o.get("n_contrib")
    W, H = o.W, o.H
    rows = []
    f32 = np.float32
    for pix in range(W * H):
        px, py = pix % W, pix // W
        t = (py // 16) * ((W + 15) // 16) + (px // 16)
        a = ranges[t][0]
        gid = vals[a:a + n_contrib[pix]]
        if gid.size == 0:
            rows.append([])
            continue
        # float32 element-wise, in the kernel's expression order (forward.cu:353-365)
        dx = means2D[gid, 0] - f32(px)
        dy = means2D[gid, 1] - f32(py)
        co = conic[gid]
        power = f32(-0.5) * (co[:, 0] * dx * dx + co[:, 2] * dy * dy) - co[:, 1] * dx * dy
        alpha = np.minimum(f32(0.99), co[:, 3] * np.exp(power))
        keep = ~(power > 0) & ~(alpha < f32(1.0) / f32(255.0))
        rows.append([int(g) for g in gid[keep]])
    return rows


def dense_forward(inp, cam, H, W, deg, bg, contrib, antialiasing=False, scale_modifier=1.0):
    """inp: dict of float64 tensors (means3D, opacities, shs|colors_precomp, scales+rotations|cov3D_precomp)."""
    V = cam["view"]  # (4,4) as stored: p_view = [p,1] @ V
    Pm = cam["proj"]
    m = inp["means3D"]
    P = m.shape[0]
    ones = torch.ones(P, 1, dtype=m.dtype)
    mh = torch.cat([m, ones], 1)
    t = mh @ V
    ph = mh @ Pm
    pw = 1.0 / (ph[:, 3:4] + 1e-7)
    ndc = ph[:, :2] * pw
    px = ((ndc[:, 0] + 1.0) * W - 1.0) * 0.5
    py = ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5
    if "cov3D_precomp" in inp:
        c = inp["cov3D_precomp"]
        Sig = torch.stack([torch.stack([c[:, 0], c[:, 1], c[:, 2]], -1),
                           torch.stack([c[:, 1], c[:, 3], c[:, 4]], -1),
                           torch.stack([c[:, 2], c[:, 4], c[:, 5]], -1)], -2)
    else:
        R = quat_to_R(inp["rotations"])
        S = torch.diag_embed(scale_modifier * inp["scales"])
        M = R @ S
        Sig = M @ M.transpose(1, 2)
    tanx, tany = cam["tanfovx"], cam["tanfovy"]
    fx = W / (2.0 * tanx)
    fy = H / (2.0 * tany)
    tz = t[:, 2]
    tx = torch.clamp(t[:, 0] / tz, -1.3 * tanx, 1.3 * tanx) * tz
    ty = torch.clamp(t[:, 1] / tz, -1.3 * tany, 1.3 * tany) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / (tz * tz)], -1),
                     torch.stack([zero, fy / tz, -fy * ty / (tz * tz)], -1)], -2)  # (P,2,3)
    Wr = V[:3, :3].T  # world->view rotation (math convention)
    Tm = J @ Wr
    cov2 = Tm @ Sig @ Tm.transpose(1, 2)
    cxx, cxy, cyy = cov2[:, 0, 0], cov2[:, 0, 1], cov2[:, 1, 1]
    opac = inp["opacities"][:, 0]
    if antialiasing:
        opac = opac * RefAAScale.apply(cxx, cyy, cxy)
    cxx = cxx + 0.3
    cyy = cyy + 0.3
    det = cxx * cyy - cxy * cxy
    ca, cb, cc = cyy / det, -cxy / det, cxx / det
    if "colors_precomp" in inp:
        rgb = inp["colors_precomp"]
    else:
        d = m - cam["campos"][None]
        d = d / torch.linalg.norm(d, dim=1, keepdim=True)
        rgb = sh_to_rgb(deg, inp["shs"], d)
    invz = 1.0 / tz

    # ragged contributor lists -> padded (Npix, K)
    K = max(1, max(len(r) for r in contrib))
    N = H * W
    ids = torch.zeros(N, K, dtype=torch.long)
    mask = torch.zeros(N, K, dtype=torch.bool)
    for p, r in enumerate(contrib):
        if r:
            ids[p, :len(r)] = torch.tensor(r)
            mask[p, :len(r)] = True
    pix = torch.arange(N)
    pxf = (pix % W).to(m.dtype)[:, None]
    pyf = (pix // W).to(m.dtype)[:, None]
    dx = px[ids] - pxf
    dy = py[ids] - pyf
    power = -0.5 * (ca[ids] * dx * dx + cc[ids] * dy * dy) - cb[ids] * dx * dy
    alpha = torch.where(mask, opac[ids] * torch.exp(power), torch.zeros_like(power))
    one_m = 1.0 - alpha
    Tk = torch.cumprod(torch.cat([torch.ones(N, 1, dtype=m.dtype), one_m[:, :-1]], 1), 1)
    Tfin = torch.prod(one_m, 1)
    w = alpha * Tk
    col = torch.einsum("nk,nkc->cn", w, rgb[ids]) + Tfin[None] * bg[:, None]
    inv = (w * invz[ids]).sum(1)
    return col.reshape(3, H, W), inv.reshape(1, H, W), alpha
