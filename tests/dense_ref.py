"""Dense differentiable restatement of the rasterizer forward (torch, float64, CPU).

An oracle pin that shares nothing with oracle/gsr_oracle.c: standard-math formulas, float64,
and its OWN per-pixel decisions.  Every (pixel, Gaussian) pair is evaluated densely with the
Gaussians in (depth, index) order; the reference's rules decide which pairs blend
(forward.cu:326-385, backward.cu:552-571):

* tile membership: the Gaussian's rect ceil(3 sqrt(lambda_max)) around its pixel centre
  (forward.cu:236-243, getRect auxiliary.h:45-55) must contain the pixel's 16x16 tile;
* skip if power > 0 or alpha = min(0.99, o exp(power)) < 1/255 (forward.cu:356-365);
* stop BEFORE the Gaussian whose blend would take T (1 - alpha) below 1e-4 -- that Gaussian is
  not blended (forward.cu:366-370);
* n_contrib = tile-list position + 1 of the last blended Gaussian (forward.cu:375-383).

The decisions are made on detached values; the colour is then a smooth function of the inputs
with those decisions fixed, so torch.autograd gives the analytic gradient at the point, and
central finite differences of `dense_render` (decisions re-made at every evaluation) give the
numeric one.  Formulas:
    cov3D = R S^2 R^T,  cov2D = (J W) cov3D (J W)^T + 0.3 I,  conic = cov2D^-1,
    pixel = ((ndc + 1) * size - 1) / 2,  rgb = max(SH(dir) + 0.5, 0),
    C = sum_k c_k a_k T_k + T_final * bg,  invdepth = sum_k a_k T_k / z_k.
"""
import torch

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435]
BLOCK = 16


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
    so the dense pin can reproduce the same rule (aa_quirk=True) or take the exact derivative
    (aa_quirk=False, what finite differences measure)."""

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


def aa_scale_exact(cxx, cyy, cxy):
    det0 = cxx * cyy - cxy * cxy
    det1 = (cxx + 0.3) * (cyy + 0.3) - cxy * cxy
    return torch.sqrt(torch.clamp_min(det0 / det1, 0.000025))


def project(inp, cam, H, W, deg, antialiasing=False, scale_modifier=1.0, aa_quirk=True):
    """Per-Gaussian screen-space quantities (forward.cu:154-272 restated in float64)."""
    V = cam["view"]  # (4,4) as stored: p_view = [p,1] @ V
    Pm = cam["proj"]
    m = inp["means3D"]
    P = m.shape[0]
    mh = torch.cat([m, torch.ones(P, 1, dtype=m.dtype)], 1)
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
        M = R @ torch.diag_embed(scale_modifier * inp["scales"])
        Sig = M @ M.transpose(1, 2)
    tanx, tany = cam["tanfovx"], cam["tanfovy"]
    fx, fy = W / (2.0 * tanx), H / (2.0 * tany)
    tz = t[:, 2]
    tx = torch.clamp(t[:, 0] / tz, -1.3 * tanx, 1.3 * tanx) * tz
    ty = torch.clamp(t[:, 1] / tz, -1.3 * tany, 1.3 * tany) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / (tz * tz)], -1),
                     torch.stack([zero, fy / tz, -fy * ty / (tz * tz)], -1)], -2)  # (P,2,3)
    Tm = J @ V[:3, :3].T  # world->view rotation (math convention)
    cov2 = Tm @ Sig @ Tm.transpose(1, 2)
    cxx, cxy, cyy = cov2[:, 0, 0], cov2[:, 0, 1], cov2[:, 1, 1]
    opac = inp["opacities"][:, 0]
    if antialiasing:
        opac = opac * (RefAAScale.apply(cxx, cyy, cxy) if aa_quirk else aa_scale_exact(cxx, cyy, cxy))
    cxx = cxx + 0.3
    cyy = cyy + 0.3
    det = cxx * cyy - cxy * cxy
    if "colors_precomp" in inp:
        rgb = inp["colors_precomp"]
    else:
        d = m - cam["campos"][None]
        rgb = sh_to_rgb(deg, inp["shs"], d / torch.linalg.norm(d, dim=1, keepdim=True))
    with torch.no_grad():  # extent and culling: decisions, not differentiated
        mid = 0.5 * (cxx + cyy)
        lam = mid + torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3.0 * torch.sqrt(lam))
        gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK

        def tile_lo(p, g):
            return torch.clamp(torch.trunc((p - radius) / BLOCK), 0, g)

        def tile_hi(p, g):
            return torch.clamp(torch.trunc((p + radius + BLOCK - 1) / BLOCK), 0, g)

        rect = torch.stack([tile_lo(px, gx), tile_lo(py, gy), tile_hi(px, gx), tile_hi(py, gy)], 1)
        visible = (tz > 0.2) & (det != 0) & ((rect[:, 2] - rect[:, 0]) * (rect[:, 3] - rect[:, 1]) > 0)
    return {"px": px, "py": py, "ca": cyy / det, "cb": -cxy / det, "cc": cxx / det, "opac": opac, "rgb": rgb,
            "invz": 1.0 / tz, "depth": tz.detach(), "radius": torch.where(visible, radius, 0).to(torch.int64),
            "rect": rect.to(torch.int64), "visible": visible}


def decide(pr, H, W):
    """The reference's per-pixel decisions, made independently in float64 on the dense
    (pixel, Gaussian-in-depth-order) grid.  Returns the depth order, the blend mask (N, K),
    n_contrib (N,) and a per-pixel flag marking decisions within float32 reach of a threshold
    (|alpha - 1/255| or |T (1 - alpha) - 1e-4| relative below 1e-5: a float32 restatement may
    decide those differently)."""
    with torch.no_grad():
        vis = torch.nonzero(pr["visible"])[:, 0]
        # (depth, index) order: stable sort on depth keeps index order on ties
        order = vis[torch.sort(pr["depth"][vis], stable=True).indices]
        N = H * W
        pix = torch.arange(N)
        pxf = (pix % W).to(torch.float64)[:, None]
        pyf = (pix // W).to(torch.float64)[:, None]
        tx = (pix % W) // BLOCK
        ty = (pix // W) // BLOCK
        rect = pr["rect"][order]
        member = ((rect[None, :, 0] <= tx[:, None]) & (tx[:, None] < rect[None, :, 2])
                  & (rect[None, :, 1] <= ty[:, None]) & (ty[:, None] < rect[None, :, 3]))
        dx = pr["px"].detach()[order][None] - pxf
        dy = pr["py"].detach()[order][None] - pyf
        power = (-0.5 * (pr["ca"].detach()[order][None] * dx * dx + pr["cc"].detach()[order][None] * dy * dy)
                 - pr["cb"].detach()[order][None] * dx * dy)
        raw = pr["opac"].detach()[order][None] * torch.exp(power)
        alpha = torch.clamp_max(raw, 0.99)
        allowed = member & ~(power > 0) & ~(alpha < 1.0 / 255.0)
        om = torch.where(allowed, 1.0 - alpha, torch.ones_like(alpha))
        T_before = torch.cumprod(torch.cat([torch.ones(N, 1, dtype=om.dtype), om[:, :-1]], 1), 1)
        test_T = T_before * (1.0 - alpha)
        stops = allowed & (test_T < 1e-4)
        K = order.numel()
        kidx = torch.arange(K)[None].expand(N, K)
        first_stop = torch.where(stops, kidx, torch.full_like(kidx, K)).min(1).values
        blend = allowed & (kidx < first_stop[:, None])
        pos = torch.cumsum(member.to(torch.int64), 1)  # tile-list position + 1
        n_contrib = torch.where(blend, pos, torch.zeros_like(pos)).max(1).values if K else torch.zeros(N, dtype=torch.int64)
        live = member & (kidx <= first_stop[:, None])
        near = live & ((torch.abs(alpha - 1.0 / 255.0) < 1e-5 / 255.0)
                       | (allowed & (torch.abs(test_T - 1e-4) < 1e-9))
                       | (torch.abs(power) < 1e-9))
        tie = near.any(1)
    return order, blend, n_contrib, tie


def dense_render(inp, cam, H, W, deg, bg, antialiasing=False, scale_modifier=1.0, aa_quirk=True):
    """Colour (3,H,W), invdepth (1,H,W) and the decisions, differentiable in every input at
    fixed decisions."""
    pr = project(inp, cam, H, W, deg, antialiasing, scale_modifier, aa_quirk)
    order, blend, n_contrib, tie = decide(pr, H, W)
    N = H * W
    pix = torch.arange(N)
    dtype = inp["means3D"].dtype
    pxf = (pix % W).to(dtype)[:, None]
    pyf = (pix // W).to(dtype)[:, None]
    dx = pr["px"][order][None] - pxf
    dy = pr["py"][order][None] - pyf
    power = -0.5 * (pr["ca"][order][None] * dx * dx + pr["cc"][order][None] * dy * dy) - pr["cb"][order][None] * dx * dy
    alpha = torch.where(blend, torch.clamp_max(pr["opac"][order][None] * torch.exp(power), 0.99),
                        torch.zeros_like(power))
    one_m = 1.0 - alpha
    Tk = torch.cumprod(torch.cat([torch.ones(N, 1, dtype=dtype), one_m[:, :-1]], 1), 1)
    Tfin = torch.prod(one_m, 1)
    w = alpha * Tk
    col = w @ pr["rgb"][order] + Tfin[:, None] * bg[None]
    inv = w @ pr["invz"][order]
    return {"color": col.T.reshape(3, H, W), "invdepth": inv.reshape(1, H, W), "final_T": Tfin.detach(),
            "n_contrib": n_contrib, "tie": tie, "radii": pr["radius"], "alpha_max": alpha.detach().max()}


def loss_of(out, grad_color, grad_invdepth):
    return (out["color"] * grad_color).sum() + (out["invdepth"] * grad_invdepth).sum()


def finite_difference(fn, x, h_rel=1e-6):
    """Central differences of the scalar fn() w.r.t. every element of tensor x (in place)."""
    g = torch.zeros_like(x)
    flat, gf = x.view(-1), g.view(-1)
    with torch.no_grad():
        for i in range(flat.numel()):
            v = float(flat[i])
            h = h_rel * max(1.0, abs(v))
            flat[i] = v + h
            fp = float(fn())
            flat[i] = v - h
            fm = float(fn())
            flat[i] = v
            gf[i] = (fp - fm) / (2.0 * h)
    return g


def ring_cam(cam, dtype=torch.float64):
    return {"view": cam.world_view_transform.to(dtype), "proj": cam.full_proj_transform.to(dtype),
            "campos": cam.camera_center.to(dtype), "tanfovx": cam.tanfovx, "tanfovy": cam.tanfovy}

