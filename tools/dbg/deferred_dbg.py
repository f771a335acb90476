"""Debug: deferred_backward vs MultiViewRasterizer gradient differences."""
import os, sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (root, os.path.join(root, "gaussian-splatting-npu_amd"), os.path.join(root, "oracle"), os.path.join(root, "tests")):
    sys.path.insert(0, p)
import torch
import test_multiview_rasterizer as t
import diff_gaussian_rasterization as dgr

DEV = t.DEV
case = t._case()
bg = case["bg"].to(DEV)
settings = [t._settings(c, False, bg) for c in case["cams"]]
gc = torch.stack([g[0] for g in case["grads"]]).to(DEV)
gi = torch.stack([g[1] for g in case["grads"]]).to(DEV)
V, P = t.V, t.P

def multi():
    L = t._leaves(case, "sh_scales")
    m2 = torch.zeros((V, P, 3), device=DEV, requires_grad=True)
    c, r, i = dgr.MultiViewRasterizer(settings)(means2D=m2, **L)
    torch.autograd.backward([c, i], [gc, gi])
    torch.cuda.synchronize()
    return {k: v.grad.clone() for k, v in L.items()}

def deferred():
    L = t._leaves(case, "sh_scales")
    m2 = [torch.zeros((P, 3), device=DEV, requires_grad=True) for _ in range(V)]
    with dgr.deferred_backward():
        for v, s in enumerate(settings):
            cv, rv, iv = dgr.GaussianRasterizer(s)(means2D=m2[v], **L)
            torch.autograd.backward([cv, iv], [gc[v], gi[v]])
    torch.cuda.synchronize()
    return {k: v.grad.clone() for k, v in L.items()}

a, a2, b, b2 = multi(), multi(), deferred(), deferred()
for k in a:
    d = lambda x, y: ((x - y).abs().max().item(), (x != y).sum().item())
    print(k, "multi-multi", d(a[k], a2[k]), "def-def", d(b[k], b2[k]), "multi-def", d(a[k], b[k]), "max", a[k].abs().max().item())

# C-level: the same forward state through backward_views and through render + preprocess_views
from diff_gaussian_rasterization import _C
L = t._leaves(case, "sh_scales")
colors = torch.empty((V, 3, t.H, t.W), device=DEV); radii = torch.empty((V, P), dtype=torch.int32, device=DEV)
inv = torch.empty((V, 1, t.H, t.W), device=DEV)
s0 = settings[0]
Ls, geoms, bins, imgs = _C.rasterize_gaussians_views(
    s0.bg, L["means3D"].detach(), torch.Tensor([]), L["opacities"].detach(), L["scales"].detach(), L["rotations"].detach(), 1.0,
    torch.Tensor([]), [s.viewmatrix for s in settings], [s.projmatrix for s in settings], [s.tanfovx for s in settings],
    [s.tanfovy for s in settings], t.H, t.W, L["shs"].detach(), 3, [s.campos for s in settings], False, False, False,
    out=(colors, radii, inv))
args = (L["means3D"].detach(), [radii[v] for v in range(V)], torch.Tensor([]), L["opacities"].detach(), L["scales"].detach(),
        L["rotations"].detach(), 1.0, torch.Tensor([]), [s.viewmatrix for s in settings], [s.projmatrix for s in settings],
        [s.tanfovx for s in settings], [s.tanfovy for s in settings])
ga = _C.rasterize_gaussians_backward_views(s0.bg, *args, gc, gi, L["shs"].detach(), 3, [s.campos for s in settings],
                                           geoms, Ls, bins, imgs, False, False)
torch.cuda.synchronize()
for v in range(V):
    _C.rasterize_gaussians_render_backward(s0.bg, P, Ls[v], geoms[v], bins[v], imgs[v], gc[v], gi[v], False)
gb = _C.rasterize_gaussians_preprocess_backward_views(*args, t.H, t.W, L["shs"].detach(), 3, [s.campos for s in settings],
                                                      geoms, Ls, bins, True, False, False)
torch.cuda.synchronize()
for j, (x, y) in enumerate(zip(ga, gb)):
    if x is not None:
        print("C-level", j, (x - y).abs().max().item(), (x != y).sum().item())
