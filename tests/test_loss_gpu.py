"""The training loss fused into the render kernels (core/models.py:133-167) against its torch
restatement on the same render outputs, and its gradient against the unfused path (render, then the loss in torch,
then autograd into the render backward).

Tolerances: loss terms 1e-5 relative (double-accumulated per-tile sums vs torch's fp32 mean); d_gaussians per
parameter group within 1e-4 relative L2 of the unfused path (the seeds round differently, then float-atomic
ordering), the repo's gradient bar."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from lgm_amd import GaussianRenderer, Options
from lgm_amd.cameras import orbit_cameras
from lgm_amd.synthetic import synthetic_gaussians
from tests.render_cases import rel_l2

pytestmark = pytest.mark.gpu
GROUPS = {"mean": slice(0, 3), "opacity": slice(3, 4), "scale": slice(4, 7), "rot": slice(7, 11), "rgb": slice(11, 14)}


def _reference_loss(image, alpha, gt, mask, bg):
    """core/models.py:145-148,165-167 on the render outputs."""
    gt_c = gt * mask + bg.view(1, 1, 3, 1, 1) * (1 - mask)
    loss = F.mse_loss(image, gt_c) + F.mse_loss(alpha, mask)
    psnr = -10 * torch.log10(torch.mean((image.detach() - gt_c) ** 2))
    return loss, psnr, F.mse_loss(image, gt_c), F.mse_loss(alpha, mask)


def _case(B, V, N, S, seed):
    gen = torch.Generator().manual_seed(seed)
    g = synthetic_gaussians(B, N, seed=seed)
    cv, cvp, cp = orbit_cameras(V)
    cv, cvp, cp = (t[None].expand(B, *t.shape).contiguous() for t in (cv, cvp, cp))
    gt = torch.rand(B, V, 3, S, S, generator=gen)
    mask = (torch.rand(B, V, 1, S, S, generator=gen) > 0.4).float()
    bg = torch.rand(3, generator=gen)
    w_img = torch.randn(B, V, 3, S, S, generator=gen)  # an extra loss on the image (LPIPS stands in for it)
    w_a = torch.randn(B, V, 1, S, S, generator=gen)
    return g, cv, cvp, cp, gt, mask, bg, w_img, w_a


@pytest.mark.parametrize("B,V,N,S,extra", [(1, 2, 3000, 64, False), (2, 3, 5000, 96, True),
                                           (1, 6, 100_000, 256, False), (1, 6, 100_000, 256, True)])
def test_fused_loss_matches_torch(cuda, B, V, N, S, extra):
    g, cv, cvp, cp, gt, mask, bg, w_img, w_a = (t.to(cuda) for t in _case(B, V, N, S, seed=N + S))
    r = GaussianRenderer(Options(output_size=S))
    # fused
    gf = g.clone().requires_grad_(True)
    out = r.render(gf, cv, cvp, cp, bg_color=bg, gt_images=gt, gt_masks=mask)
    total = out["loss_mse"] + 0.5 * out["mse_image"] + 0.25 * out["mse_alpha"]
    if extra:
        total = total + 1e-4 * ((out["image"] * w_img).sum() + (out["alpha"] * w_a).sum())
    total.backward()
    # unfused: the same render, the loss in torch
    gu = g.clone().requires_grad_(True)
    ou = r.render(gu, cv, cvp, cp, bg_color=bg)
    loss, psnr, mi, ma = _reference_loss(ou["image"], ou["alpha"], gt, mask, bg)
    tu = loss + 0.5 * mi + 0.25 * ma
    if extra:
        tu = tu + 1e-4 * ((ou["image"] * w_img).sum() + (ou["alpha"] * w_a).sum())
    tu.backward()
    torch.cuda.synchronize()
    assert torch.equal(out["image"], ou["image"]) and torch.equal(out["alpha"], ou["alpha"])
    for k, ref in (("loss_mse", loss), ("mse_image", mi), ("mse_alpha", ma), ("psnr", psnr)):
        a, b = float(out[k]), float(ref)
        assert abs(a - b) <= 1e-5 * abs(b), (k, a, b)
    dgf, dgu = gf.grad.cpu().numpy(), gu.grad.cpu().numpy()
    for name, sl in GROUPS.items():
        e = rel_l2(dgf[..., sl], dgu[..., sl])
        assert e < 1e-4, f"d_{name}: {e:.3e}"


def test_fused_loss_psnr_gradient(cuda):
    """psnr is differentiable here (the reference computes it under no_grad): d psnr = -10 / (ln 10 mse) d mse."""
    from lgm_amd.gs import rasterize
    g, cv, cvp, cp, gt, mask, bg, _, _ = (t.to(cuda) for t in _case(1, 2, 2000, 64, seed=5))
    tan = float(GaussianRenderer(Options(output_size=64)).tan_half_fov)
    ga = g.clone().requires_grad_(True)
    o4 = rasterize(ga, cv, cvp, bg, tan, tan, 64, 64, clamp=True, gt_images=gt, gt_masks=mask)[3]
    (o4[1] * (-10.0 / np.log(10.0) / float(o4[1]))).backward()
    gb = g.clone().requires_grad_(True)
    o4b = rasterize(gb, cv, cvp, bg, tan, tan, 64, 64, clamp=True, gt_images=gt, gt_masks=mask)[3]
    o4b[3].backward()
    assert rel_l2(gb.grad.cpu().numpy(), ga.grad.cpu().numpy()) < 1e-4
