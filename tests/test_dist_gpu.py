"""Multi-process GPU path on the one-GPU test box: two ranks (gloo, 127.0.0.1) share cuda:0 and run the HIP renderer.
View-sharded: each rank renders its half of one scene's views and the per-scene dL/dgaussians is summed with
lgm_amd.dist.allreduce_scene_grads; scene-sharded: each rank renders its own objects. Both must equal the
single-process render (RCCL needs one GPU per rank, so the collective here is gloo on the same tensors)."""
import os

import numpy as np
import pytest
import torch

from lgm_amd import dist as D
from tests.render_cases import TAN, rel_l2, scene, upstream

pytestmark = pytest.mark.gpu
WORLD = 2


def _render(g, cv, cvp, bg, d_img, d_alpha, H):
    from lgm_amd.gs import rasterize
    dev = torch.device("cuda:0")
    gd = g.to(dev).requires_grad_(True)
    img, _, alp = rasterize(gd, cv.to(dev), cvp.to(dev), bg.to(dev), TAN, TAN, H, H, clamp=True)
    torch.autograd.backward([img, alp], [d_img.to(dev), d_alpha.to(dev)])
    torch.cuda.synchronize()
    return img.detach().cpu(), gd.grad.detach().cpu()


def _case():
    g, cv, cvp = scene(B=3, N=4000, V=5, seed=77, elevation=10.0)
    d_img, _, d_alpha, bg = upstream(3, 5, 64, 64, seed=78)
    return g, cv, cvp, bg, d_img, d_alpha


def _worker(tmp, mode):
    info = D.rank_info()
    D.init("gloo", info)
    try:
        g, cv, cvp, bg, d_img, d_alpha = _case()
        if mode == "views":  # scene 0, views split over the ranks
            v0, v1 = D.shard_range(5, info.rank, info.world)
            _, dg = _render(g[:1], cv[:1, v0:v1], cvp[:1, v0:v1], bg, d_img[:1, v0:v1], d_alpha[:1, v0:v1], 64)
            dg = D.allreduce_scene_grads(dg.double(), info)  # the RCCL all-reduce's role
            np.save(os.path.join(tmp, f"v{info.rank}.npy"), dg.numpy())
        else:  # objects split over the ranks
            s0, s1 = D.shard_range(3, info.rank, info.world)
            img, dg = _render(g[s0:s1], cv[s0:s1], cvp[s0:s1], bg, d_img[s0:s1], d_alpha[s0:s1], 64)
            np.savez(os.path.join(tmp, f"s{info.rank}.npz"), img=img.numpy(), dg=dg.numpy(), rng=np.array([s0, s1]))
    finally:
        D.finalize(info)


def test_view_sharded_gpu_allreduce(cuda, tmp_path):
    D.spawn_ranks(_worker, WORLD, str(tmp_path), "views")
    g, cv, cvp, bg, d_img, d_alpha = _case()
    _, full = _render(g[:1], cv[:1], cvp[:1], bg, d_img[:1], d_alpha[:1], 64)
    parts = [np.load(os.path.join(tmp_path, f"v{r}.npy")) for r in range(WORLD)]
    np.testing.assert_array_equal(parts[0], parts[1])
    assert rel_l2(parts[0], full.numpy()) < 1e-5


def test_scene_sharded_gpu(cuda, tmp_path):
    D.spawn_ranks(_worker, WORLD, str(tmp_path), "scenes")
    g, cv, cvp, bg, d_img, d_alpha = _case()
    img, full = _render(g, cv, cvp, bg, d_img, d_alpha, 64)
    for r in range(WORLD):
        z = np.load(os.path.join(tmp_path, f"s{r}.npz"))
        s0, s1 = z["rng"]
        np.testing.assert_array_equal(z["img"], img.numpy()[s0:s1])  # the forward is deterministic
        assert rel_l2(z["dg"], full.numpy()[s0:s1]) < 1e-5


def _rccl_worker(tmp):
    """One rank on cuda:0 with the nccl (= RCCL) backend: the collectives bench.py and the view-sharded backward
    issue, on a real RCCL communicator. (RCCL takes one GPU per rank, so the test box -- one GPU -- runs a
    single-rank group; the 2..8-rank runs are the driver's.)"""
    import torch.distributed as dist
    info = D.rank_info()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=info.rank, world_size=info.world, device_id=dev)
    try:
        g, cv, cvp, bg, d_img, d_alpha = _case()
        _, dg = _render(g[:1], cv[:1], cvp[:1], bg, d_img[:1], d_alpha[:1], 64)
        grad = dg.to(dev)
        # the view-sharded backward's in-place SUM (a one-rank group: the sum is the tensor itself); the RankInfo
        # stand-in only opens allreduce_scene_grads' world > 1 gate, the collective runs on the real group
        summed = D.allreduce_scene_grads(grad.clone(), D.RankInfo(0, 2, 0))
        flat = torch.randn(3_000_001, generator=torch.Generator().manual_seed(5)).to(dev)
        red = D.allreduce_bucketed(flat.clone(), 1_000_000, D.RankInfo(0, 2, 0), bf16=False)  # averages by 2
        mx = D.max_over_ranks(3.5, D.RankInfo(0, 2, 0), dev)
        torch.cuda.synchronize()
        np.savez(os.path.join(tmp, "rccl.npz"), grad=grad.cpu().numpy(), summed=summed.cpu().numpy(),
                 flat=flat.cpu().numpy(), red=red.cpu().numpy(), mx=np.array(mx),
                 backend=np.array(dist.get_backend()))
    finally:
        dist.destroy_process_group()


def test_rccl_collectives_single_rank(cuda, tmp_path):
    D.spawn_ranks(_rccl_worker, 1, str(tmp_path))
    z = np.load(os.path.join(tmp_path, "rccl.npz"))
    assert str(z["backend"]) == "nccl"
    np.testing.assert_array_equal(z["summed"], z["grad"])
    np.testing.assert_allclose(z["red"], z["flat"] / 2, rtol=0, atol=0)
    assert float(z["mx"]) == 3.5


class _TinyLGM(torch.nn.Module):
    """A stand-in for LGM's trainable part: a conv for the UNet (9 -> 14 channels, as core/unet.py's in/out) and
    the fused Gaussian head (core/models.py:96-117) -- enough to exercise DDP's reducer on real gradients of the
    render path."""

    def __init__(self):
        super().__init__()
        from lgm_amd.head import GaussianHead
        self.unet = torch.nn.Conv2d(9, 14, 3, padding=1)
        self.head = GaussianHead()
        with torch.no_grad():  # splats of the synthetic distribution's size (as bench.cfg5_inputs)
            self.head.conv.weight.copy_(torch.diag(torch.tensor([0.35] * 3 + [1.0] * 11)).view(14, 14, 1, 1))
            self.head.conv.bias.zero_()
            self.head.conv.bias[4:7] = -2.2522

    def forward(self, images):  # [V_in, 9, h, w] -> gaussians [1, V_in*h*w, 14]
        return self.head(self.unet(images), 1, images.shape[0])


def _train_step(model, opt, images, cams, gt, mask, bg, renderer):
    """main.py:99-109: forward, render + fused MSE loss (core/models.py:141-148), backward, clip, AdamW step."""
    opt.zero_grad()
    g = model(images)
    out = renderer.render(g, *cams, bg_color=bg, gt_images=gt, gt_masks=mask)
    out["loss_mse"].backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    grads = [p.grad.detach().clone() for p in model.parameters()]
    opt.step()
    return float(out["loss_mse"]), grads


def _ddp_inputs(dev):
    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import orbit_cameras
    gen = torch.Generator().manual_seed(31)
    images = torch.randn(4, 9, 32, 32, generator=gen).to(dev)
    cams = tuple(t[None].to(dev) for t in orbit_cameras(4, elevation=-10.0))
    gt = torch.rand(1, 4, 3, 96, 96, generator=gen).to(dev)
    mask = (torch.rand(1, 4, 1, 96, 96, generator=gen) > 0.5).float().to(dev)
    bg = torch.rand(3, generator=gen).to(dev)
    return images, cams, gt, mask, bg, GaussianRenderer(Options(output_size=96))


def _ddp_worker(tmp, bf16):
    """make_ddp on a real RCCL communicator (one rank on cuda:0): two training steps through DDP's reducer
    (100 MB buckets; fp32 or the bf16 compression hook), deterministic render gradients."""
    import torch.distributed as dist
    os.environ["LGM_AMD_DETERMINISTIC"] = "1"
    torch.backends.cudnn.deterministic = True
    info = D.rank_info()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=info.rank, world_size=info.world, device_id=dev)
    try:
        torch.manual_seed(3)
        model = _TinyLGM().to(dev)
        ddp = D.make_ddp(model, device=dev, bf16_compress=bf16)
        assert isinstance(ddp, torch.nn.parallel.DistributedDataParallel)
        opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3)
        inputs = _ddp_inputs(dev)
        losses, grads = [], []
        for _ in range(2):
            l, gr = _train_step(ddp, opt, *inputs)
            losses.append(l)
            grads.append(gr)
        torch.cuda.synchronize()
        np.savez(os.path.join(tmp, "ddp.npz"), losses=np.array(losses),
                 **{f"g{s}_{i}": t.cpu().numpy() for s, gr in enumerate(grads) for i, t in enumerate(gr)},
                 **{f"p_{i}": p.detach().cpu().numpy() for i, p in enumerate(model.parameters())},
                 backend=np.array(dist.get_backend()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bf16", [False, True])
def test_make_ddp_rccl_single_rank(cuda, tmp_path, monkeypatch, bf16):
    """The DDP-wrapped training step on RCCL equals the same step without DDP: to fp32 rounding with fp32 gradients
    (a one-rank all-reduce averages by 1; the render and head gradients are deterministic, the stand-in conv's
    MIOpen backward need not be bitwise across processes), to bf16 rounding with the compression hook; the
    parameters after AdamW likewise."""
    D.spawn_ranks(_ddp_worker, 1, str(tmp_path), bf16)
    z = np.load(os.path.join(tmp_path, "ddp.npz"))
    assert str(z["backend"]) == "nccl"
    monkeypatch.setenv("LGM_AMD_DETERMINISTIC", "1")
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(3)
    model = _TinyLGM().to(cuda)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    inputs = _ddp_inputs(cuda)
    for s in range(2):
        loss, grads = _train_step(model, opt, *inputs)
        for i, gr in enumerate(grads):
            got = z[f"g{s}_{i}"]
            if bf16:
                err = np.abs(got - gr.cpu().numpy()).max()
                assert err <= 2.0 ** -7 * np.abs(gr.cpu().numpy()).max() + 1e-12, (s, i, err)
            else:
                ref = gr.cpu().numpy()
                np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
        assert abs(float(z["losses"][s]) - loss) <= 1e-6 * abs(loss)
    for i, p in enumerate(model.parameters()):
        ref = p.detach().cpu().numpy()
        np.testing.assert_allclose(z[f"p_{i}"], ref, rtol=0, atol=(1e-3 if bf16 else 1e-6) * np.abs(ref).max())


def _accum_worker(tmp):
    """make_ddp + GradAccumulator (2 micro-steps, accelerate.accumulate's path) on a real one-rank RCCL group: the
    first micro-step's backward runs under no_sync, the second all-reduces the summed gradients; then the clip and
    AdamW step of main.py:99-109."""
    import torch.distributed as dist
    os.environ["LGM_AMD_DETERMINISTIC"] = "1"
    torch.backends.cudnn.deterministic = True
    info = D.rank_info()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=info.rank, world_size=info.world, device_id=dev)
    try:
        torch.manual_seed(3)
        model = _TinyLGM().to(dev)
        ddp = D.make_ddp(model, device=dev)
        opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3)
        images, cams, gt, mask, bg, renderer = _ddp_inputs(dev)
        acc = D.GradAccumulator(ddp, 2)
        syncs = []
        for k in range(2):
            with acc.accumulate():
                out = renderer.render(ddp(images * (1.0 + 0.25 * k)), *cams, bg_color=bg, gt_images=gt, gt_masks=mask)
                acc.backward(out["loss_mse"])
                syncs.append(acc.sync_gradients)
                if acc.sync_gradients:
                    torch.nn.utils.clip_grad_norm_(ddp.parameters(), 1.0)
                    grads = [p.grad.detach().clone() for p in model.parameters()]
                    opt.step()
                    opt.zero_grad()
        torch.cuda.synchronize()
        np.savez(os.path.join(tmp, "acc.npz"), syncs=np.array(syncs),
                 **{f"g_{i}": t.cpu().numpy() for i, t in enumerate(grads)},
                 **{f"p_{i}": p.detach().cpu().numpy() for i, p in enumerate(model.parameters())})
    finally:
        dist.destroy_process_group()


def test_gradient_accumulation_rccl_single_rank(cuda, tmp_path, monkeypatch):
    """Gradient accumulation through DDP on RCCL (GradAccumulator: no_sync micro-step, then one all-reduce) equals
    the accumulated plain step: the summed gradients of loss / 2 over both micro-batches (fp32 rounding; the render
    and head gradients are deterministic), and the parameters after the clip and AdamW step."""
    D.spawn_ranks(_accum_worker, 1, str(tmp_path))
    z = np.load(os.path.join(tmp_path, "acc.npz"))
    assert z["syncs"].tolist() == [False, True]
    monkeypatch.setenv("LGM_AMD_DETERMINISTIC", "1")
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(3)
    model = _TinyLGM().to(cuda)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    images, cams, gt, mask, bg, renderer = _ddp_inputs(cuda)
    for k in range(2):
        out = renderer.render(model(images * (1.0 + 0.25 * k)), *cams, bg_color=bg, gt_images=gt, gt_masks=mask)
        (out["loss_mse"] / 2).backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    for i, p in enumerate(model.parameters()):
        ref = p.grad.cpu().numpy()
        np.testing.assert_allclose(z[f"g_{i}"], ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
    opt.step()
    for i, p in enumerate(model.parameters()):
        ref = p.detach().cpu().numpy()
        np.testing.assert_allclose(z[f"p_{i}"], ref, rtol=0, atol=1e-6 * np.abs(ref).max())
