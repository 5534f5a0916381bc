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
