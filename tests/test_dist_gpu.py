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
