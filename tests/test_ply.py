import numpy as np
import torch

from lgm_amd import GaussianRenderer, Options
from lgm_amd.synthetic import synthetic_gaussians


def test_ply_roundtrip(tmp_path):
    r = GaussianRenderer(Options())
    g = synthetic_gaussians(1, 300, seed=4)
    g[0, :10, 3] = 0.001  # pruned (< 0.005), core/gs.py:116
    p = str(tmp_path / "x.ply")
    r.save_ply(g, p)
    back = r.load_ply(p)
    keep = g[0, :, 3] >= 0.005
    assert back.shape == (int(keep.sum()), 14)
    assert torch.allclose(back, g[0][keep], atol=2e-5)
    head = open(p, "rb").read(400)
    assert b"property float f_dc_0" in head and b"property float rot_3" in head
