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


def test_ply_bytes_follow_the_reference_recipe(tmp_path):
    """save_ply's file is byte for byte what core/gs.py:101-152 hands plyfile: the structured float32 'vertex'
    element (x y z f_dc_0..2 opacity scale_0..2 rot_0..3, filled row by row from the concatenated attributes) under
    plyfile's binary_little_endian 1.0 header (one 'property float' line per field)."""
    r = GaussianRenderer(Options())
    g = synthetic_gaussians(1, 257, seed=9)
    g[0, 3:9, 3] = 0.002  # pruned
    p = str(tmp_path / "y.ply")
    r.save_ply(g, p)
    # the reference's construction, restated (core/gs.py:105-152; kiui.op.inverse_sigmoid clamps to [1e-6, 1-1e-6])
    x = g[0].double()
    keep = x[:, 3] >= 0.005
    x = x[keep].float()
    o = x[:, 3:4].clamp(1e-6, 1 - 1e-6)
    attrs = torch.cat([x[:, 0:3], (x[:, 11:14] - 0.5) / 0.28209479177387814, torch.log(o / (1 - o)),
                       torch.log(x[:, 4:7] + 1e-8), x[:, 7:11]], dim=1).numpy()
    names = ["x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2", "opacity", "scale_0", "scale_1", "scale_2", "rot_0",
             "rot_1", "rot_2", "rot_3"]
    el = np.empty(attrs.shape[0], dtype=[(n, "f4") for n in names])
    el[:] = list(map(tuple, attrs))
    header = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % attrs.shape[0] + \
        "".join(f"property float {n}\n" for n in names) + "end_header\n"
    want = header.encode("ascii") + el.astype(el.dtype.newbyteorder("<")).tobytes()
    got = open(p, "rb").read()
    assert got[:len(header)] == want[:len(header)]
    assert got == want  # byte for byte, body included
