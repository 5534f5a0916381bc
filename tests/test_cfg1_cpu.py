"""BASELINE config 1 end to end on the CPU (scripts/cfg1_cpu.py): the reference's 'big' UNet with its 16
MVAttention blocks swapped for lgm_amd's, the catstatue PNG as 4 views + rays, the Gaussian head, save_ply and one
256^2 render through lgm_amd.GaussianRenderer on CPU tensors. Checks: the swapped UNet equals the unswapped
reference UNet (same weights, the reference's fallback attention) to fp32 rounding; the render equals the oracle's
on the same Gaussians; the PLY round-trips. Needs the reference checkout for the UNet (this container only)."""
import os

import numpy as np
import pytest
import torch

from tests.render_cases import rel_l2

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "core")), reason="reference checkout absent")
PNG = os.path.join(os.path.dirname(__file__), "golden", "catstatue_rgba.png")


def test_cfg1_big_cpu_end_to_end(tmp_path, oracle_mod):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "scripts"))
    import cfg1_cpu as H
    res = H.run(REF, PNG, str(tmp_path), seed=0)
    print({k: v for k, v in res.items() if k != "_frame"})
    assert res["swapped_mvattention_blocks"] == 16
    assert res["unet_out"] == [4, 14, 128, 128] and res["gaussians"] == [1, 65536, 14]
    assert res["image_finite"] and res["frame"] == [1, 256, 256, 3]

    # the swapped UNet == the reference UNet with its own (fallback) attention, same weights
    from core.unet import UNet
    torch.manual_seed(0)
    swapped, _ = H.build_big_unet(REF)
    torch.manual_seed(0)
    ref = UNet(9, 14, **H.BIG)
    swapped.eval()
    ref.eval()
    x = H.load_views(PNG).view(4, 9, 256, 256)
    with torch.no_grad():
        a, b = swapped(x), ref(x)
    assert rel_l2(a.numpy(), b.numpy()) < 1e-5

    # the harness's render vs the oracle on the same Gaussians and camera
    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import cameras_from_c2w, orbit_camera, projection_matrix
    from lgm_amd.head import GaussianHead
    torch.manual_seed(0)
    H.build_big_unet(REF)  # (consumes the same random stream as run(): the head's init follows)
    head = GaussianHead()
    with torch.no_grad():
        g = head(a, 1, 4)
    opt = Options(output_size=256)
    pose = torch.from_numpy(orbit_camera(0, 0, radius=1.5, opengl=True)).unsqueeze(0)
    cv, cvp, cp = cameras_from_c2w(pose, projection_matrix(opt.fovy, opt.znear, opt.zfar))
    with torch.no_grad():
        out = GaussianRenderer(opt).render(g, cv[None], cvp[None], cp[None])
    o = oracle_mod.render(g.numpy(), cv[None].numpy(), cvp[None].numpy(), float(np.tan(0.5 * np.deg2rad(49.1))),
                          256, 256, np.ones(3, np.float32))
    assert rel_l2(out["image"].numpy(), np.clip(o["image"], 0, 1)) < 1e-4
    assert rel_l2(out["alpha"].numpy(), o["alpha"]) < 1e-4

    # save_ply wrote what load_ply reads back (opacity-pruned, inverse activations round-tripped)
    back = GaussianRenderer(opt).load_ply(str(tmp_path / "catstatue.ply"))
    keep = g[0, :, 3] >= 0.005
    assert back.shape == (int(keep.sum()), 14)
