"""Device-side batched orbit cameras (lgm_amd.cameras.orbit_cameras_batched) against the per-view recipe of
infer.py:135-142 (orbit_camera -> flip -> inverse^T -> @ proj), and the batched video frames against per-frame
renders (CPU path here; the same code drives the GPU kernels)."""
import numpy as np
import torch

from lgm_amd import GaussianRenderer, Options
from lgm_amd.cameras import (cameras_from_c2w, orbit_camera, orbit_cameras_batched, projection_matrix,
                             render_orbit_frames)
from lgm_amd.synthetic import synthetic_gaussians


def test_batched_cameras_match_per_view_recipe():
    az = np.arange(0, 360, 2)
    for elev in (0.0, -30.0, 20.0):
        cv, cvp, cp = orbit_cameras_batched(elev, torch.from_numpy(az.astype(np.float32)), radius=1.5)
        poses = torch.from_numpy(np.stack([orbit_camera(elev, float(a), radius=1.5) for a in az]))
        rv, rvp, rp = cameras_from_c2w(poses, projection_matrix(49.1, 0.5, 2.5))
        assert cv.shape == (180, 4, 4) and cp.shape == (180, 3)
        np.testing.assert_allclose(cv.numpy(), rv.numpy(), atol=2e-6)
        np.testing.assert_allclose(cvp.numpy(), rvp.numpy(), atol=5e-6)
        np.testing.assert_allclose(cp.numpy(), rp.numpy(), atol=2e-6)


def test_orbit_frames_match_per_frame_renders():
    r = GaussianRenderer(Options(output_size=32))
    g = synthetic_gaussians(1, 400, seed=3)
    az = torch.arange(0, 360, 45, dtype=torch.float32)
    frames = render_orbit_frames(r, g, az, elevation=-15.0, chunk=3)
    assert frames.shape == (8, 32, 32, 3) and frames.dtype == torch.uint8
    for k, a in enumerate(az.tolist()):
        cv, cvp, cp = orbit_cameras_batched(-15.0, [a])
        img = r.render(g, cv[None], cvp[None], cp[None])["image"][0, 0]
        ref = (img.permute(1, 2, 0) * 255).to(torch.uint8)
        assert (frames[k].int() - ref.int()).abs().max() <= 1
