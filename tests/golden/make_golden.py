"""Generates tests/golden/render_*.npz from the CPU oracle (inputs + expected outputs + gradients).
Run: python tests/golden/make_golden.py. The reference rasterizer is absent (EXT, un-vendored), so these vectors
pin the restatement (regression fixtures) and give the GPU tests fixed expected values; they are NOT reference
outputs (parity unpinned, see oracle/raster_oracle.c)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402
from tests.render_cases import TAN, scene, upstream  # noqa: E402

CASES = [
    # name, B, N, V, H, W, seed, scale_modifier, elevation
    ("tiny", 1, 16, 1, 16, 16, 0, 1.0, 0.0),
    ("small_2view", 1, 200, 2, 32, 32, 1, 1.0, 0.0),
    ("ragged_batch", 2, 400, 2, 40, 24, 2, 0.8, 20.0),
    ("dense_64", 1, 2000, 3, 64, 64, 3, 1.0, -15.0),
]

if __name__ == "__main__":
    for name, B, N, V, H, W, seed, mod, elev in CASES:
        g, cv, cvp = scene(B=B, N=N, V=V, seed=seed, elevation=elev)
        d_img, d_dep, d_alp, bg = upstream(B, V, H, W, seed=seed + 100)
        out = O.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg.numpy(), mod, d_image=d_img.numpy(),
                       d_depth=d_dep.numpy(), d_alpha=d_alp.numpy())
        np.savez_compressed(os.path.join(HERE, f"render_{name}.npz"), gaussians=g.numpy(), cam_view=cv.numpy(),
                            cam_view_proj=cvp.numpy(), tanfov=np.float64(TAN), H=H, W=W, bg=bg.numpy(),
                            scale_modifier=np.float64(mod), d_image=d_img.numpy(), d_depth=d_dep.numpy(),
                            d_alpha=d_alp.numpy(), image=out["image"], depth=out["depth"], alpha=out["alpha"],
                            d_gaussians=out["d_gaussians"], K=np.int64(out["K"]))
        print(name, "K =", out["K"])
