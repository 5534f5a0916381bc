"""lgm_amd: MI355X-native (gfx950 / CDNA4) hot path of LGM -- the differentiable Gaussian-splat renderer
(drop-in for core/gs.py GaussianRenderer) and the multi-view attention (drop-in for core/attention.py
MemEffAttention and core/unet.py MVAttention). Compute lives in hand-written HIP kernels behind a C ABI
(include/*.h, lgm_amd/_lib/liblgm_amd.so); this package is the host side."""
from .options import Options
from .gs import GaussianRenderer, rasterize

__all__ = ["Options", "GaussianRenderer", "rasterize"]
__version__ = "0.1.0"
