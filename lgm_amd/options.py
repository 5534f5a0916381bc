"""The subset of core/options.py:6-75 `Options` that the render / attention path reads (fovy, znear, zfar,
output_size, cam_radius, num_input_views). Plain dataclass: tyro and the training presets are out of scope."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class Options:
    input_size: int = 256
    splat_size: int = 64
    output_size: int = 256
    fovy: float = 49.1
    znear: float = 0.5
    zfar: float = 2.5
    num_views: int = 12
    num_input_views: int = 4
    cam_radius: float = 1.5
