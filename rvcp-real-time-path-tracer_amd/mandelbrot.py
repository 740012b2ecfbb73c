"""The reference's second compute operator: the Mandelbrot viewer
of src/mandelbrot/ (assets/shaders/mandelbrot.comp), behind the same C-ABI
(``rvcp_mandelbrot``).  ``Config`` mirrors src/mandelbrot/config.rs:1-16 and
``update_keyboard_state`` src/mandelbrot/vulkan.rs:445-477 (f32, libm powf)."""
from __future__ import annotations

import ctypes
import ctypes.util
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np

f32 = np.float32

# == rvcp_mandelbrot_push_t / CameraData (src/mandelbrot/shader.rs:9-12)
MANDELBROT_PUSH_DTYPE = np.dtype([("position", "<f4", 2), ("scale", "<f4")])
assert MANDELBROT_PUSH_DTYPE.itemsize == 12

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
_libm.powf.restype = ctypes.c_float


@dataclass
class Config:
    """src/mandelbrot/config.rs:1-16."""
    camera_position: List[float] = field(default_factory=lambda: [0.0, 0.0])
    camera_scale: float = 1.0
    camera_move_speed: float = 0.5

    def push_constant(self) -> np.ndarray:
        rec = np.zeros((), dtype=MANDELBROT_PUSH_DTYPE)
        rec["position"] = self.camera_position
        rec["scale"] = self.camera_scale
        return rec


def update_keyboard_state(pressing: Dict[str, bool], config: Config, delta_time: float) -> bool:
    """src/mandelbrot/vulkan.rs:445-477; returns whether new push constants are needed."""
    scale_abs = f32(abs(f32(config.camera_scale)))
    g = max(f32(_libm.powf(float(scale_abs), 1.2)), f32(1.0))
    h = f32(f32(1.0) / scale_abs)
    speed, dt = f32(config.camera_move_speed), f32(delta_time)
    pos_v = f32(f32(h * speed) * dt)
    scale_v = f32(f32(g * speed) * dt)
    new = False
    p = [f32(config.camera_position[0]), f32(config.camera_position[1])]
    s = f32(config.camera_scale)
    for key, (idx, sign) in (("A", (0, -1)), ("D", (0, 1)), ("W", (1, -1)), ("S", (1, 1))):
        if pressing.get(key, False):
            new = True
            p[idx] = f32(p[idx] - pos_v) if sign < 0 else f32(p[idx] + pos_v)
    if pressing.get("Q", False):
        new = True
        s = f32(s - scale_v)
    if pressing.get("E", False):
        new = True
        s = f32(s + scale_v)
    config.camera_position = [float(p[0]), float(p[1])]
    config.camera_scale = float(s)
    return new
