"""Interactive caller: headless mirror of the reference's window loop
(src/ray_tracer/ray_tracer.rs:22-164 + vulkan.rs:37-79, 298-452).

The reference drives the kernel from a winit event loop: key / mouse events update a
``RuntimeInfo``, every ``MainEventsCleared`` counts FPS (``ray_tracer.rs:80-87``), moves the
camera (``update_camera_state``, ``:104-164``) and renders a frame whose RNG seed is
``unix_secs % 1000`` (``vulkan.rs:418-421``).  There is no display here, so the loop is
driven by a scripted input timeline and frames can be written to PPM / PNG files.

Camera arithmetic is float32 like glam 0.29 on the Rust side; ``sin``/``cos``/``atan2``/
``asin`` are the C library's float functions (Rust's ``f32::sin`` etc. call the platform
libm), ``to_radians``/``to_degrees`` multiply by Rust's f32 constants.
"""
from __future__ import annotations

import os
import struct
import time as _time
import zlib
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional, Tuple

import numpy as np

from .scene import DEGS_PER_RAD, RADS_PER_DEG, Camera, Y, _libm, cross, normalize, vec3

f32 = np.float32

# winit VirtualKeyCode names the reference reacts to (ray_tracer.rs:124-129)
KEYS = ("A", "D", "S", "W", "Q", "E")


def yaw_pitch_of(forward) -> Tuple[float, float]:
    """``Camera::new``'s ``forward.z.atan2(forward.x).to_degrees()`` and
    ``forward.y.asin().to_degrees()`` (camera.rs:67-69), in f32."""
    yaw = f32(f32(_libm.atan2f(float(forward[2]), float(forward[0]))) * DEGS_PER_RAD)
    pitch = f32(f32(_libm.asinf(float(forward[1]))) * DEGS_PER_RAD)
    return float(yaw), float(pitch)


@dataclass
class RuntimeInfo:
    """The input / timing half of ``RuntimeInfo`` (vulkan.rs:37-55)."""
    window_size: Tuple[int, int] = (384, 384)           # ray_tracer.rs:28
    is_new_push_constants: bool = False
    fps_last_time: float = field(default_factory=_time.perf_counter)
    fps_frame_count: int = 0
    last_tick_time: float = field(default_factory=_time.perf_counter)
    keyboard_is_pressing: Dict[str, bool] = field(default_factory=dict)
    mouse_cur_position: Tuple[float, float] = (0.0, 0.0)
    is_mouse_right_button_pressing: bool = False

    # winit events (ray_tracer.rs:46-77)
    def key(self, name: str, pressed: bool):
        self.keyboard_is_pressing[name] = pressed

    def mouse_right(self, pressed: bool):
        self.is_mouse_right_button_pressing = pressed
        self.mouse_cur_position = (float(f32(self.window_size[0] // 2)),
                                   float(f32(self.window_size[1] // 2)))

    def cursor(self, x: float, y: float):
        self.mouse_cur_position = (float(f32(x)), float(f32(y)))


def update_camera_state(info: RuntimeInfo, camera: Camera, delta_time: float) -> bool:
    """``update_camera_state`` (ray_tracer.rs:104-164).  Mutates ``camera``; returns whether
    new push constants are needed.  The cursor re-centring of ``:153-163`` is a window
    operation: here the cursor is reset to the window centre."""
    dt = f32(delta_time)
    move_v = f32(f32(camera.move_speed) * dt)
    rotate_v = f32(f32(camera.rotate_speed) * dt)
    pressed = lambda k: bool(info.keyboard_is_pressing.get(k, False))   # noqa: E731

    pos = np.asarray(camera.position, dtype=f32)
    if pressed("A"):
        info.is_new_push_constants = True
        pos = (pos - (camera.right * move_v).astype(f32)).astype(f32)
    if pressed("D"):
        info.is_new_push_constants = True
        pos = (pos + (camera.right * move_v).astype(f32)).astype(f32)
    if pressed("S"):
        info.is_new_push_constants = True
        pos = (pos - (camera.forward * move_v).astype(f32)).astype(f32)
    if pressed("W"):
        info.is_new_push_constants = True
        pos = (pos + (camera.forward * move_v).astype(f32)).astype(f32)
    if pressed("Q"):
        info.is_new_push_constants = True
        pos = (pos - (Y * move_v).astype(f32)).astype(f32)
    if pressed("E"):
        info.is_new_push_constants = True
        pos = (pos + (Y * move_v).astype(f32)).astype(f32)
    camera.position = pos

    cx, cy = info.window_size[0] // 2, info.window_size[1] // 2
    if info.is_mouse_right_button_pressing:
        info.is_new_push_constants = True
        dx = f32(f32(info.mouse_cur_position[0]) - f32(cx))
        dy = f32(f32(info.mouse_cur_position[1]) - f32(cy))
        yaw = f32(f32(camera.yaw) + f32(dx * rotate_v))
        pitch = f32(f32(camera.pitch) - f32(dy * rotate_v))
        pitch = f32(min(max(pitch, f32(-89.0)), f32(89.0)))
        yaw_rad = f32(yaw * RADS_PER_DEG)
        pitch_rad = f32(pitch * RADS_PER_DEG)
        cy_, sy_ = f32(_libm.cosf(float(yaw_rad))), f32(_libm.sinf(float(yaw_rad)))
        cp_, sp_ = f32(_libm.cosf(float(pitch_rad))), f32(_libm.sinf(float(pitch_rad)))
        camera.forward = normalize(vec3(f32(cy_ * cp_), sp_, f32(sy_ * cp_)))
        camera.right = normalize(cross(camera.forward, Y))
        camera.up = normalize(cross(camera.right, camera.forward))
        camera.yaw, camera.pitch = float(yaw), float(pitch)
        info.mouse_cur_position = (float(cx), float(cy))          # set_cursor_position (:155)
    return info.is_new_push_constants


# ---------------------------------------------------------------------- image files
def write_ppm(path: str, rgba: np.ndarray):
    """Binary PPM (P6) of an RGBA8 frame (alpha dropped)."""
    h, w = rgba.shape[:2]
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(rgba[..., :3]).tobytes())


def read_ppm(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255"
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], dtype=np.uint8).reshape(h, w, 3)


def write_png(path: str, rgba: np.ndarray):
    """Minimal RGBA8 PNG writer (zlib, filter 0) -- no imaging library needed."""
    h, w = rgba.shape[:2]
    raw = b"".join(b"\x00" + np.ascontiguousarray(rgba[y]).tobytes() for y in range(h))

    def chunk(tag, body):
        return (struct.pack(">I", len(body)) + tag + body +
                struct.pack(">I", zlib.crc32(tag + body) & 0xFFFFFFFF))
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


# ---------------------------------------------------------------------- the loop
# A scripted input event: (frame index, kind, args) with kind in
#   "key" (name, pressed) | "mouse_right" (pressed,) | "cursor" (x, y)
Event = Tuple[int, str, tuple]


def run_headless(tracer, scene, frames: int, width: int, height: int,
                 events: Iterable[Event] = (), fixed_dt: Optional[float] = None,
                 time_seed: Optional[Callable[[int], float]] = None,
                 dump_dir: Optional[str] = None, dump_format: str = "ppm",
                 on_fps: Optional[Callable[[int], None]] = None) -> dict:
    """``main_loop`` (ray_tracer.rs:22-100) without a window.

    Per frame: apply this frame's scripted events, count FPS (printed once a second as
    ``Rendering FPS: n``, :80-87), advance the camera by the elapsed time (or ``fixed_dt``
    for reproducible runs), render through ``tracer`` (a RayTracer with the scene uploaded)
    with time seed ``time_seed(i)`` or ``unix_secs % 1000``, and optionally dump the frame.
    Returns per-frame render times and the final camera."""
    info = RuntimeInfo(window_size=(width, height))
    by_frame: Dict[int, List[Event]] = {}
    for ev in events:
        by_frame.setdefault(int(ev[0]), []).append(ev)
    cam = scene.camera
    if dump_dir:
        os.makedirs(dump_dir, exist_ok=True)
    frame_ms, fps_reports, moved = [], [], []
    for i in range(frames):
        for _, kind, args in by_frame.get(i, []):
            if kind == "key":
                info.key(*args)
            elif kind == "mouse_right":
                info.mouse_right(*args)
            elif kind == "cursor":
                info.cursor(*args)
            else:
                raise ValueError(f"unknown event kind {kind!r}")
        info.fps_frame_count += 1
        now = _time.perf_counter()
        if now - info.fps_last_time >= 1.0:
            fps_reports.append(info.fps_frame_count)
            (on_fps or (lambda n: print(f"Rendering FPS: {n}", flush=True)))(info.fps_frame_count)
            info.fps_frame_count = 0
            info.fps_last_time = now
        dt = fixed_dt if fixed_dt is not None else now - info.last_tick_time
        info.last_tick_time = now
        info.is_new_push_constants = False
        moved.append(update_camera_state(info, cam, dt))
        t = time_seed(i) if time_seed else float(f32(_time.time() % 1000.0))
        t0 = _time.perf_counter()
        rgba = tracer.render(width, height, t)
        frame_ms.append((_time.perf_counter() - t0) * 1000.0)
        if dump_dir:
            path = os.path.join(dump_dir, f"frame_{i:05d}.{dump_format}")
            (write_png if dump_format == "png" else write_ppm)(path, rgba)
    return dict(frame_ms=frame_ms, fps_reports=fps_reports, camera_moved=moved, camera=cam)
