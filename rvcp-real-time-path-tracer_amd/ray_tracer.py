"""RayTracer: host-side mirror of the reference's ``Vk`` runtime (src/ray_tracer/vulkan.rs),
driving librvcp through its C-ABI.

    reference (vulkan.rs)                       here
    ------------------------------------------  -----------------------------------------
    Vk::new -> create_compute_pipeline (:576)   RayTracer(config)        -> rvcp_create
    create_descriptor_set_0s (:454-574)         RayTracer.upload_scene   -> rvcp_upload_scene
    create_command_buffers + dispatch (:406)    RayTracer.render         -> rvcp_render
    Vk::update_frame (:298-404)                 RayTracer.update_frame (render + FPS tick)

There is no CPU fallback: constructing a RayTracer without a HIP device or without the built
library raises.
"""
from __future__ import annotations

import ctypes
import time as _time
from typing import Optional

import numpy as np

from . import abi, scene_io
from .scene import CAMERA_DTYPE, PUSH_DTYPE, Scene, push_constant


class RayTracer:
    def __init__(self, config: Optional[np.ndarray] = None, **overrides):
        self._lib = abi.load()
        if config is None:
            config = abi.make_config(**overrides)
        self.config = np.ascontiguousarray(config)
        h = ctypes.c_void_p()
        rc = self._lib.rvcp_create(abi.ptr(self.config), ctypes.byref(h))
        if rc != abi.RVCP_OK:
            raise abi.RvcpError(rc, self._lib.rvcp_last_error(None).decode())
        self._ctx = h
        self.scene: Optional[Scene] = None
        self.last_stats = None
        # FPS counter (src/ray_tracer/ray_tracer.rs:80-86)
        self.fps_frame_count = 0
        self.fps_last_time = _time.perf_counter()
        self.fps = None

    # ------------------------------------------------------------------ lifetime
    def close(self):
        """rvcp_destroy; returns its code (RVCP_E_TIMEOUT: a gather was still stuck behind a
        collective at the deadline and the context's device memory was leaked, rvcp.h)."""
        rc = abi.RVCP_OK
        if getattr(self, "_ctx", None):
            rc = self._lib.rvcp_destroy(self._ctx)
            self._ctx = None
        return rc

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc):
        if rc != abi.RVCP_OK:
            raise abi.RvcpError(rc, self._lib.rvcp_last_error(self._ctx).decode())

    @property
    def handle(self):
        return self._ctx

    # ------------------------------------------------------------------ scene
    def upload_arrays(self, materials, vertices, faces, lum_face_ids, spheres=None,
                      lum_sphere_ids=None):
        materials = np.ascontiguousarray(materials)
        vertices = np.ascontiguousarray(vertices)
        faces = np.ascontiguousarray(faces)
        lum = np.ascontiguousarray(lum_face_ids, dtype=np.uint32)
        sph = None if spheres is None or len(spheres) == 0 else np.ascontiguousarray(spheres)
        lsph = None if lum_sphere_ids is None or len(lum_sphere_ids) == 0 else \
            np.ascontiguousarray(lum_sphere_ids, dtype=np.uint32)
        self._check(self._lib.rvcp_upload_scene(
            self._ctx, abi.ptr(materials), len(materials), abi.ptr(vertices), len(vertices),
            abi.ptr(faces), len(faces), abi.ptr(sph), 0 if sph is None else len(sph),
            abi.ptr(lum), len(lum), abi.ptr(lsph), 0 if lsph is None else len(lsph)))

    def upload_scene(self, scene: Scene):
        self.upload_arrays(scene.aligned_materials(), scene.mesh.aligned_vertices(),
                           scene.mesh.aligned_faces(), scene.luminous_face_ids(),
                           scene.aligned_spheres(), scene.luminous_sphere_ids())
        self.scene = scene

    def upload_scene_file(self, path: str) -> np.ndarray:
        """Upload a binary scene file natively (rvcp_upload_scene_file); returns the stored
        AlignedCamera record and keeps the Python-side Scene for render()."""
        cam = np.zeros((), dtype=CAMERA_DTYPE)
        self._check(self._lib.rvcp_upload_scene_file(self._ctx, str(path).encode(), abi.ptr(cam)))
        self.scene = scene_io.load(path)
        return cam

    # ------------------------------------------------------------------ render
    def render_push(self, push: np.ndarray, width: int, height: int, want_linear: bool = False):
        push = np.ascontiguousarray(push, dtype=PUSH_DTYPE)
        rgba = np.empty((height, width, 4), dtype=np.uint8)
        lin = np.empty((height, width, 3), dtype=np.float32) if want_linear else None
        stats = np.zeros((), dtype=abi.STATS_DTYPE)
        self._check(self._lib.rvcp_render(self._ctx, abi.ptr(push), width, height, abi.ptr(rgba),
                                          abi.ptr(lin), abi.ptr(stats)))
        self.last_stats = stats
        return (rgba, lin) if want_linear else rgba

    def render(self, width: int, height: int, time: float, want_linear: bool = False):
        if self.scene is None:
            raise RuntimeError("upload_scene first")
        return self.render_push(push_constant(self.scene.camera, time), width, height, want_linear)

    def update_frame(self, width: int, height: int, time: Optional[float] = None):
        """One frame of the interactive loop (vulkan.rs:298-404): time seed = unix secs % 1000
        (vulkan.rs:418-421) unless given; counts FPS like ray_tracer.rs:80-86."""
        if time is None:
            time = float(np.float32(_time.time() % 1000.0))
        img = self.render(width, height, time)
        self.fps_frame_count += 1
        now = _time.perf_counter()
        if now - self.fps_last_time >= 1.0:
            self.fps = self.fps_frame_count / (now - self.fps_last_time)
            self.fps_frame_count = 0
            self.fps_last_time = now
        return img

    def mandelbrot(self, push: np.ndarray, width: int, height: int, want_value: bool = False):
        """The Mandelbrot operator (rvcp_mandelbrot): grey RGBA8 frame [, escape values]."""
        from .mandelbrot import MANDELBROT_PUSH_DTYPE
        push = np.ascontiguousarray(push, dtype=MANDELBROT_PUSH_DTYPE)
        rgba = np.empty((height, width, 4), dtype=np.uint8)
        val = np.empty((height, width), dtype=np.float32) if want_value else None
        stats = np.zeros((), dtype=abi.STATS_DTYPE)
        self._check(self._lib.rvcp_mandelbrot(self._ctx, abi.ptr(push), width, height,
                                              abi.ptr(rgba), abi.ptr(val), abi.ptr(stats)))
        self.last_stats = stats
        return (rgba, val) if want_value else rgba

    # ------------------------------------------------------------------ device-side API
    def render_shard_async(self, push, width, height, shard_index, shard_count, d_rgba: int,
                           d_linear: int = 0, stream: int = 0):
        push = np.ascontiguousarray(push, dtype=PUSH_DTYPE)
        self._push_keepalive = push
        self._check(self._lib.rvcp_render_shard_async(
            self._ctx, abi.ptr(push), width, height, shard_index, shard_count,
            ctypes.c_void_p(d_rgba), ctypes.c_void_p(d_linear) if d_linear else None,
            ctypes.c_void_p(stream) if stream else None))

    def render_frames_async(self, pushes, width, height, shard_index, shard_count, d_rgba: int,
                            d_linear: int = 0, stream: int = 0):
        """rvcp_render_frames_async: a batch of len(pushes) consecutive frames of one shard in
        one path kernel; frame k's rows start at pixel k * shard_rows(height, 0, shard_count) *
        width of d_rgba (and of d_linear).  Wait with sync_stats() / wait()."""
        pushes = np.ascontiguousarray(pushes, dtype=PUSH_DTYPE).reshape(-1)
        self._push_keepalive = pushes
        self._check(self._lib.rvcp_render_frames_async(
            self._ctx, abi.ptr(pushes), len(pushes), width, height, shard_index, shard_count,
            ctypes.c_void_p(d_rgba), ctypes.c_void_p(d_linear) if d_linear else None,
            ctypes.c_void_p(stream) if stream else None))

    def render_async(self, push, width, height, d_rgba: int, d_linear: int = 0, stream: int = 0):
        """rvcp_render_async: enqueue one full frame into device memory; see wait()."""
        push = np.ascontiguousarray(push, dtype=PUSH_DTYPE)
        self._push_keepalive = push
        self._check(self._lib.rvcp_render_async(
            self._ctx, abi.ptr(push), width, height, ctypes.c_void_p(d_rgba),
            ctypes.c_void_p(d_linear) if d_linear else None,
            ctypes.c_void_p(stream) if stream else None))

    def wait(self):
        """rvcp_wait: block until the last async render is done; returns its stats."""
        stats = np.zeros((), dtype=abi.STATS_DTYPE)
        self._check(self._lib.rvcp_wait(self._ctx, abi.ptr(stats)))
        self.last_stats = stats
        return stats

    def sync_stats(self):
        stats = np.zeros((), dtype=abi.STATS_DTYPE)
        self._check(self._lib.rvcp_sync_stats(self._ctx, abi.ptr(stats)))
        self.last_stats = stats
        return stats

    def assemble_frame_async(self, d_gathered: int, slot_rows: int, width: int, height: int,
                             shard_count: int, d_frame: int, stream: int = 0):
        self._check(self._lib.rvcp_assemble_frame_async(
            self._ctx, ctypes.c_void_p(d_gathered), slot_rows, width, height, shard_count,
            ctypes.c_void_p(d_frame), ctypes.c_void_p(stream) if stream else None))

    # ------------------------------------------------------------------ one process per GPU
    def rccl_init(self, unique_id: bytes, world: int, rank: int):
        """rvcp_rccl_init: join the frame-gather communicator (collective over `world` ranks;
        `unique_id` from rccl_unique_id() on rank 0, shared out of band)."""
        if len(unique_id) != abi.RCCL_ID_BYTES:
            raise ValueError("unique_id must be 128 bytes")
        buf = (ctypes.c_uint8 * abi.RCCL_ID_BYTES).from_buffer_copy(unique_id)
        self._check(self._lib.rvcp_rccl_init(self._ctx, ctypes.cast(buf, ctypes.c_void_p), world, rank))

    def rccl_attach(self, nccl_comm: int, world: int, rank: int):
        """rvcp_rccl_attach: gather over the caller's communicator (an ncclComm_t on this
        context's device; blocking or not); the caller keeps it and is the one to abort it."""
        self._check(self._lib.rvcp_rccl_attach(self._ctx, ctypes.c_void_p(nccl_comm), world, rank))

    def rccl_set_timeout(self, timeout_ms: int):
        """rvcp_rccl_set_timeout: deadline of rccl_init / gather_wait in ms (0 = none); past it
        they raise RvcpError with code RVCP_E_TIMEOUT and the communicator is aborted."""
        self._check(self._lib.rvcp_rccl_set_timeout(self._ctx, int(timeout_ms)))

    def gather_frame_async(self, d_shard: int, width: int, height: int, d_gathered: int = 0,
                           d_frame: int = 0, stream: int = 0):
        """rvcp_gather_frame_async: RCCL gather of the shards to rank 0 + device assembly
        there (d_gathered / d_frame only on rank 0)."""
        self._check(self._lib.rvcp_gather_frame_async(
            self._ctx, ctypes.c_void_p(d_shard), width, height,
            ctypes.c_void_p(d_gathered) if d_gathered else None,
            ctypes.c_void_p(d_frame) if d_frame else None,
            ctypes.c_void_p(stream) if stream else None))

    def gather_wait(self):
        """rvcp_gather_wait: block until the last gather is done; returns (gather_ms,
        render-start-to-gather-end ms) from HIP events on the gather's stream."""
        g, f = ctypes.c_float(0.0), ctypes.c_float(0.0)
        self._check(self._lib.rvcp_gather_wait(self._ctx, ctypes.byref(g), ctypes.byref(f)))
        return float(g.value), float(f.value)


def rccl_unique_id() -> bytes:
    """rvcp_rccl_unique_id (rank 0): the 128-byte RCCL communicator id."""
    L = abi.load()
    buf = (ctypes.c_uint8 * abi.RCCL_ID_BYTES)()
    rc = L.rvcp_rccl_unique_id(ctypes.cast(buf, ctypes.c_void_p))
    if rc != abi.RVCP_OK:
        raise abi.RvcpError(rc, L.rvcp_last_error(None).decode())
    return bytes(buf)


def shard_rows(height: int, shard_index: int, shard_count: int) -> int:
    """Rows of shard `shard_index` (8-row stripes dealt round-robin).  Pure-Python twin of
    rvcp_shard_rows for hosts without the library loaded."""
    stripes = (height + 7) // 8
    return sum(min(8, height - 8 * s) for s in range(shard_index, stripes, shard_count))


def shard_row_ids(height: int, shard_index: int, shard_count: int) -> np.ndarray:
    """Global row ids of a shard's packed rows, in order."""
    stripes = (height + 7) // 8
    rows = [y for s in range(shard_index, stripes, shard_count)
            for y in range(8 * s, min(8 * s + 8, height))]
    return np.array(rows, dtype=np.int64)
