"""ctypes wrapper of the CPU oracle (oracle/build/librvcp_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  The product path (librvcp.so) never uses it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "librvcp_oracle.so")
# the same source at -O3: the copy bench.py's cpu_baseline times
LIB_PATH_O3 = os.path.join(_HERE, "build", "librvcp_oracle_o3.so")
_libs = {}


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    if force or not os.path.exists(LIB_PATH) or not os.path.exists(LIB_PATH_O3):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib(o3: bool = False):
    """The checker (-O2), or with o3 the timing copy (-O3)."""
    path = LIB_PATH_O3 if o3 else LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.rvcp_oracle_sinf.argtypes = [ctypes.c_float]
        L.rvcp_oracle_sinf.restype = ctypes.c_float
        L.rvcp_oracle_gamma_u8.argtypes = [ctypes.c_float]
        L.rvcp_oracle_gamma_u8.restype = ctypes.c_uint8
        L.rvcp_oracle_gamma_threshold.argtypes = [ctypes.c_int]
        L.rvcp_oracle_gamma_threshold.restype = ctypes.c_float
        L.rvcp_oracle_rand_sequence.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                ctypes.c_int, P]
        L.rvcp_oracle_rand_sequence.restype = None
        L.rvcp_oracle_intersect.argtypes = [P, P, P]
        L.rvcp_oracle_intersect.restype = ctypes.c_int
        L.rvcp_oracle_sample_ray.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, P]
        L.rvcp_oracle_sample_ray.restype = None
        u32 = ctypes.c_uint32
        L.rvcp_oracle_render.argtypes = [P, u32, P, u32, P, u32, P, u32, P, u32, P, P,
                                         u32, u32, u32, u32, u32, u32, P, P, P, ctypes.c_int]
        L.rvcp_oracle_unorm_u8.argtypes = [ctypes.c_float]
        L.rvcp_oracle_unorm_u8.restype = ctypes.c_uint8
        for f in ("rvcp_oracle_unorm_u8_rule", "rvcp_oracle_gamma_u8_rule"):
            getattr(L, f).argtypes = [ctypes.c_float, ctypes.c_int]
            getattr(L, f).restype = ctypes.c_uint8
        L.rvcp_oracle_gamma_threshold_rule.argtypes = [ctypes.c_int, ctypes.c_int]
        L.rvcp_oracle_gamma_threshold_rule.restype = ctypes.c_float
        L.rvcp_oracle_render.restype = ctypes.c_int
        L.rvcp_oracle_mandelbrot.argtypes = [P, u32, u32, ctypes.c_int, P, P]
        L.rvcp_oracle_mandelbrot.restype = ctypes.c_int
        _libs[path] = L
    return _libs[path]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def sinf(x: float) -> float:
    return float(lib().rvcp_oracle_sinf(ctypes.c_float(x)))


def gamma_u8(c: float, unorm_rule: int = 0) -> int:
    """pow(clamp(c), 0.6) stored as UNORM8 under rvcp_config_t.unorm_rule (0 driver, 1 nearest)."""
    return int(lib().rvcp_oracle_gamma_u8_rule(ctypes.c_float(c), int(unorm_rule)))


def unorm_u8(c: float, unorm_rule: int = 0) -> int:
    """clamp(c) stored as UNORM8 under rvcp_config_t.unorm_rule (0 driver, 1 nearest)."""
    return int(lib().rvcp_oracle_unorm_u8_rule(ctypes.c_float(c), int(unorm_rule)))


def gamma_threshold(k: int, unorm_rule: int = 0) -> float:
    return float(lib().rvcp_oracle_gamma_threshold_rule(int(k), int(unorm_rule)))


def rand_sequence(time: float, u: float, v: float, n: int) -> np.ndarray:
    out = np.zeros(n + 1, dtype=np.float32)
    lib().rvcp_oracle_rand_sequence(ctypes.c_float(time), ctypes.c_float(u), ctypes.c_float(v),
                                    n, _ptr(out))
    return out


def intersect(ray, tri):
    ray = np.ascontiguousarray(ray, dtype=np.float32)
    tri = np.ascontiguousarray(tri, dtype=np.float32).reshape(9)
    out = np.zeros(3, dtype=np.float32)
    hit = lib().rvcp_oracle_intersect(_ptr(ray), _ptr(tri), _ptr(out))
    return bool(hit), out


def sample_ray(push, W, H, x, y) -> np.ndarray:
    push = np.ascontiguousarray(push)
    out = np.zeros(8, dtype=np.float32)
    lib().rvcp_oracle_sample_ray(_ptr(push), W, H, x, y, _ptr(out))
    return out


def default_threads() -> int:
    """Worker threads for the oracle: OMP_NUM_THREADS when set (the GPU box sets it to its CPU
    share, 16 per GPU), else the CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0)) or 1
    except AttributeError:
        return os.cpu_count() or 1


def render(scene_arrays: dict, push, cfg, W, H, rect=None, threads=None, want_linear=True,
           o3=False):
    """Render with the oracle.  scene_arrays: materials/vertices/faces/lum_face_ids numpy
    record arrays (scene.py dtypes); push: PUSH_DTYPE record; cfg: rvcp_config_t bytes
    (numpy record of CONFIG_DTYPE).  Returns (linear [th,tw,3] f32 | None, rgba [th,tw,4] u8,
    traversals).  o3: render with the -O3 timing copy (same bits)."""
    x0, y0, tw, th = rect if rect is not None else (0, 0, W, H)
    threads = threads or default_threads()
    mats = np.ascontiguousarray(scene_arrays["materials"])
    verts = np.ascontiguousarray(scene_arrays["vertices"])
    faces = np.ascontiguousarray(scene_arrays["faces"])
    lum = np.ascontiguousarray(scene_arrays["lum_face_ids"], dtype=np.uint32)
    sph = scene_arrays.get("spheres")
    sph = np.ascontiguousarray(sph) if sph is not None and len(sph) else None
    push = np.ascontiguousarray(push)
    cfg = np.ascontiguousarray(cfg)
    lin = np.zeros((th, tw, 3), dtype=np.float32) if want_linear else None
    rgba = np.zeros((th, tw, 4), dtype=np.uint8)
    trav = np.zeros(1, dtype=np.uint64)
    rc = lib(o3).rvcp_oracle_render(_ptr(mats), len(mats), _ptr(verts), len(verts), _ptr(faces),
                                  len(faces), _ptr(sph), 0 if sph is None else len(sph),
                                  _ptr(lum), len(lum), _ptr(push), _ptr(cfg),
                                  W, H, x0, y0, tw, th, _ptr(lin), _ptr(rgba), _ptr(trav),
                                  int(threads))
    if rc != 0:
        raise ValueError(f"rvcp_oracle_render failed: {rc}")
    return lin, rgba, int(trav[0])


def mandelbrot(push, W, H, unorm_rule=0):
    """The Mandelbrot operator (mandelbrot.comp): returns (rgba [H,W,4] u8, i [H,W] f32).
    push: a MANDELBROT_PUSH_DTYPE record (position[2], scale); unorm_rule: rvcp_config_t's."""
    push = np.ascontiguousarray(push)
    rgba = np.zeros((H, W, 4), dtype=np.uint8)
    val = np.zeros((H, W), dtype=np.float32)
    rc = lib().rvcp_oracle_mandelbrot(_ptr(push), W, H, int(unorm_rule), _ptr(rgba), _ptr(val))
    if rc != 0:
        raise ValueError(f"rvcp_oracle_mandelbrot failed: {rc}")
    return rgba, val
