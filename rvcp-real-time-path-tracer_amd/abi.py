"""ctypes binding of librvcp (include/rvcp.h) -- the product's C-ABI.

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950)
into ``csrc/build/librvcp.so``.  There is no fallback: if the library is missing,
``load()`` raises, so nothing can silently run a CPU path in its place.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RVCP_LIB") or os.path.join(_HERE, "csrc", "build", "librvcp.so")

# rvcp_config_t (include/rvcp.h)
CONFIG_DTYPE = np.dtype([("device", "<i4"), ("integrator", "<i4"), ("spp", "<u4"),
                         ("max_bounces", "<u4"), ("attenuation_stop_eps", "<f4"),
                         ("ray_t_min", "<f4"), ("ray_t_max", "<f4"), ("rr_probability", "<f4"),
                         ("eps", "<f4"), ("lum_id_std140_quirk", "<i4"), ("kernel_variant", "<i4"),
                         ("accel", "<i4"), ("n_gpus", "<i4"), ("unorm_rule", "<i4"),
                         ("specialize", "<i4"), ("grid_waves_per_simd", "<u4")])
STATS_DTYPE = np.dtype([("kernel_ms", "<f8"), ("traversals", "<u8"),
                        ("traversals_executed", "<u8"), ("samples", "<u8"), ("faces", "<u4"),
                        ("kernel_variant", "<i4"), ("wave_iterations", "<u8"),
                        ("main_kernel_ms", "<f8"), ("shader_clock_ghz", "<f8")])
assert CONFIG_DTYPE.itemsize == 64 and STATS_DTYPE.itemsize == 64
# rvcp_stats_t.kernel_variant -> the dominant kernel's name as rocprofv3 reports it
KERNEL_NAMES = {1: "games101_kernel", 2: "games101_dual_kernel", 3: "games101_path_kernel<5>",
                4: "games101_tiled_kernel", 5: "games101_tiled_single_kernel",
                6: "games101_path_kernel<6>", 7: "games101_bvh_path_kernel", 8: "legacy_kernel",
                10: "games101_tiled_pool_kernel",
                # + RVCP_VARIANT_SPECIALIZED (16): the scene-specialised module (rvcp_jit.cpp)
                19: "rvcp_spec_path_kernel5", 22: "rvcp_spec_path_kernel6", 23: "rvcp_spec_bvh_path_kernel",
                24: "rvcp_spec_legacy_kernel"}
VARIANT_SPECIALIZED = 16

# Defaults == the shader's #defines (ray_tracer_games101_branch.comp:5-13).
DEFAULTS = dict(device=0, integrator=0, spp=20, max_bounces=15, attenuation_stop_eps=0.05,
                ray_t_min=0.01, ray_t_max=10000.0, rr_probability=0.8, eps=0.001,
                lum_id_std140_quirk=1, kernel_variant=0, accel=0, n_gpus=1, unorm_rule=0, specialize=0,
                grid_waves_per_simd=0)

# Error codes
RVCP_OK, RVCP_E_INVALID, RVCP_E_HIP, RVCP_E_NO_SCENE, RVCP_E_UNSUPPORTED, RVCP_E_NOMEM, \
    RVCP_E_INTERNAL, RVCP_E_TIMEOUT, RVCP_E_BUSY = 0, -1, -2, -3, -4, -5, -6, -7, -8
# RVCP_ABI_VERSION of include/rvcp.h this binding's struct layouts follow (load() checks it)
ABI_VERSION = 2
RCCL_ID_BYTES = 128

EXPORTED = ["rvcp_version", "rvcp_config_default", "rvcp_config_default_for", "rvcp_create",
            "rvcp_destroy", "rvcp_last_error", "rvcp_upload_scene", "rvcp_render", "rvcp_render_shard_async",
            "rvcp_sync_stats", "rvcp_shard_rows", "rvcp_assemble_frame_async",
            "rvcp_upload_scene_file", "rvcp_mandelbrot", "rvcp_render_async", "rvcp_wait",
            "rvcp_rccl_unique_id", "rvcp_rccl_init", "rvcp_rccl_attach", "rvcp_gather_frame_async",
            "rvcp_gather_wait", "rvcp_render_frames_async", "rvcp_rccl_set_timeout",
            "rvcp_abi_version", "rvcp_set_code_cache_dir", "rvcp_code_cache_counts"]


# Integrator mode 2 (ray_tracer.comp ray_trace): its own #defines (ray_tracer.comp:5-13).
LEGACY_DEFAULTS = dict(device=0, integrator=1, spp=5, max_bounces=3, attenuation_stop_eps=0.01,
                       ray_t_min=0.01, ray_t_max=1000.0, rr_probability=1.0, eps=0.001,
                       lum_id_std140_quirk=1, kernel_variant=0, accel=0, n_gpus=1, unorm_rule=0, specialize=0,
                       grid_waves_per_simd=0)
INTEGRATOR_GAMES101, INTEGRATOR_LEGACY = 0, 1
ACCEL_NONE, ACCEL_BVH = 0, 1
UNORM_DRIVER, UNORM_NEAREST = 0, 1
SPECIALIZE_AUTO, SPECIALIZE_OFF = 0, 1


def make_config(**kw) -> np.ndarray:
    """rvcp_config_t with the #define defaults of the selected integrator, overridden by kw."""
    cfg = np.zeros((), dtype=CONFIG_DTYPE)
    vals = dict(LEGACY_DEFAULTS if kw.get("integrator", 0) == INTEGRATOR_LEGACY else DEFAULTS)
    vals.update(kw)
    for k, v in vals.items():
        cfg[k] = v
    return cfg


class RvcpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rvcp error {code}: {msg}")
        self.code = code


_lib = None


def _share_torch_hip_runtime():
    """PyTorch-ROCm bundles its own libamdhip64.so and NEEDs it by the unversioned name, while
    librvcp NEEDs libamdhip64.so.7.  If librvcp loaded first, a later `import torch` would
    load a SECOND HIP runtime that sees no GPU.  Preloading torch's copy (soname
    libamdhip64.so.7) makes both resolve to one runtime whatever the import order, so device
    pointers and streams from torch are valid in librvcp.  RVCP_HIP_RUNTIME=system skips it."""
    if os.environ.get("RVCP_HIP_RUNTIME") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    # (RCCL is not preloaded: librvcp dlopen()s "librccl.so.1" when a gather needs it, which
    # resolves by soname to the copy `import torch` already loaded.  Preloading torch's
    # librccl.so before torch itself aborts the interpreter at exit.)
    for d in spec.submodule_search_locations:
        for name in ("libhsa-runtime64.so", "libamdhip64.so"):
            f = os.path.join(d, "lib", name)
            if os.path.exists(f):
                ctypes.CDLL(f, mode=ctypes.RTLD_GLOBAL)


def load():
    """Load librvcp.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"librvcp.so not built ({LIB_PATH}); run __graft_entry__.build()")
    _share_torch_hip_runtime()
    L = ctypes.CDLL(LIB_PATH)
    P, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.rvcp_version.restype = ctypes.c_char_p
    L.rvcp_abi_version.restype = u32
    L.rvcp_set_code_cache_dir.argtypes = [ctypes.c_char_p]
    L.rvcp_code_cache_counts.argtypes = [P]
    L.rvcp_config_default.argtypes = [P]
    L.rvcp_config_default_for.argtypes = [ctypes.c_int32, P]
    L.rvcp_create.argtypes = [P, ctypes.POINTER(ctypes.c_void_p)]
    L.rvcp_destroy.argtypes = [P]
    L.rvcp_last_error.argtypes = [P]
    L.rvcp_last_error.restype = ctypes.c_char_p
    L.rvcp_upload_scene.argtypes = [P, P, u32, P, u32, P, u32, P, u32, P, u32, P, u32]
    L.rvcp_upload_scene_file.argtypes = [P, ctypes.c_char_p, P]
    L.rvcp_mandelbrot.argtypes = [P, P, u32, u32, P, P, P]
    L.rvcp_render.argtypes = [P, P, u32, u32, P, P, P]
    L.rvcp_render_shard_async.argtypes = [P, P, u32, u32, u32, u32, P, P, P]
    L.rvcp_render_frames_async.argtypes = [P, P, u32, u32, u32, u32, u32, P, P, P]
    L.rvcp_sync_stats.argtypes = [P, P]
    L.rvcp_render_async.argtypes = [P, P, u32, u32, P, P, P]
    L.rvcp_wait.argtypes = [P, P]
    L.rvcp_shard_rows.argtypes = [u32, u32, u32]
    L.rvcp_shard_rows.restype = u32
    L.rvcp_assemble_frame_async.argtypes = [P, P, u32, u32, u32, u32, P, P]
    L.rvcp_rccl_unique_id.argtypes = [P]
    L.rvcp_rccl_init.argtypes = [P, P, u32, u32]
    L.rvcp_rccl_attach.argtypes = [P, P, u32, u32]
    L.rvcp_rccl_set_timeout.argtypes = [P, u32]
    L.rvcp_gather_frame_async.argtypes = [P, P, u32, u32, P, P, P]
    L.rvcp_gather_wait.argtypes = [P, P, P]
    for name in ("rvcp_config_default", "rvcp_config_default_for", "rvcp_create", "rvcp_destroy", "rvcp_upload_scene",
                 "rvcp_render", "rvcp_render_shard_async", "rvcp_sync_stats",
                 "rvcp_assemble_frame_async", "rvcp_upload_scene_file", "rvcp_mandelbrot",
                 "rvcp_render_async", "rvcp_wait", "rvcp_rccl_unique_id", "rvcp_rccl_init",
                 "rvcp_rccl_attach", "rvcp_gather_frame_async", "rvcp_gather_wait",
                 "rvcp_render_frames_async", "rvcp_rccl_set_timeout", "rvcp_set_code_cache_dir",
                 "rvcp_code_cache_counts"):
        getattr(L, name).restype = ctypes.c_int
    if L.rvcp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI revision {L.rvcp_abi_version()}, this binding "
                           f"follows {ABI_VERSION} (rebuild: __graft_entry__.build())")
    _lib = L
    return L


def ptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    return a.ctypes.data_as(ctypes.c_void_p)


def set_code_cache_dir(path):
    """rvcp_set_code_cache_dir: the on-disk cache of scene-specialised code objects (None or ""
    disables it; default $XDG_CACHE_HOME/rvcp-mi355x, else ~/.cache/rvcp-mi355x)."""
    rc = load().rvcp_set_code_cache_dir(None if path is None else os.fsencode(path))
    if rc != RVCP_OK:
        raise RvcpError(rc, "rvcp_set_code_cache_dir failed")


def code_cache_counts():
    """rvcp_code_cache_counts: dict(loads, compiles, rejects) of the on-disk module cache."""
    out = (ctypes.c_uint64 * 3)()
    rc = load().rvcp_code_cache_counts(ctypes.cast(out, ctypes.c_void_p))
    if rc != RVCP_OK:
        raise RvcpError(rc, "rvcp_code_cache_counts failed")
    return dict(loads=int(out[0]), compiles=int(out[1]), rejects=int(out[2]))
