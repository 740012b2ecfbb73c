"""C-ABI checks that need no GPU: struct layouts, exported symbols, host-only entry points."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import rvcp_amd
from rvcp_amd import abi, scene
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rvcp.h")

LAYOUT_PROG = r"""
#include <stdio.h>
#include <stddef.h>
#include "rvcp.h"
#define F(T, m) printf(#T "." #m " %zu\n", offsetof(T, m))
#define S(T) printf(#T " %zu\n", sizeof(T))
int main(void) {
  S(rvcp_camera_t); F(rvcp_camera_t, position); F(rvcp_camera_t, up); F(rvcp_camera_t, forward);
  F(rvcp_camera_t, t_near); F(rvcp_camera_t, t_far); F(rvcp_camera_t, vertical_fov);
  S(rvcp_push_constant_t); F(rvcp_push_constant_t, time);
  S(rvcp_material_t); F(rvcp_material_t, albedo); F(rvcp_material_t, ty); F(rvcp_material_t, fuzz);
  F(rvcp_material_t, refraction_ratio);
  S(rvcp_vertex_t); F(rvcp_vertex_t, position); F(rvcp_vertex_t, normal);
  S(rvcp_face_t); F(rvcp_face_t, vertices); F(rvcp_face_t, material_id);
  S(rvcp_sphere_t); F(rvcp_sphere_t, center); F(rvcp_sphere_t, radius); F(rvcp_sphere_t, material_id);
  S(rvcp_config_t); F(rvcp_config_t, spp); F(rvcp_config_t, max_bounces);
  F(rvcp_config_t, attenuation_stop_eps); F(rvcp_config_t, ray_t_min); F(rvcp_config_t, ray_t_max);
  F(rvcp_config_t, rr_probability); F(rvcp_config_t, eps); F(rvcp_config_t, lum_id_std140_quirk);
  F(rvcp_config_t, kernel_variant); F(rvcp_config_t, accel); F(rvcp_config_t, n_gpus); F(rvcp_config_t, unorm_rule); F(rvcp_config_t, specialize); F(rvcp_config_t, grid_waves_per_simd);
  S(rvcp_stats_t); F(rvcp_stats_t, kernel_ms); F(rvcp_stats_t, traversals);
  F(rvcp_stats_t, traversals_executed); F(rvcp_stats_t, samples); F(rvcp_stats_t, faces);
  F(rvcp_stats_t, wave_iterations); F(rvcp_stats_t, main_kernel_ms);
  F(rvcp_stats_t, shader_clock_ghz);
  S(rvcp_lengths_t);
  S(rvcp_mandelbrot_push_t); F(rvcp_mandelbrot_push_t, position); F(rvcp_mandelbrot_push_t, scale);
  return 0;
}
"""

DTYPES = {"rvcp_camera_t": scene.CAMERA_DTYPE, "rvcp_push_constant_t": scene.PUSH_DTYPE,
          "rvcp_material_t": scene.MATERIAL_DTYPE, "rvcp_vertex_t": scene.VERTEX_DTYPE,
          "rvcp_face_t": scene.FACE_DTYPE, "rvcp_sphere_t": scene.SPHERE_DTYPE,
          "rvcp_config_t": abi.CONFIG_DTYPE, "rvcp_stats_t": abi.STATS_DTYPE,
          "rvcp_mandelbrot_push_t": __import__("rvcp_amd").mandelbrot.MANDELBROT_PUSH_DTYPE}


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("layout")
    src, exe = d / "layout.c", d / "layout"
    src.write_text(LAYOUT_PROG)
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.dirname(HEADER),
                    str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in (line.split() for line in out.strip().splitlines())}


def test_header_compiles_as_cpp(tmp_path):
    src = tmp_path / "h.cpp"
    src.write_text('#include "rvcp.h"\nint main() { return 0; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I",
                    os.path.dirname(HEADER), str(src)], check=True)


def test_reference_struct_sizes(c_layout):
    # sizes the reference's Rust structs / GLSL blocks imply
    assert c_layout["rvcp_camera_t"] == 64            # AlignedCamera, camera.rs:27-37
    assert c_layout["rvcp_push_constant_t"] == 68     # PushConstant, vulkan.rs:113-118
    assert c_layout["rvcp_push_constant_t.time"] == 64
    assert c_layout["rvcp_material_t"] == 32          # AlignedMaterial, material.rs:20-28
    assert c_layout["rvcp_vertex_t"] == 32            # AlignedVertex, mesh.rs:13-18
    assert c_layout["rvcp_face_t"] == 16              # AlignedFace, mesh.rs:37-42
    assert c_layout["rvcp_sphere_t"] == 32            # AlignedSphere, sphere.rs:10-17
    assert c_layout["rvcp_lengths_t"] == 24           # LengthBuffer, vulkan.rs:492-499
    # std430 push block: forward@32, t_near@44 (camera.rs:30-33)
    assert c_layout["rvcp_camera_t.forward"] == 32 and c_layout["rvcp_camera_t.t_near"] == 44


def test_numpy_dtypes_match_header(c_layout):
    for cname, dt in DTYPES.items():
        assert dt.itemsize == c_layout[cname], cname
        for field in dt.names:
            key = f"{cname}.{field}"
            if key in c_layout:
                assert dt.fields[field][1] == c_layout[key], key


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rvcp_[a-z_0-9]+)\s*\(", text)) - {"rvcp_ctx"})


def test_library_exports_every_declared_symbol():
    lib = abi.LIB_PATH
    assert os.path.exists(lib)
    out = subprocess.run(["nm", "-D", "--defined-only", lib], check=True, capture_output=True,
                         text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    declared = _declared_functions()
    assert declared, "no functions parsed from rvcp.h"
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(abi.EXPORTED) == declared


def test_abi_revision_matches_header_and_binding():
    """rvcp_stats_t grew to 64 B in revision 2; the header's RVCP_ABI_VERSION, the
    library's rvcp_abi_version() and the Python binding's struct layouts name one revision, and
    the version string says so (rvcp_abi_version needs no GPU)."""
    text = open(HEADER).read()
    m = re.search(r"#define RVCP_ABI_VERSION (\d+)", text)
    assert m and int(m.group(1)) == abi.ABI_VERSION == 2
    L = abi.load()
    assert L.rvcp_abi_version() == abi.ABI_VERSION
    assert b"ABI 2" in L.rvcp_version()
    assert abi.STATS_DTYPE.itemsize == 64


def test_library_links_no_oracle():
    """The product must not link or embed the CPU oracle."""
    out = subprocess.run(["nm", "-D", abi.LIB_PATH], check=True, capture_output=True, text=True).stdout
    assert "rvcp_oracle" not in out
    ldd = subprocess.run(["ldd", abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "amdhip64" in ldd


def test_product_library_reads_no_debug_knobs():
    """Experiment knobs (RVCP_DEBUG_*, RVCP_NO_SPECIALIZE) live only in the
    -DRVCP_DEBUG_KNOBS build (csrc/build/librvcp_debug.so); the product library must not
    change behaviour with the environment."""
    blob = open(abi.LIB_PATH, "rb").read()
    for knob in (b"RVCP_DEBUG_", b"RVCP_NO_SPECIALIZE", b"RVCP_JIT_FLAGS"):
        assert knob not in blob, knob
    dbg = os.path.join(os.path.dirname(abi.LIB_PATH), "librvcp_debug.so")
    if os.path.exists(dbg):
        assert b"RVCP_DEBUG_TIMELINE" in open(dbg, "rb").read()


def test_library_has_gfx950_code_object():
    blob = open(abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # the offload bundle targets gfx950
    assert b"games101_kernel" in blob
    assert b"legacy_kernel" in blob


def test_config_default_matches_reference_defines():
    L = abi.load()
    c = np.zeros((), dtype=abi.CONFIG_DTYPE)
    assert L.rvcp_config_default(abi.ptr(c)) == 0
    ref = abi.make_config()
    assert c.tobytes() == ref.tobytes()
    # ray_tracer_games101_branch.comp:5-13
    assert (int(c["spp"]), int(c["max_bounces"])) == (20, 15)
    assert np.float32(c["rr_probability"]) == np.float32(0.8)
    assert np.float32(c["eps"]) == np.float32(0.001)


def test_config_default_for_legacy_matches_ray_tracer_comp():
    L = abi.load()
    c = np.zeros((), dtype=abi.CONFIG_DTYPE)
    assert L.rvcp_config_default_for(abi.INTEGRATOR_LEGACY, abi.ptr(c)) == 0
    assert c.tobytes() == abi.make_config(integrator=abi.INTEGRATOR_LEGACY).tobytes()
    # ray_tracer.comp:5-13
    assert (int(c["integrator"]), int(c["spp"]), int(c["max_bounces"])) == (1, 5, 3)
    assert np.float32(c["rr_probability"]) == np.float32(1.0)
    assert np.float32(c["ray_t_max"]) == np.float32(1000.0)
    g = np.zeros((), dtype=abi.CONFIG_DTYPE)
    assert L.rvcp_config_default_for(abi.INTEGRATOR_GAMES101, abi.ptr(g)) == 0
    assert g.tobytes() == abi.make_config().tobytes()
    assert L.rvcp_config_default_for(9, abi.ptr(g)) == abi.RVCP_E_UNSUPPORTED


def test_create_rejects_bad_config_without_device():
    L = abi.load()
    h = ctypes.c_void_p()
    bad = abi.make_config(spp=0)
    assert L.rvcp_create(abi.ptr(bad), ctypes.byref(h)) == abi.RVCP_E_INVALID
    assert b"spp" in L.rvcp_last_error(None)
    bad = abi.make_config(integrator=7)
    assert L.rvcp_create(abi.ptr(bad), ctypes.byref(h)) == abi.RVCP_E_UNSUPPORTED
    assert L.rvcp_create(None, ctypes.byref(h)) == abi.RVCP_E_INVALID
    assert L.rvcp_destroy(None) == 0
    # 7 and 8 are not schedules; 9 (the BVH wavefront form) only with the BVH
    for v, accel in ((7, 0), (8, 1), (9, 0), (11, 0), (-1, 0)):
        bad = abi.make_config(kernel_variant=v, accel=accel)
        assert L.rvcp_create(abi.ptr(bad), ctypes.byref(h)) == abi.RVCP_E_INVALID, (v, accel)


def test_render_entry_points_reject_a_null_context():
    """The render entry points (including the frame batch) return RVCP_E_INVALID for a NULL
    context without touching a device."""
    L = abi.load()
    p = ctypes.c_void_p(1)
    assert L.rvcp_render_frames_async(None, p, 3, 64, 64, 0, 1, p, None, None) == abi.RVCP_E_INVALID
    assert L.rvcp_render_shard_async(None, p, 64, 64, 0, 1, p, None, None) == abi.RVCP_E_INVALID
    assert L.rvcp_render_async(None, p, 64, 64, p, None, None) == abi.RVCP_E_INVALID
    assert L.rvcp_sync_stats(None, None) == abi.RVCP_E_INVALID


def test_shard_rows_library_matches_python():
    L = abi.load()
    for H in (1, 7, 8, 9, 83, 1024, 1448, 2896):
        for n in (1, 2, 3, 4, 8):
            tot = 0
            for k in range(n):
                a = L.rvcp_shard_rows(H, k, n)
                assert a == rvcp_amd.shard_rows(H, k, n) == len(rvcp_amd.shard_row_ids(H, k, n))
                tot += a
            assert tot == H
    assert L.rvcp_shard_rows(100, 3, 3) == 0 and L.rvcp_shard_rows(100, 0, 0) == 0


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(abi, "_lib", None)
    monkeypatch.setattr(abi, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="not built"):
        rvcp_amd.RayTracer()
