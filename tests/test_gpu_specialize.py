"""The scene-specialised path kernels (rvcp_jit.cpp) on the GPU.

Every frame here is compared bit for bit (linear RGB bitwise, RGBA8 bytes, traversal count)
with the CPU oracle and/or with the generic kernels (rvcp_config_t.specialize = OFF); the
stats report which kernel ran (kernel_variant | RVCP_VARIANT_SPECIALIZED)."""
import time

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

pytestmark = pytest.mark.gpu
TIME = 123.0
SPEC = rvcp_amd.abi.VARIANT_SPECIALIZED


def _render(sc, W, H, time_=TIME, **kw):
    with rvcp_amd.RayTracer(**kw) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(W, H, time_, want_linear=True)
        return rgba, lin, rt.last_stats.copy()


def _same(a, b):
    assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    assert np.array_equal(a[0], b[0])
    assert int(a[2]["traversals"]) == int(b[2]["traversals"])


@pytest.mark.parametrize("W,H,spp", [(1024, 1024, 30), (384, 384, 10), (129, 67, 7)])
def test_specialised_equals_generic(cornell, W, H, spp):
    s = _render(cornell, W, H, spp=spp)
    g = _render(cornell, W, H, spp=spp, specialize=rvcp_amd.abi.SPECIALIZE_OFF)
    assert int(s[2]["kernel_variant"]) & SPEC and not int(g[2]["kernel_variant"]) & SPEC
    _same(s, g)


@pytest.mark.parametrize("case", ["quirk_off", "params", "moved_camera", "extra_tris", "seed"])
def test_specialised_vs_oracle(cornell, case):
    sc, kw, t = cornell, dict(spp=3), TIME
    if case == "quirk_off":
        kw["lum_id_std140_quirk"] = 0
    elif case == "params":
        kw.update(max_bounces=4, rr_probability=0.6, eps=0.01, ray_t_min=0.5, ray_t_max=900.0)
    elif case == "moved_camera":
        sc = rvcp_amd.Scene(rvcp_amd.Camera.new([120.0, 400.0, -700.0], [-50.0, 150.0, 100.0],
                                                0.1, 10000.0, 55.0, 150.0, 5.0),
                            cornell.materials, [], cornell.mesh)
    elif case == "extra_tris":        # 52 faces, 20 of them with no zero component
        sc = rvcp_amd.scene.with_random_triangles(cornell, 20)
    else:
        t = 987.0
    W, H = 96, 80
    s = _render(sc, W, H, t, **kw)
    assert int(s[2]["kernel_variant"]) & SPEC
    cfg = rvcp_amd.abi.make_config(**kw)
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(t), cfg, W, H)
    assert np.array_equal(s[1].view(np.uint32), o_lin.view(np.uint32))
    assert np.array_equal(s[0], o_rgba) and int(s[2]["traversals"]) == o_trav


def test_nonpositive_t_min_uses_generic(cornell):
    """The exactness argument needs t_min > 0: with ray_t_min = 0 the generic kernel runs."""
    s = _render(cornell, 64, 64, spp=2, ray_t_min=0.0)
    assert not int(s[2]["kernel_variant"]) & SPEC
    cfg = rvcp_amd.abi.make_config(spp=2, ray_t_min=0.0)
    o_lin, o_rgba, _ = O.render(scene_arrays(cornell), cornell.push_constant(TIME), cfg, 64, 64)
    assert np.array_equal(s[1].view(np.uint32), o_lin.view(np.uint32))


def test_large_scene_not_specialised(cornell):
    sc = rvcp_amd.scene.with_random_triangles(cornell, 100)
    s = _render(sc, 32, 32, spp=1)
    assert not int(s[2]["kernel_variant"]) & SPEC


def test_compiled_once_per_scene(cornell):
    """The module cache: a second context uploading the same scene does not recompile."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, 7)     # a scene no other test uses
    times = []
    for _ in range(2):
        with rvcp_amd.RayTracer(spp=1) as rt:
            t0 = time.perf_counter()
            rt.upload_scene(sc)
            times.append(time.perf_counter() - t0)
            rt.render(16, 16, TIME)
            assert int(rt.last_stats["kernel_variant"]) & SPEC
    assert times[1] < 0.5 * times[0] or times[0] < 0.05, times


_CACHE_CHILD = r"""
import json, sys, time
import numpy as np
import rvcp_amd
rvcp_amd.abi.set_code_cache_dir(sys.argv[1])
sc = rvcp_amd.Scene.default()
with rvcp_amd.RayTracer(spp=2) as rt:
    t0 = time.perf_counter()
    rt.upload_scene(sc)
    up = time.perf_counter() - t0
    img = rt.render(64, 48, 123.0)
    spec = bool(int(rt.last_stats["kernel_variant"]) & 16)
print(json.dumps(dict(upload_s=up, spec=spec, counts=rvcp_amd.abi.code_cache_counts(),
                      digest=int(np.frombuffer(img.tobytes(), np.uint64).sum() % (1 << 61)))))
"""


def test_code_cache_across_processes(tmp_path):
    """a second process uploading the Cornell scene loads the specialised
    module from the on-disk cache instead of compiling it (upload < 0.05 s), and renders the
    same frame; a corrupted entry is recompiled, not trusted."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cache = tmp_path / "cc"

    def child():
        r = subprocess.run([sys.executable, "-c", _CACHE_CHILD, str(cache)], cwd=root,
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-3000:]
        return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    first = child()
    assert first["spec"] and first["counts"]["compiles"] == 1 and first["counts"]["loads"] == 0
    second = child()
    assert second["spec"] and second["counts"] == dict(loads=1, compiles=0, rejects=0)
    assert second["upload_s"] < 0.05, (first["upload_s"], second["upload_s"])
    assert second["digest"] == first["digest"]
    (entry,) = list(cache.glob("*.rvcpco"))
    blob = bytearray(entry.read_bytes())
    blob[len(blob) // 2] ^= 0xFF                                   # inside the code object
    entry.write_bytes(bytes(blob))
    third = child()
    assert third["counts"] == dict(loads=0, compiles=1, rejects=1), third
    assert third["spec"] and third["digest"] == first["digest"]
    assert child()["counts"] == dict(loads=1, compiles=0, rejects=0)   # rewritten entry


@pytest.mark.parametrize("W,H,spp", [(1024, 1024, 5), (97, 61, 3)])
def test_specialised_mode2_equals_generic(W, H, spp):
    """Mode 2 (ray_tracer.comp) with the specialised triangle scan equals the generic mode-2
    kernel bit for bit (sphere room, 12 faces)."""
    sc = rvcp_amd.scene.sphere_scene()
    s = _render(sc, W, H, spp=spp, integrator=1)
    g = _render(sc, W, H, spp=spp, integrator=1, specialize=rvcp_amd.abi.SPECIALIZE_OFF)
    assert int(s[2]["kernel_variant"]) & SPEC and not int(g[2]["kernel_variant"]) & SPEC
    _same(s, g)


def test_specialised_mode2_vs_oracle():
    sc = rvcp_amd.scene.sphere_scene()
    kw = dict(spp=2, integrator=1)
    W, H = 80, 64
    s = _render(sc, W, H, **kw)
    assert int(s[2]["kernel_variant"]) & SPEC
    cfg = rvcp_amd.abi.make_config(**kw)
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(TIME), cfg, W, H)
    assert np.array_equal(s[1].view(np.uint32), o_lin.view(np.uint32))
    assert np.array_equal(s[0], o_rgba)
    assert int(s[2]["traversals"]) == int(o_trav)


def test_specialised_mode2_t_min_zero_vs_oracle():
    """Secondary rays with t_min = 0: the specialised mode-2 kernel's per-wave guard takes the
    generic scan (and the IEEE sphere roots) for them."""
    sc = rvcp_amd.scene.sphere_scene()
    kw = dict(spp=2, integrator=1, ray_t_min=0.0)
    s = _render(sc, 48, 40, **kw)
    cfg = rvcp_amd.abi.make_config(**kw)
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(TIME), cfg, 48, 40)
    assert np.array_equal(s[1].view(np.uint32), o_lin.view(np.uint32))
    assert np.array_equal(s[0], o_rgba)


def _with_huge_wall(base, scale=1e20):
    """The Cornell box plus a wall behind the camera (z = -1100, facing +z) whose two triangles
    reach +-scale in x and y: paths leaving through the open side hit it at t ~ 1e3, and its
    coordinates are far outside the specialised scan's range."""
    ArrayMesh, VERTEX_DTYPE, FACE_DTYPE = (rvcp_amd.scene.ArrayMesh, rvcp_amd.scene.VERTEX_DTYPE,
                                           rvcp_amd.scene.FACE_DTYPE)
    bv = base.mesh.aligned_vertices()
    bf = base.mesh.aligned_faces()
    s = np.float32(scale)
    nv = np.zeros(4, dtype=VERTEX_DTYPE)
    nv["position"][:, :3] = np.array([[-s, -s, -1100.0], [s, -s, -1100.0], [s, s, -1100.0],
                                      [-s, s, -1100.0]], np.float32)
    nv["normal"][:, :3] = [0.0, 0.0, 1.0]
    nf = np.zeros(2, dtype=FACE_DTYPE)
    nf["vertices"] = len(bv) + np.array([[0, 1, 2], [0, 2, 3]], np.uint32)
    nf["material_id"] = 0
    mesh = ArrayMesh(np.concatenate([bv, nv]), np.concatenate([bf, nf]))
    return rvcp_amd.Scene(base.camera, list(base.materials), list(base.spheres), mesh)


@pytest.mark.parametrize("integrator", [0, 1])
def test_out_of_range_scene_uses_generic_vs_oracle(cornell, integrator):
    """A scene with coordinates around 1e20 (where the generic test's intermediates overflow
    and inf * 0 = NaN decides) is not specialised (jit_scene_in_range), and its frame equals
    the oracle's bit for bit."""
    sc = _with_huge_wall(cornell)
    kw = dict(spp=3, integrator=integrator)
    W, H = 64, 48
    s = _render(sc, W, H, **kw)
    assert not int(s[2]["kernel_variant"]) & SPEC
    cfg = rvcp_amd.abi.make_config(**kw)
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(TIME), cfg, W, H)
    assert np.array_equal(s[1].view(np.uint32), o_lin.view(np.uint32))
    assert np.array_equal(s[0], o_rgba) and int(s[2]["traversals"]) == int(o_trav)
    # the same wall at 2^38 is in range: specialised, and still the oracle's frame
    sc2 = _with_huge_wall(cornell, 2.0 ** 38)
    s2 = _render(sc2, W, H, **kw)
    assert int(s2[2]["kernel_variant"]) & SPEC
    o_lin2, o_rgba2, _ = O.render(scene_arrays(sc2), sc2.push_constant(TIME), cfg, W, H)
    assert np.array_equal(s2[1].view(np.uint32), o_lin2.view(np.uint32))
    assert np.array_equal(s2[0], o_rgba2)
