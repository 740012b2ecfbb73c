"""Fuzz of the scene-specialised scan's exactness proof on the GPU.

The headline kernel is code generated per scene (rvcp_jit.cpp): products with exact-zero
components dropped, reciprocals without their class check where a grain/magnitude analysis
proves the denominator zero or normal.  A wrong bound would change
bits silently on exactly the path that sets the headline, so every seeded scene of
tests/fuzz_scenes.py -- scales 2^-20 .. 2^38, slivers, point/line-degenerate, coplanar and
duplicated triangles, mixed axis-aligned and off-axis faces, cameras inside the geometry,
t_min / eps / bounce / quirk variations -- is rendered three ways and compared bit for bit:

    specialised scan (the default; asserted to have run) == generic scan (specialize = OFF)
                                                         == the CPU oracle

on linear RGB bits, RGBA8 bytes and the reference-algorithm traversal count
(ray_tracer_games101_branch.comp:238-298 is the scan being specialised)."""
import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays
from fuzz_scenes import N_FUZZ, fuzz_scene

pytestmark = pytest.mark.gpu
SPEC = rvcp_amd.abi.VARIANT_SPECIALIZED
W, H = 48, 40


def _render(sc, t, **kw):
    with rvcp_amd.RayTracer(**kw) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(W, H, t, want_linear=True)
        return rgba, lin, rt.last_stats.copy()


def _diff(a, b):
    return int(np.count_nonzero(np.any(a[1].view(np.uint32) != b[1].view(np.uint32), axis=-1)))


@pytest.mark.parametrize("seed", range(N_FUZZ))
def test_specialised_equals_generic_equals_oracle(seed):
    sc, kw, desc = fuzz_scene(seed)
    t = 100.0 + seed
    s = _render(sc, t, **kw)
    g = _render(sc, t, specialize=rvcp_amd.abi.SPECIALIZE_OFF, **kw)
    assert int(s[2]["kernel_variant"]) & SPEC, desc
    assert not int(g[2]["kernel_variant"]) & SPEC
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(t),
                                     rvcp_amd.abi.make_config(**kw), W, H)
    o = (o_rgba, o_lin, {"traversals": o_trav})
    assert _diff(s, g) == 0, f"specialised != generic on {_diff(s, g)} pixels; {desc}"
    assert _diff(s, o) == 0, f"specialised != oracle on {_diff(s, o)} pixels; {desc}"
    assert np.array_equal(s[0], g[0]) and np.array_equal(s[0], o_rgba), desc
    assert int(s[2]["traversals"]) == int(g[2]["traversals"]) == int(o_trav), desc
    # not an empty frame: some paths hit the geometry
    assert int(o_trav) > W * H * kw["spp"], desc


def _with_specks(sc, n, seed):
    """The fuzz scene with n small triangles appended, scattered over its bounding box
    (material 0): enough faces behind the room for the BVH hybrid to leave
    the leading room faces to the specialised scan and build the BVH over the rest."""
    v = sc.mesh.aligned_vertices()
    f = sc.mesh.aligned_faces()
    pos = v["position"][:, :3].astype(np.float64)
    lo, hi = pos.min(0), pos.max(0)
    ext = np.maximum(hi - lo, 1e-30)
    rng = np.random.default_rng(0xB1D + seed)
    c = lo + rng.random((n, 3)) * ext
    p = (c[:, None, :] + (rng.random((n, 3, 3)) - 0.5) * ext / 64).astype(np.float32)
    V = rvcp_amd.scene.VERTEX_DTYPE
    F = rvcp_amd.scene.FACE_DTYPE
    nv = np.zeros(3 * n, V)
    nv["position"][:, :3] = p.reshape(3 * n, 3)
    nv["normal"][:, 1] = 1.0
    nf = np.zeros(n, F)
    nf["vertices"] = len(v) + np.arange(3 * n, dtype=np.uint32).reshape(n, 3)
    mesh = rvcp_amd.scene.ArrayMesh(np.concatenate([v, nv]), np.concatenate([f, nf]))
    return rvcp_amd.Scene(sc.camera, list(sc.materials), [], mesh)


def test_bvh_hybrid_fuzz():
    """The BVH hybrid on every fuzz scene with 160 small triangles appended: the specialised
    scan over the leading faces plus the BVH over the rest == the generic brute-force scan,
    bit for bit (linear RGB, RGBA8, traversal count).  The hybrid must engage (the stats name
    the specialised module) on most of the scenes."""
    engaged = 0
    for seed in range(N_FUZZ):
        sc0, kw, desc = fuzz_scene(seed)
        sc = _with_specks(sc0, 160, seed)
        t = 100.0 + seed
        b = _render(sc, t, accel=rvcp_amd.abi.ACCEL_BVH, **kw)
        g = _render(sc, t, specialize=rvcp_amd.abi.SPECIALIZE_OFF, **kw)
        engaged += bool(int(b[2]["kernel_variant"]) & SPEC)
        assert _diff(b, g) == 0, f"hybrid != generic on {_diff(b, g)} pixels; {desc}"
        assert np.array_equal(b[0], g[0]), desc
        assert int(b[2]["traversals"]) == int(g[2]["traversals"]), desc
    assert engaged >= N_FUZZ // 2, f"hybrid engaged on {engaged} of {N_FUZZ} scenes"


def _mode2_scene(sc, seed):
    """The fuzz scene for integrator mode 2 (ray_tracer.comp, the shader north_star names):
    its faces keep their materials with material 1 turned into a fuzzy metal, and two spheres
    -- a dielectric and a metal -- sit between the camera and its look point, sized to the
    room, so that every material branch of mode 2's scatter runs next to the specialised
    triangle scan."""
    M = rvcp_amd.scene.Material
    mats = [sc.materials[0], M.new_metal([0.8, 0.8, 0.8], 0.25), sc.materials[2],
            M.new_dielectric(1.5), M.new_metal([0.9, 0.6, 0.4], 0.0)]
    pos = sc.mesh.aligned_vertices()["position"][:, :3].astype(np.float64)
    lo, hi = pos.min(0), pos.max(0)
    c = (lo + hi) / 2
    r = float(np.float32(np.max(hi - lo) / 8))
    rng = np.random.default_rng(0x3D2 + seed)
    sph = [rvcp_amd.scene.Sphere((c + rng.uniform(-1, 1, 3) * r).astype(np.float32), r, 3),
           rvcp_amd.scene.Sphere((c + rng.uniform(-1, 1, 3) * r).astype(np.float32),
                                 float(np.float32(r / 2)), 4)]
    return rvcp_amd.Scene(sc.camera, mats, sph, sc.mesh)


@pytest.mark.parametrize("seed", range(N_FUZZ))
def test_mode2_specialised_equals_generic_equals_oracle(seed):
    """Mode 2 with the scene-specialised triangle scan (rvcp_spec_legacy_kernel) on every fuzz
    scene, with spheres of every material beside it: == the generic mode-2 kernel == the CPU
    oracle, bit for bit (ray_tracer.comp:300-393 is the scene intersection being specialised)."""
    sc0, kw, desc = fuzz_scene(seed)
    sc = _mode2_scene(sc0, seed)
    kw = dict(kw, integrator=rvcp_amd.abi.INTEGRATOR_LEGACY)
    t = 200.0 + seed
    s = _render(sc, t, **kw)
    g = _render(sc, t, specialize=rvcp_amd.abi.SPECIALIZE_OFF, **kw)
    assert int(s[2]["kernel_variant"]) & SPEC, desc
    assert not int(g[2]["kernel_variant"]) & SPEC
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(t),
                                     rvcp_amd.abi.make_config(**kw), W, H)
    o = (o_rgba, o_lin, {"traversals": o_trav})
    assert _diff(s, g) == 0, f"mode 2: specialised != generic on {_diff(s, g)} pixels; {desc}"
    assert _diff(s, o) == 0, f"mode 2: specialised != oracle on {_diff(s, o)} pixels; {desc}"
    assert np.array_equal(s[0], g[0]) and np.array_equal(s[0], o_rgba), desc
    assert int(s[2]["traversals"]) == int(g[2]["traversals"]) == int(o_trav), desc
