"""Integrator mode 2 -- ray_trace of assets/shaders/ray_tracer.comp, the file north_star names
-- HIP kernel vs CPU oracle (run on an MI355X: pytest -m gpu).

Tolerance: bit-exact, as for games101: linear RGB bitwise equal, RGBA8
equal, traversal counts equal.  Scenes: the deprecated host's sphere room
(src/ray_tracer_deprecated/scene/mod.rs:21-185, scene.sphere_scene), the Cornell box, and
seeded random sphere fields exercising every material branch (Lambertian, metal with and
without fuzz, dielectric seen from outside and from inside, unknown material types).
"""
import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

pytestmark = pytest.mark.gpu
LEGACY = rvcp_amd.abi.INTEGRATOR_LEGACY


def _cfg(**kw):
    return rvcp_amd.abi.make_config(integrator=LEGACY, **kw)


def _oracle(sc, cfg, W, H, time, rect=None):
    return O.render(scene_arrays(sc), sc.push_constant(time), cfg, W, H, rect=rect)


def _gpu(sc, cfg, W, H, time):
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(W, H, time, want_linear=True)
        return rgba, lin, rt.last_stats


def _assert_same(gpu, orc):
    rgba, lin, stats = gpu
    o_lin, o_rgba, o_trav = orc
    diff = np.any(lin.view(np.uint32) != o_lin.view(np.uint32), axis=-1)
    assert not diff.any(), f"{int(diff.sum())} pixels differ in linear RGB, first at " \
                           f"{np.argwhere(diff)[:3].tolist()}"
    assert np.array_equal(rgba, o_rgba)
    assert int(stats["traversals"]) == o_trav


def _check(sc, cfg, W, H, time=3.25):
    _assert_same(_gpu(sc, cfg, W, H, time), _oracle(sc, cfg, W, H, time))


@pytest.fixture(scope="module")
def spheres():
    return rvcp_amd.scene.sphere_scene()


def sphere_field(n, seed, camera=None, extra_types=False):
    """n random spheres over the sphere room's floor, random materials of every type."""
    base = rvcp_amd.scene.sphere_scene()
    rng = np.random.default_rng(seed)
    mats = list(base.materials)
    sph = list(base.spheres)
    for _ in range(n):
        kind = int(rng.integers(0, 5 if extra_types else 4))
        if kind == 0:
            m = rvcp_amd.Material.new_lambertian(rng.uniform(0.05, 1.0, 3).astype(np.float32))
        elif kind == 1:
            m = rvcp_amd.Material.new_metal(rng.uniform(0.3, 1.0, 3).astype(np.float32),
                                            float(rng.choice([0.0, 0.1, 0.6])))
        elif kind == 2:
            m = rvcp_amd.Material.new_dielectric(float(rng.uniform(1.1, 2.6)))
        elif kind == 3:
            m = rvcp_amd.Material.new_light(rng.uniform(0.5, 1.5, 3).astype(np.float32))
        else:
            m = rvcp_amd.Material.new_lambertian([0.7, 0.7, 0.7])
            m.ty = 7                       # unknown type: attenuation 0 (ray_tracer.comp:655)
        mats.append(m)
        c = rvcp_amd.scene.vec3(rng.uniform(-4, 4), rng.uniform(0.1, 3.0), rng.uniform(-4, 2.5))
        sph.append(rvcp_amd.Sphere(c, float(np.float32(rng.uniform(0.1, 0.7))), len(mats) - 1))
    return rvcp_amd.Scene(camera or base.camera, mats, sph, base.mesh)


@pytest.mark.parametrize("W,H,spp", [(64, 64, 5), (128, 96, 1), (37, 23, 3), (8, 8, 30),
                                     (1, 1, 7), (130, 3, 2)])
def test_bitexact_sphere_scene(spheres, W, H, spp):
    _check(spheres, _cfg(spp=spp), W, H)


@pytest.mark.parametrize("kw", [dict(max_bounces=1), dict(max_bounces=8),
                                dict(max_bounces=12, rr_probability=0.7),
                                dict(rr_probability=0.5, spp=4),
                                dict(eps=0.05, ray_t_min=0.05),
                                dict(ray_t_max=4.0)])
def test_bitexact_params(spheres, kw):
    _check(spheres, _cfg(**kw), 48, 40)


@pytest.mark.parametrize("time", [0.0, 1.5, 999.0, 421.25])
def test_bitexact_time_seeds(spheres, time):
    _check(spheres, _cfg(spp=3), 40, 32, time=time)


def test_bitexact_cornell_mode2(cornell):
    _check(cornell, _cfg(spp=4, max_bounces=6), 64, 64, time=123.0)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bitexact_sphere_field(seed):
    sc = sphere_field(40, seed, extra_types=True)
    _check(sc, _cfg(spp=3, max_bounces=6), 64, 48, time=float(seed))


def test_bitexact_sphere_field_beyond_literals():
    """68 spheres: more than the specialised module writes as literals (rvcp_jit.cpp
    kJitMaxSpheres = 64), so its kernel keeps the loop over the records (and, with 68
    materials, reads them from global memory instead of LDS copies)."""
    sc = sphere_field(60, 4, extra_types=True)
    assert len(sc.spheres) > 64
    _check(sc, _cfg(spp=2, max_bounces=6), 48, 40, time=4.0)


def test_bitexact_sphere_literal_edge_values():
    """Sphere records the literal form must carry bit for bit: signed-zero centres, a negative
    and a zero radius, a subnormal coordinate (rvcp_jit.cpp jit_sphere_source)."""
    base = rvcp_amd.scene.sphere_scene()
    sph = list(base.spheres)
    vec3 = rvcp_amd.scene.vec3
    sph.append(rvcp_amd.Sphere(vec3(-0.0, 0.5, -0.0), 0.5, sph[0].material_id))
    sph.append(rvcp_amd.Sphere(vec3(0.75, 0.3, 0.5), -0.3, sph[1].material_id))
    sph.append(rvcp_amd.Sphere(vec3(-0.75, 0.3, 1e-40), 0.0, sph[2].material_id))
    sph.append(rvcp_amd.Sphere(vec3(-1.25, 0.35, 0.75), 0.35, sph[3].material_id))
    sc = rvcp_amd.Scene(base.camera, base.materials, sph, base.mesh)
    _check(sc, _cfg(spp=3, max_bounces=6), 56, 40, time=2.5)


@pytest.mark.parametrize("seed", [0, 1])
def test_bitexact_extreme_sphere_roots(seed):
    """The FAST sphere roots (rvcp_kernels.hip sphere_accept: Markstein quotients, no swap) on
    spheres whose root numerators -b -+ sq leave [2^-60, 2^60]: a ground sphere of radius
    1e19 whose surface passes near the room's floor (cancellation, |b| ~ 2e19), spheres 3e18
    and 1e19 away (roots beyond 2^30 in both forms, b^2 overflowing to inf so that sq = inf and
    the Markstein quotients are NaN where the IEEE roots are +-inf), a sphere of radius 2^-70
    (delta ~ 0) and one of radius 0 -- each decision and accepted t must be the shader's."""
    base = rvcp_amd.scene.sphere_scene()
    vec3 = rvcp_amd.scene.vec3
    mats = list(base.materials)
    sph = list(base.spheres)
    m0 = sph[0].material_id
    rng = np.random.default_rng(seed)
    sph.append(rvcp_amd.Sphere(vec3(0.0, -1e19, 0.0), 1e19, sph[1].material_id))
    sph.append(rvcp_amd.Sphere(vec3(3e18, 0.5, 0.0), 1.0, m0))
    sph.append(rvcp_amd.Sphere(vec3(0.0, 1e19, 1e19), 2.0, m0))
    sph.append(rvcp_amd.Sphere(vec3(-2.5, 1.0, 0.5), 2.0 ** -70, m0))
    sph.append(rvcp_amd.Sphere(vec3(2.5, 1.5, 1.0), 0.0, m0))
    for _ in range(6):                     # and ordinary ones of every material around them
        sph.append(rvcp_amd.Sphere(vec3(rng.uniform(-4, 4), rng.uniform(0.2, 2.5),
                                        rng.uniform(-4, 2.5)),
                                   float(np.float32(rng.uniform(0.2, 0.9))),
                                   int(rng.integers(1, len(mats)))))
    sc = rvcp_amd.Scene(base.camera, mats, sph, base.mesh)
    _check(sc, _cfg(spp=3, max_bounces=6), 56, 40, time=1.75 + seed)


def test_bitexact_camera_inside_dielectric(spheres):
    """The camera inside a glass sphere: is_normal_outward = false on the first hit
    (ray_tracer.comp:316-319), refraction_ratio not inverted (:562)."""
    cam = rvcp_amd.Camera.new(rvcp_amd.scene.vec3(1.25, 0.25, 1.25),
                              rvcp_amd.scene.vec3(0.0, 0.5, -2.0), 0.01, 1000.0, 90.0, 3.0, 10.0)
    sc = rvcp_amd.Scene(cam, spheres.materials, spheres.spheres, spheres.mesh)
    _check(sc, _cfg(spp=4, max_bounces=8), 48, 48)


def test_bitexact_spheres_only():
    base = rvcp_amd.scene.sphere_scene()
    sc = rvcp_amd.Scene(base.camera, base.materials, base.spheres,
                        rvcp_amd.scene.ArrayMesh(base.mesh.aligned_vertices(),
                                                 base.mesh.aligned_faces()[:0]))
    _check(sc, _cfg(spp=2), 40, 30)


def test_bitexact_random_mesh_and_spheres():
    sc = rvcp_amd.scene.with_random_triangles(sphere_field(10, 9), 150)
    _check(sc, _cfg(spp=2, max_bounces=5), 40, 36)


def test_trivial_max_bounces_zero(spheres):
    rgba, lin, st = _gpu(spheres, _cfg(max_bounces=0), 16, 16, 1.0)
    assert (lin == 0).all() and (rgba[..., :3] == 0).all() and (rgba[..., 3] == 255).all()
    assert int(st["traversals"]) == 0
    _check(spheres, _cfg(max_bounces=0), 16, 16)


def test_kernel_variant_ignored(spheres):
    ref = _gpu(spheres, _cfg(spp=2), 32, 32, 2.0)
    for v in (1, 2, 3, 4):
        got = _gpu(spheres, _cfg(spp=2, kernel_variant=v), 32, 32, 2.0)
        assert np.array_equal(got[1].view(np.uint32), ref[1].view(np.uint32))


def test_sphere_material_validation(spheres):
    arrays = scene_arrays(spheres)
    sph = arrays["spheres"].copy()
    sph[3]["material_id"] = len(arrays["materials"])
    with rvcp_amd.RayTracer(_cfg()) as rt:
        with pytest.raises(rvcp_amd.abi.RvcpError) as e:
            rt.upload_arrays(arrays["materials"], arrays["vertices"], arrays["faces"],
                             arrays["lum_face_ids"], spheres=sph)
        assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID


# ---- full size: the deprecated host's 1024^2 window at its SPP=5 ----
@pytest.fixture(scope="module")
def full_render(spheres):
    with rvcp_amd.RayTracer(_cfg()) as rt:
        rt.upload_scene(spheres)
        a, lin = rt.render(1024, 1024, 5.0, want_linear=True)
        b = rt.render(1024, 1024, 5.0)
        return a, lin, b, rt.last_stats


def test_full_deterministic(full_render):
    a, _, b, _ = full_render
    assert np.array_equal(a, b)


def test_full_rows_bitexact(spheres, full_render):
    a, lin, _, st = full_render
    cfg = _cfg()
    for y0 in (0, 337, 512, 1016):
        o_lin, o_rgba, _ = _oracle(spheres, cfg, 1024, 1024, 5.0, rect=(0, y0, 1024, 8))
        assert np.array_equal(lin[y0:y0 + 8].view(np.uint32), o_lin.view(np.uint32)), y0
        assert np.array_equal(a[y0:y0 + 8], o_rgba), y0


def test_full_traversals(full_render):
    st = full_render[3]
    per_sample = int(st["traversals"]) / (1024 * 1024 * 5)
    assert 1.0 <= per_sample <= 3.0


@pytest.mark.parametrize("n_shards", [2, 3])
def test_shard_assembly_bitexact(spheres, full_render, n_shards):
    """Stripe sharding (the multi-GPU path) reproduces the single-GPU frame."""
    import torch
    a = full_render[0]
    W = H = 1024
    frame = np.empty_like(a)
    with rvcp_amd.RayTracer(_cfg()) as rt:
        rt.upload_scene(spheres)
        for k in range(n_shards):
            rows = rvcp_amd.shard_rows(H, k, n_shards)
            buf = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
            rt.render_shard_async(spheres.push_constant(5.0), W, H, k, n_shards, buf.data_ptr())
            rt.sync_stats()
            frame[rvcp_amd.shard_row_ids(H, k, n_shards)] = buf.cpu().numpy()
    assert np.array_equal(frame, a)
