"""Opt-in BVH (rvcp_config_t.accel = RVCP_ACCEL_BVH) against the brute-force parity path.

The BVH tests only triangles whose enlarged boxes the ray reaches, with the same exact
triangle test and nearest-hit rule, so frames are expected to be identical to the
brute-force frames; the one documented exception is a ray running almost
parallel to a triangle's plane, where the exact test can accept a hit outside every box.
Tolerance here: bit-identical linear RGB on every pixel, and identical traversal counts, for
the scenes below (none of them is expected to hit the exception); a mismatch count is
reported if one appears."""
import numpy as np
import pytest

import rvcp_amd

pytestmark = pytest.mark.gpu


def _render(sc, W, H, time=5.0, **kw):
    with rvcp_amd.RayTracer(rvcp_amd.abi.make_config(**kw)) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(W, H, time, want_linear=True)
        return rgba, lin, rt.last_stats


def _same(sc, W, H, time=5.0, **kw):
    a = _render(sc, W, H, time, **kw)
    b = _render(sc, W, H, time, accel=rvcp_amd.abi.ACCEL_BVH, **kw)
    diff = np.any(a[1].view(np.uint32) != b[1].view(np.uint32), axis=-1)
    assert not diff.any(), f"{int(diff.sum())} of {diff.size} pixels differ"
    assert np.array_equal(a[0], b[0])
    assert int(a[2]["traversals"]) == int(b[2]["traversals"])
    return a, b


def test_bvh_cornell(cornell):
    _same(cornell, 96, 96, spp=4)


@pytest.mark.parametrize("n", [50, 2000])
def test_bvh_random_mesh(cornell, n):
    _same(rvcp_amd.scene.with_random_triangles(cornell, n), 64, 48, spp=2)


def test_bvh_c5_mesh(cornell):
    """The C5 mesh (Cornell + 100k random triangles)."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, 100000)
    _same(sc, 48, 48, spp=1)


@pytest.mark.parametrize("n", [310, 3000, 20000])
def test_bvh_hybrid_prefix(cornell, n):
    """The hybrid: the Cornell faces that lead the mesh are scanned by the
    scene-specialised module and left out of the BVH, which holds the random triangles only.
    The stats must name the specialised module, and the frame and traversal count must be
    the brute-force ones; 310 is the c6 mesh, the 20k case is large enough for carried
    traversals."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, n)
    _, b = _same(sc, 160, 128, spp=2, time=3.5)
    assert int(b[2]["kernel_variant"]) & rvcp_amd.abi.VARIANT_SPECIALIZED


def test_bvh_hybrid_prefix_generic(cornell):
    """ray_t_min = 0 leaves the specialised module's range (its exactness argument needs
    t_min > 0): the built-in BVH kernels then test the same prefix faces with the generic
    test before the BVH (bvh_prefix_scan<false>); frames and counts as the brute-force scan."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, 3000)
    _, b = _same(sc, 96, 80, spp=2, time=4.5, ray_t_min=0.0)
    assert not int(b[2]["kernel_variant"]) & rvcp_amd.abi.VARIANT_SPECIALIZED


def test_bvh_moved_camera(cornell):
    base = rvcp_amd.Scene(rvcp_amd.Camera.new([120.0, 400.0, -700.0], [-50.0, 150.0, 100.0],
                                              0.1, 10000.0, 55.0, 150.0, 5.0),
                          cornell.materials, [], cornell.mesh)
    _same(rvcp_amd.scene.with_random_triangles(base, 300), 64, 64, spp=2, time=1.5)


def _translated(sc, off):
    """The scene and its camera moved by `off` (float32): the quantised nodes' origins and
    power-of-two scales then sit far from the coordinate origin."""
    off = np.asarray(off, np.float32)
    v = sc.mesh.aligned_vertices().copy()
    v["position"][:, :3] = (v["position"][:, :3] + off).astype(np.float32)
    cam = sc.camera
    look = (cam.position + cam.forward * np.float32(100.0)).astype(np.float32)
    c2 = rvcp_amd.Camera.new((cam.position + off).astype(np.float32), (look + off).astype(np.float32),
                             cam.t_near, cam.t_far, cam.vertical_fov, cam.move_speed,
                             cam.rotate_speed)
    return rvcp_amd.Scene(c2, sc.materials, [], rvcp_amd.scene.ArrayMesh(v, sc.mesh.aligned_faces()))


def test_bvh_far_from_origin(cornell):
    """Byte-quantised nodes with the scene 3e4..5e4 units from the origin."""
    sc = _translated(rvcp_amd.scene.with_random_triangles(cornell, 500), [3.0e4, -2.0e4, 5.0e4])
    _same(sc, 48, 40, spp=2)


def test_bvh_flat_mesh(cornell):
    """Many triangles in one plane (zero extent on an axis before the build's enlargement)."""
    rng = np.random.default_rng(7)
    n = 400
    c = np.stack([rng.uniform(-250, 250, n), np.full(n, 1.0), rng.uniform(-250, 250, n)], 1)
    d = rng.uniform(-8, 8, (n, 3, 3))
    d[:, :, 1] = 0.0
    p = (c[:, None, :] + d).astype(np.float32)
    bv = cornell.mesh.aligned_vertices()
    bf = cornell.mesh.aligned_faces()
    nv = np.zeros(3 * n, dtype=bv.dtype)
    nv["position"][:, :3] = p.reshape(-1, 3)
    nv["normal"][:, :3] = np.array([0.0, 1.0, 0.0], np.float32)
    nf = np.zeros(n, dtype=bf.dtype)
    nf["vertices"] = len(bv) + np.arange(3 * n, dtype=np.uint32).reshape(n, 3)
    mesh = rvcp_amd.scene.ArrayMesh(np.concatenate([bv, nv]), np.concatenate([bf, nf]))
    _same(rvcp_amd.Scene(cornell.camera, cornell.materials, [], mesh), 48, 40, spp=2)


def test_bvh_obj_and_params(cornell):
    _same(cornell, 40, 40, spp=3, max_bounces=4, rr_probability=0.5, lum_id_std140_quirk=0)


def test_bvh_rejected_for_mode2():
    with pytest.raises(rvcp_amd.abi.RvcpError) as e:
        rvcp_amd.RayTracer(integrator=1, accel=rvcp_amd.abi.ACCEL_BVH)
    assert e.value.code == rvcp_amd.abi.RVCP_E_UNSUPPORTED


def test_bvh_full_c3_identical(cornell):
    a = _render(cornell, 1024, 1024, 123.0, spp=30)
    b = _render(cornell, 1024, 1024, 123.0, spp=30, accel=rvcp_amd.abi.ACCEL_BVH)
    assert np.array_equal(a[0], b[0])


def test_bvh_carried_traversals(cornell):
    """A frame large enough that the wave pools carry unfinished traversals into later
    iterations (bvh_pool): frozen owners and resumed stacks must leave every
    pixel and the traversal count as the brute-force scan has them."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, 20000)
    _same(sc, 192, 160, spp=4, time=2.5)
