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


def test_bvh_moved_camera(cornell):
    base = rvcp_amd.Scene(rvcp_amd.Camera.new([120.0, 400.0, -700.0], [-50.0, 150.0, 100.0],
                                              0.1, 10000.0, 55.0, 150.0, 5.0),
                          cornell.materials, [], cornell.mesh)
    _same(rvcp_amd.scene.with_random_triangles(base, 300), 64, 64, spp=2, time=1.5)


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
