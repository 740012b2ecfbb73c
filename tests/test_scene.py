"""Host-side scene model (mirror of src/ray_tracer/scene/*.rs): no GPU."""
import hashlib

import numpy as np

import rvcp_amd
from rvcp_amd import scene as S


def test_cornell_counts(cornell):
    # scene/mod.rs:21-259: 68 vertices, 32 faces (back wall commented out), 4 materials
    assert list(cornell.lengths()) == [4, 0, 68, 32, 0, 2]
    assert list(cornell.luminous_face_ids()) == [0, 1]


def test_cornell_camera_basis(cornell):
    cam = cornell.camera
    assert np.array_equal(cam.forward, [0, 0, 1]) and np.array_equal(cam.up, [0, 1, 0])
    assert np.array_equal(cam.right, [-1, 0, 0])
    rec = cam.aligned()
    assert np.array_equal(rec["position"], [0, 274, -1050, 0])
    assert rec["t_near"] == np.float32(0.1) and rec["vertical_fov"] == np.float32(40.0)


def test_cornell_geometry(cornell):
    v = cornell.mesh.aligned_vertices()
    assert np.all(v["position"][0:4, 1] == np.float32(548.8) - np.float32(0.01))   # light y
    assert np.all(np.abs(v["position"][:, [0, 2]]) <= 275.0)
    n = v["normal"][:, :3].astype(np.float64)
    assert np.allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-6)
    # tall box v01 side normal: (v1 - v0) x Y normalised (mod.rs:54)
    d = np.array([265.0 - 423.0, 0.0, 296.0 - 247.0])
    expect = np.cross(d, [0, 1, 0])
    assert np.allclose(v["normal"][32, :3], expect / np.linalg.norm(expect), atol=1e-7)
    f = cornell.mesh.aligned_faces()
    assert f["vertices"].max() == 67 and set(f["material_id"].tolist()) == {0, 1, 2, 3}


def test_light_material(cornell):
    m = cornell.aligned_materials()
    assert int(m[3]["ty"]) == 3
    assert np.allclose(m[3]["albedo"], [47.8348, 38.5664, 31.0808], atol=1e-3)


def test_metal_fuzz_assert():
    import pytest
    with pytest.raises(ValueError):
        S.Material.new_metal([1, 1, 1], 1.5)            # material.rs:52


def test_random_triangles_deterministic(cornell):
    a = S.with_random_triangles(cornell, 1000)
    b = S.with_random_triangles(cornell, 1000)
    assert a.mesh.aligned_vertices().tobytes() == b.mesh.aligned_vertices().tobytes()
    v = a.mesh.aligned_vertices()[68:]
    c = v["position"][:, :3].reshape(-1, 3, 3).mean(axis=1)
    assert c[:, 0].min() > -271 and c[:, 0].max() < 271 and c[:, 1].min() > 4 and c[:, 1].max() < 544
    assert len(a.luminous_face_ids()) == 2


def test_c5_buffers_pinned(cornell):
    """SHA-256 of the C5 (Cornell + 100k random triangles) upload buffers, so the benchmark
    scene cannot drift silently (SURVEY.md §8(d) C5 generator)."""
    sc = S.with_random_triangles(cornell, 100000)
    h = hashlib.sha256()
    h.update(sc.mesh.aligned_vertices().tobytes())
    h.update(sc.mesh.aligned_faces().tobytes())
    assert len(sc.mesh.aligned_faces()) == 100032
    assert h.hexdigest() == C5_SHA256


C5_SHA256 = "c3ec005e6ca14f9ff73518a1c57cb11d7e7212df05667b06a9ff31628951ac49"


def test_splitmix64_reference_values():
    # splitmix64 reference output for seed 0 (Vigna's published test vector)
    out = S.splitmix64(0, 3)
    assert [int(x) for x in out] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]
