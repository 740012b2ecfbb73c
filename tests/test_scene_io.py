"""Scene formats (rvcp_amd.scene_io): the binary upload-array dump (.rvcpscn, read natively by
rvcp_upload_scene_file) and the Wavefront OBJ/MTL loader."""
import os
import struct

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

S = rvcp_amd.scene_io


def _scenes():
    return {"cornell": rvcp_amd.Scene.default(), "spheres": rvcp_amd.scene.sphere_scene(),
            "random": rvcp_amd.scene.with_random_triangles(rvcp_amd.Scene.default(), 500)}


@pytest.mark.parametrize("name", ["cornell", "spheres", "random"])
def test_binary_round_trip(tmp_path, name):
    sc = _scenes()[name]
    p = str(tmp_path / f"{name}.rvcpscn")
    S.save(p, sc)
    back = S.load(p)
    a, b = scene_arrays(sc), scene_arrays(back)
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k
    assert back.camera.aligned().tobytes() == sc.camera.aligned().tobytes()
    assert back.luminous_sphere_ids().tobytes() == sc.luminous_sphere_ids().tobytes()
    assert back.camera.move_speed == np.float32(sc.camera.move_speed)


def test_binary_layout(tmp_path):
    sc = rvcp_amd.scene.sphere_scene()
    p = str(tmp_path / "s.rvcpscn")
    S.save(p, sc)
    raw = open(p, "rb").read()
    assert raw[:8] == b"RVCPSCN1"
    assert struct.unpack_from("<II", raw, 8) == (1, 128)
    lengths = struct.unpack_from("<6I", raw, 16)             # rvcp_lengths_t order
    assert lengths == (11, 8, 28, 12, len(sc.luminous_sphere_ids()), 2)
    assert raw[40:104] == sc.camera.aligned().tobytes()
    assert raw[128:128 + 32] == sc.aligned_materials()[:1].tobytes()
    assert len(raw) == 128 + 32 * (11 + 8 + 28) + 16 * 12 + 4 * (lengths[4] + lengths[5])


@pytest.mark.parametrize("damage", ["magic", "truncate", "trailing", "version"])
def test_binary_rejects_damaged(tmp_path, damage):
    p = str(tmp_path / "c.rvcpscn")
    S.save(p, rvcp_amd.Scene.default())
    raw = bytearray(open(p, "rb").read())
    if damage == "magic":
        raw[0] = ord("X")
    elif damage == "truncate":
        raw = raw[:-3]
    elif damage == "trailing":
        raw += b"\0"
    else:
        raw[8] = 2
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        S.load(p)


OBJ = """# a unit cube with a light quad above it
mtllib cube.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
v 1 0 1
v 1 1 1
v 0 1 1
vn 0 0 -1
vn 0 0 1
usemtl red
f 1//1 4//1 3//1 2//1
f 5//2 6//2 7//2 8//2
usemtl white
f 1 2 6 5
f -5 -1 -2 -6
usemtl lamp
v 0.25 2 0.25
v 0.75 2 0.25
v 0.75 2 0.75
v 0.25 2 0.75
f 9 10 11 12
usemtl glass
f 2 3 7
usemtl nosuch
f 1 5 8
"""
MTL = """newmtl red
Kd 0.8 0.1 0.1
newmtl white
Kd 0.7 0.7 0.7
newmtl lamp
Kd 0 0 0
Ke 10 9 8
newmtl glass
Ni 1.5
d 0.5
"""


def _write_obj(tmp_path):
    (tmp_path / "cube.mtl").write_text(MTL)
    p = tmp_path / "cube.obj"
    p.write_text(OBJ)
    return str(p)


def test_obj_loader(tmp_path):
    sc = S.load_obj(_write_obj(tmp_path))
    f = sc.mesh.aligned_faces()
    v = sc.mesh.aligned_vertices()
    assert len(f) == 2 + 2 + 2 + 2 + 2 + 1 + 1          # 5 quads fan-split, 2 triangles
    tys = [int(m.ty) for m in sc.materials]
    assert tys == [0, 0, 0, 3, 2]       # default, red, white, lamp, glass
    assert np.allclose(sc.materials[1].albedo, [0.8, 0.1, 0.1])
    assert np.allclose(sc.materials[3].albedo, [10, 9, 8])
    assert abs(sc.materials[4].refraction_ratio - 1.5) < 1e-7
    assert list(f["material_id"]) == [1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 4, 0]
    # face 0 uses the explicit normal (0, 0, -1); the white quads get geometric normals
    assert np.array_equal(v[f[0]["vertices"][0]]["normal"][:3], np.array([0, 0, -1], np.float32))
    n = v[f[4]["vertices"][0]]["normal"][:3]
    assert np.allclose(n, [0, -1, 0], atol=1e-6) or np.allclose(n, [0, 1, 0], atol=1e-6)
    # the negative-index quad is f 4 8 7 3 (the y = 1 face)
    ys = v[f[6]["vertices"]]["position"][:, 1]
    assert np.all(ys == 1.0)
    assert list(sc.luminous_face_ids()) == [8, 9]


def test_obj_vertex_split_and_render(tmp_path):
    sc = S.load_obj(_write_obj(tmp_path))
    v = sc.mesh.aligned_vertices()
    # corner 1 is used with normal (0,0,-1) and with per-face geometric normals
    at0 = [i for i in range(len(v)) if np.array_equal(v[i]["position"][:3], np.zeros(3, np.float32))]
    assert len(at0) >= 3
    lin, rgba, trav = O.render(scene_arrays(sc), sc.push_constant(1.0),
                               rvcp_amd.abi.make_config(spp=2), 32, 32)
    assert trav >= 32 * 32 * 2 and np.isfinite(lin).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell", "spheres", "random"])
def test_native_file_upload_matches_arrays(tmp_path, name):
    sc = _scenes()[name]
    p = str(tmp_path / f"{name}.rvcpscn")
    S.save(p, sc)
    integ = 1 if name == "spheres" else 0
    cfg = rvcp_amd.abi.make_config(integrator=integ, spp=2)
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(sc)
        ref = rt.render(64, 48, 5.0)
    with rvcp_amd.RayTracer(cfg) as rt:
        cam = rt.upload_scene_file(p)
        got = rt.render(64, 48, 5.0)
    assert cam.tobytes() == sc.camera.aligned().tobytes()
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_native_file_upload_rejects_damaged(tmp_path):
    p = str(tmp_path / "c.rvcpscn")
    S.save(p, rvcp_amd.Scene.default())
    raw = open(p, "rb").read()
    open(p, "wb").write(raw[:-1])
    with rvcp_amd.RayTracer(spp=1) as rt:
        with pytest.raises(rvcp_amd.abi.RvcpError) as e:
            rt.upload_scene_file(p)
        assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID
        with pytest.raises(rvcp_amd.abi.RvcpError):
            rt.upload_scene_file(str(tmp_path / "missing.rvcpscn"))


@pytest.mark.gpu
def test_obj_scene_bitexact(tmp_path):
    sc = S.load_obj(_write_obj(tmp_path))
    cfg = rvcp_amd.abi.make_config(spp=3)
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(40, 40, 2.0, want_linear=True)
        st = rt.last_stats
    o_lin, o_rgba, o_trav = O.render(scene_arrays(sc), sc.push_constant(2.0), cfg, 40, 40)
    assert np.array_equal(lin.view(np.uint32), o_lin.view(np.uint32))
    assert np.array_equal(rgba, o_rgba) and int(st["traversals"]) == o_trav
