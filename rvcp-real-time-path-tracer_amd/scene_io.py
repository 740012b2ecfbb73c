"""Scene formats: a binary dump of the reference's upload arrays,
and a Wavefront OBJ (+ MTL) loader for meshes larger than the built-in scenes.

Binary scene file (``.rvcpscn``), little-endian, read natively by
``rvcp_upload_scene_file`` (include/rvcp.h) and by ``load`` below:

    off  size  field
      0     8  magic "RVCPSCN1"
      8     4  u32 version = 1
     12     4  u32 header bytes = 128
     16    24  rvcp_lengths_t: materials, spheres, vertices, faces, lum_sphere_ids,
               lum_face_ids (the LengthBuffer of vulkan.rs:481-500)
     40    64  rvcp_camera_t (AlignedCamera, camera.rs:27-37)
    104     8  f32 move_speed, f32 rotate_speed (camera.rs:15-16; not part of AlignedCamera)
    112    16  reserved (0)
    128     -  materials[] (32 B AlignedMaterial), spheres[] (32 B AlignedSphere),
               vertices[] (32 B AlignedVertex), faces[] (16 B AlignedFace),
               lum_sphere_ids[] (u32), lum_face_ids[] (u32, packed as vulkan.rs:473-478)

The arrays are exactly the bytes ``Vk::create_descriptor_set_0s`` uploads
(vulkan.rs:467-552), so a Rust host can write the file with ``bytemuck::cast_slice`` of the
same ``Vec``s.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

from .scene import (CAMERA_DTYPE, FACE_DTYPE, MATERIAL_DTYPE, SPHERE_DTYPE, VERTEX_DTYPE,
                    ArrayMesh, Camera, Material, MaterialType, Scene, Sphere, cross, normalize,
                    vec3)

f32 = np.float32
MAGIC = b"RVCPSCN1"
VERSION = 1
HEADER_BYTES = 128
_HEAD = struct.Struct("<8sII6I")          # magic, version, header bytes, lengths


def _camera_from_aligned(rec, move_speed: float, rotate_speed: float) -> Camera:
    """Rebuild a Camera from its AlignedCamera: Camera::new with look_at = position +
    forward, then the stored up (camera.rs:52-90 recomputes right/up from forward)."""
    pos = np.array(rec["position"][:3], dtype=f32)
    fwd = np.array(rec["forward"], dtype=f32)
    cam = Camera.new(pos, (pos + fwd).astype(f32), float(rec["t_near"]), float(rec["t_far"]),
                     float(rec["vertical_fov"]), move_speed, rotate_speed)
    # keep the exact stored vectors (the push constant carries them verbatim)
    cam.forward = fwd
    cam.up = np.array(rec["up"][:3], dtype=f32)
    cam.right = normalize(cross(fwd, vec3(0.0, 1.0, 0.0)))
    return cam


def save(path: str, scene: Scene) -> None:
    mats = scene.aligned_materials()
    sph = scene.aligned_spheres()
    verts = scene.mesh.aligned_vertices()
    faces = scene.mesh.aligned_faces()
    lsph = scene.luminous_sphere_ids().astype("<u4")
    lface = scene.luminous_face_ids().astype("<u4")
    cam = scene.camera.aligned()
    with open(path, "wb") as f:
        f.write(_HEAD.pack(MAGIC, VERSION, HEADER_BYTES, len(mats), len(sph), len(verts),
                           len(faces), len(lsph), len(lface)))
        f.write(np.ascontiguousarray(cam).tobytes())
        f.write(struct.pack("<ff", scene.camera.move_speed, scene.camera.rotate_speed))
        f.write(b"\0" * 16)
        for a in (mats, sph, verts, faces, lsph, lface):
            f.write(np.ascontiguousarray(a).tobytes())


def read_arrays(path: str) -> Dict[str, np.ndarray]:
    """The raw upload arrays + camera record of a scene file (validated)."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < HEADER_BYTES:
        raise ValueError("scene file too short")
    magic, version, hdr, nm, ns, nv, nf, nls, nlf = _HEAD.unpack_from(data, 0)
    if magic != MAGIC or version != VERSION or hdr != HEADER_BYTES:
        raise ValueError("not an RVCPSCN1 scene file")
    cam = np.frombuffer(data, dtype=CAMERA_DTYPE, count=1, offset=40)[0]
    move_speed, rotate_speed = struct.unpack_from("<ff", data, 104)
    off = HEADER_BYTES
    out = {"camera": cam, "move_speed": move_speed, "rotate_speed": rotate_speed}
    for key, dt, n in (("materials", MATERIAL_DTYPE, nm), ("spheres", SPHERE_DTYPE, ns),
                       ("vertices", VERTEX_DTYPE, nv), ("faces", FACE_DTYPE, nf),
                       ("lum_sphere_ids", np.dtype("<u4"), nls),
                       ("lum_face_ids", np.dtype("<u4"), nlf)):
        size = dt.itemsize * n
        if off + size > len(data):
            raise ValueError(f"scene file truncated in {key}")
        out[key] = np.frombuffer(data, dtype=dt, count=n, offset=off).copy()
        off += size
    if off != len(data):
        raise ValueError("trailing bytes after the scene arrays")
    return out


def load(path: str) -> Scene:
    a = read_arrays(path)
    mats = [Material(MaterialType(int(m["ty"])) if int(m["ty"]) in (0, 1, 2, 3) else int(m["ty"]),
                     np.array(m["albedo"], dtype=f32), float(m["fuzz"]),
                     float(m["refraction_ratio"])) for m in a["materials"]]
    sph = [Sphere(np.array(s["center"], dtype=f32), float(s["radius"]), int(s["material_id"]))
           for s in a["spheres"]]
    cam = _camera_from_aligned(a["camera"], a["move_speed"], a["rotate_speed"])
    return Scene(cam, mats, sph, ArrayMesh(a["vertices"], a["faces"]))


# --------------------------------------------------------------------------- OBJ / MTL
def _read_mtl(path: str) -> Dict[str, Material]:
    """Kd -> Lambertian albedo; Ke > 0 -> Light with Le = Ke; illum 3 -> Metal (fuzz from
    Pr roughness or 0); Ni with d < 1 or illum 4/6/7 -> Dielectric(Ni)."""
    mats: Dict[str, Material] = {}
    cur: Optional[dict] = None

    def finish():
        if cur is None:
            return
        kd = cur.get("Kd", (0.8, 0.8, 0.8))
        ke = cur.get("Ke", (0.0, 0.0, 0.0))
        illum = int(cur.get("illum", 2))
        if max(ke) > 0.0:
            m = Material.new_light(ke)
        elif illum in (4, 6, 7) or float(cur.get("d", 1.0)) < 1.0:
            m = Material.new_dielectric(float(cur.get("Ni", 1.5)))
        elif illum == 3:
            m = Material.new_metal(kd, min(1.0, float(cur.get("Pr", 0.0))))
        else:
            m = Material.new_lambertian(kd)
        mats[cur["name"]] = m

    with open(path) as f:
        for line in f:
            t = line.split()
            if not t or t[0].startswith("#"):
                continue
            if t[0] == "newmtl":
                finish()
                cur = {"name": " ".join(t[1:])}
            elif cur is not None and t[0] in ("Kd", "Ke"):
                cur[t[0]] = tuple(float(x) for x in t[1:4])
            elif cur is not None and t[0] in ("Ni", "d", "Pr", "illum"):
                cur[t[0]] = t[1]
    finish()
    return mats


def load_obj(path: str, camera: Optional[Camera] = None,
             materials: Optional[Dict[str, Material]] = None,
             default_material: Optional[Material] = None) -> Scene:
    """Load a Wavefront OBJ as a Scene.  Polygons are fan-triangulated; negative (relative)
    indices are resolved; an OBJ vertex/normal pair becomes one AlignedVertex (split where a
    position is used with different normals); faces without normals get the normalised
    geometric normal of the triangle (the C5 generator's convention).
    Materials: ``usemtl`` names are looked up in ``materials`` (overrides), then in the
    ``mtllib`` files; unknown or absent names use ``default_material`` (white Lambertian).
    ``camera`` defaults to one looking at the mesh's bounding box from -z."""
    base = os.path.dirname(os.path.abspath(path))
    pos: List[Tuple[float, float, float]] = []
    nrm: List[Tuple[float, float, float]] = []
    mtl: Dict[str, Material] = {}
    mat_list: List[Material] = [default_material or Material.new_lambertian([0.8, 0.8, 0.8])]
    mat_index: Dict[str, int] = {}
    cur_mat = 0
    tris: List[Tuple[Tuple[int, int], Tuple[int, int], Tuple[int, int], int]] = []

    def idx(tok: str, n: int) -> int:
        i = int(tok)
        return i - 1 if i > 0 else n + i

    with open(path) as f:
        for line in f:
            t = line.split()
            if not t or t[0].startswith("#"):
                continue
            if t[0] == "v":
                pos.append(tuple(float(x) for x in t[1:4]))
            elif t[0] == "vn":
                nrm.append(tuple(float(x) for x in t[1:4]))
            elif t[0] == "mtllib":
                for name in t[1:]:
                    p = os.path.join(base, name)
                    if os.path.exists(p):
                        mtl.update(_read_mtl(p))
            elif t[0] == "usemtl":
                name = " ".join(t[1:])
                if name not in mat_index:
                    m = (materials or {}).get(name) or mtl.get(name)
                    if m is None:
                        mat_index[name] = 0
                    else:
                        mat_list.append(m)
                        mat_index[name] = len(mat_list) - 1
                cur_mat = mat_index[name]
            elif t[0] == "f":
                corners = []
                for c in t[1:]:
                    parts = c.split("/")
                    vi = idx(parts[0], len(pos))
                    ni = idx(parts[2], len(nrm)) if len(parts) > 2 and parts[2] else -1
                    corners.append((vi, ni))
                for k in range(1, len(corners) - 1):
                    tris.append((corners[0], corners[k], corners[k + 1], cur_mat))

    P = np.asarray(pos, dtype=f32).reshape(-1, 3)
    N = np.asarray(nrm, dtype=f32).reshape(-1, 3)
    verts: List[Tuple[np.ndarray, np.ndarray]] = []
    key_to_vid: Dict[Tuple, int] = {}
    faces = np.zeros(len(tris), dtype=FACE_DTYPE)
    for fi, (a, b, c, m) in enumerate(tris):
        geo = None
        if a[1] < 0 or b[1] < 0 or c[1] < 0:
            geo = normalize(cross((P[b[0]] - P[a[0]]).astype(f32), (P[c[0]] - P[a[0]]).astype(f32)))
        ids = []
        for (vi, ni) in (a, b, c):
            if ni >= 0:
                key = (vi, "n", ni)
                n = N[ni]
            else:
                key = (vi, "g", fi)             # geometric normals are per face
                n = geo
            vid = key_to_vid.get(key)
            if vid is None:
                vid = len(verts)
                key_to_vid[key] = vid
                verts.append((P[vi], n))
            ids.append(vid)
        faces[fi]["vertices"] = ids
        faces[fi]["material_id"] = m
    V = np.zeros(len(verts), dtype=VERTEX_DTYPE)
    for i, (p, n) in enumerate(verts):
        V[i]["position"][:3] = p
        V[i]["normal"][:3] = n
    if camera is None:
        lo, hi = (P.min(0), P.max(0)) if len(P) else (np.zeros(3, f32), np.ones(3, f32))
        c = ((lo + hi) * f32(0.5)).astype(f32)
        ext = float(np.max(hi - lo)) or 1.0
        eye = vec3(float(c[0]), float(c[1]), float(c[2]) - 2.0 * ext)
        camera = Camera.new(eye, c, 0.1, 10000.0, 40.0, 100.0, 10.0)
    return Scene(camera, mat_list, [], ArrayMesh(V, faces))
