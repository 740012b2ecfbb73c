"""Scene model: host-side mirror of the reference's ``src/ray_tracer/scene/*.rs``.

The classes keep the reference's names and fields (``Camera``, ``Material``, ``Vertex``,
``Face``, ``Mesh``, ``Sphere``, ``Scene``) and their ``aligned()`` methods produce numpy
records byte-identical to the ``Aligned*`` upload structs (``include/rvcp.h``).  All
arithmetic is float32, matching glam 0.29's ``Vec3`` (``v * (1 / sqrt(dot))`` normalise,
component-wise cross), so the uploaded bytes equal what the Rust host uploads.

``Scene.default()`` is the Cornell box of ``src/ray_tracer/scene/mod.rs:21-259``.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import enum
from dataclasses import dataclass, field
from typing import List

import numpy as np

f32 = np.float32

# Rust's f32 transcendental functions call the platform libm; use the same float functions.
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _n in ("sinf", "cosf", "asinf", "tanf"):
    getattr(_libm, _n).argtypes = [ctypes.c_float]
    getattr(_libm, _n).restype = ctypes.c_float
_libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
_libm.atan2f.restype = ctypes.c_float
# core::f32::to_radians / to_degrees constants
RADS_PER_DEG = f32(f32(np.pi) / f32(180.0))
DEGS_PER_RAD = f32(57.2957795130823208767981548141051703)

# --------------------------------------------------------------------------------------
# numpy record types == include/rvcp.h structs
# --------------------------------------------------------------------------------------
CAMERA_DTYPE = np.dtype([("position", "<f4", 4), ("up", "<f4", 4), ("forward", "<f4", 3),
                         ("t_near", "<f4"), ("t_far", "<f4"), ("vertical_fov", "<f4"),
                         ("_padding", "<u4", 2)])
PUSH_DTYPE = np.dtype([("camera", CAMERA_DTYPE), ("time", "<f4")])
MATERIAL_DTYPE = np.dtype([("albedo", "<f4", 3), ("ty", "<u4"), ("fuzz", "<f4"),
                           ("refraction_ratio", "<f4"), ("_padding", "<u4", 2)])
VERTEX_DTYPE = np.dtype([("position", "<f4", 4), ("normal", "<f4", 4)])
FACE_DTYPE = np.dtype([("vertices", "<u4", 3), ("material_id", "<u4")])
SPHERE_DTYPE = np.dtype([("center", "<f4", 3), ("radius", "<f4"), ("material_id", "<u4"),
                         ("_padding", "<u4", 3)])

assert CAMERA_DTYPE.itemsize == 64 and PUSH_DTYPE.itemsize == 68
assert MATERIAL_DTYPE.itemsize == 32 and VERTEX_DTYPE.itemsize == 32
assert FACE_DTYPE.itemsize == 16 and SPHERE_DTYPE.itemsize == 32


# --------------------------------------------------------------------------------------
# glam-style f32 vector helpers
# --------------------------------------------------------------------------------------
def vec3(x, y, z) -> np.ndarray:
    return np.array([x, y, z], dtype=f32)


def _dot(a, b) -> np.float32:
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def cross(a, b) -> np.ndarray:
    """glam ``Vec3::cross`` (component-wise, f32)."""
    return np.array([f32(a[1] * b[2]) - f32(b[1] * a[2]),
                     f32(a[2] * b[0]) - f32(b[2] * a[0]),
                     f32(a[0] * b[1]) - f32(b[0] * a[1])], dtype=f32)


def normalize(a) -> np.ndarray:
    """glam ``Vec3::normalize`` = ``self * (1.0 / self.length())`` in f32."""
    inv = f32(f32(1.0) / np.sqrt(_dot(a, a), dtype=f32))
    return (a * inv).astype(f32)


Y = vec3(0.0, 1.0, 0.0)


# --------------------------------------------------------------------------------------
# Camera: src/ray_tracer/scene/camera.rs:6-90
# --------------------------------------------------------------------------------------
@dataclass
class Camera:
    position: np.ndarray
    t_near: float
    t_far: float
    vertical_fov: float
    move_speed: float
    rotate_speed: float
    up: np.ndarray
    forward: np.ndarray
    right: np.ndarray
    yaw: float
    pitch: float

    @staticmethod
    def new(position, look_at, t_near, t_far, vertical_fov, move_speed, rotate_speed) -> "Camera":
        """``Camera::new`` (camera.rs:52-90): forward/right/up basis from a look-at point."""
        position = np.asarray(position, dtype=f32)
        look_at = np.asarray(look_at, dtype=f32)
        forward = normalize((look_at - position).astype(f32))
        right = normalize(cross(forward, Y))
        up = normalize(cross(right, forward))
        # forward.z.atan2(forward.x).to_degrees(), forward.y.asin().to_degrees() in f32
        yaw = float(f32(f32(_libm.atan2f(float(forward[2]), float(forward[0]))) * DEGS_PER_RAD))
        pitch = float(f32(f32(_libm.asinf(float(forward[1]))) * DEGS_PER_RAD))
        return Camera(position, float(f32(t_near)), float(f32(t_far)), float(f32(vertical_fov)),
                      float(move_speed), float(rotate_speed), up, forward, right, yaw, pitch)

    def aligned(self) -> np.ndarray:
        """``Camera::aligned`` (camera.rs:39-50) -> one CAMERA_DTYPE record."""
        rec = np.zeros((), dtype=CAMERA_DTYPE)
        rec["position"][:3] = self.position
        rec["up"][:3] = self.up
        rec["forward"] = self.forward
        rec["t_near"] = self.t_near
        rec["t_far"] = self.t_far
        rec["vertical_fov"] = self.vertical_fov
        return rec


def push_constant(camera: Camera, time: float) -> np.ndarray:
    """``PushConstant::new(camera.aligned(), time)`` (vulkan.rs:113-127)."""
    rec = np.zeros((), dtype=PUSH_DTYPE)
    rec["camera"] = camera.aligned()
    rec["time"] = time
    return rec


# --------------------------------------------------------------------------------------
# Material: src/ray_tracer/scene/material.rs
# --------------------------------------------------------------------------------------
class MaterialType(enum.IntEnum):
    Lambertian = 0
    Metal = 1
    Dielectric = 2
    Light = 3


@dataclass
class Material:
    ty: MaterialType
    albedo: np.ndarray
    fuzz: float = 0.0
    refraction_ratio: float = 0.0

    @staticmethod
    def new_lambertian(albedo) -> "Material":
        return Material(MaterialType.Lambertian, np.asarray(albedo, dtype=f32))

    @staticmethod
    def new_metal(albedo, fuzz) -> "Material":
        if not fuzz <= 1.0:                      # material.rs:52 assert!(fuzz <= 1.0)
            raise ValueError("fuzz must be <= 1.0")
        return Material(MaterialType.Metal, np.asarray(albedo, dtype=f32), float(fuzz))

    @staticmethod
    def new_dielectric(refraction_ratio) -> "Material":
        return Material(MaterialType.Dielectric, vec3(1.0, 1.0, 1.0), 0.0, float(refraction_ratio))

    @staticmethod
    def new_light(luminance) -> "Material":
        return Material(MaterialType.Light, np.asarray(luminance, dtype=f32))

    def aligned(self) -> np.ndarray:
        rec = np.zeros((), dtype=MATERIAL_DTYPE)
        rec["albedo"] = self.albedo
        rec["ty"] = int(self.ty)
        rec["fuzz"] = self.fuzz
        rec["refraction_ratio"] = self.refraction_ratio
        return rec


# --------------------------------------------------------------------------------------
# Mesh: src/ray_tracer/scene/mesh.rs ; Sphere: scene/sphere.rs
# --------------------------------------------------------------------------------------
@dataclass
class Vertex:
    position: np.ndarray
    normal: np.ndarray


@dataclass
class Face:
    vertices: tuple
    material_id: int


@dataclass
class Mesh:
    vertices: List[Vertex] = field(default_factory=list)
    faces: List[Face] = field(default_factory=list)

    def aligned_vertices(self) -> np.ndarray:
        out = np.zeros(len(self.vertices), dtype=VERTEX_DTYPE)
        for i, v in enumerate(self.vertices):
            out[i]["position"][:3] = v.position
            out[i]["normal"][:3] = v.normal
        return out

    def aligned_faces(self) -> np.ndarray:
        out = np.zeros(len(self.faces), dtype=FACE_DTYPE)
        for i, f in enumerate(self.faces):
            out[i]["vertices"] = f.vertices
            out[i]["material_id"] = f.material_id
        return out


@dataclass
class Sphere:
    center: np.ndarray
    radius: float
    material_id: int

    def aligned(self) -> np.ndarray:
        rec = np.zeros((), dtype=SPHERE_DTYPE)
        rec["center"] = self.center
        rec["radius"] = self.radius
        rec["material_id"] = self.material_id
        return rec


# --------------------------------------------------------------------------------------
# Scene: src/ray_tracer/scene/mod.rs
# --------------------------------------------------------------------------------------
@dataclass
class Scene:
    camera: Camera
    materials: List[Material]
    spheres: List[Sphere]
    mesh: Mesh

    # ---- upload views (what Vk::create_descriptor_set_0s builds, vulkan.rs:467-552) ----
    def aligned_materials(self) -> np.ndarray:
        return np.array([m.aligned() for m in self.materials], dtype=MATERIAL_DTYPE)

    def aligned_spheres(self) -> np.ndarray:
        return np.array([s.aligned() for s in self.spheres], dtype=SPHERE_DTYPE).reshape(-1)

    def luminous_face_ids(self) -> np.ndarray:
        """Faces whose material is a Light (vulkan.rs:473-478), packed u32."""
        light = np.array([m.ty == MaterialType.Light for m in self.materials], dtype=bool)
        mat_ids = self.mesh.aligned_faces()["material_id"]
        return np.nonzero(light[mat_ids])[0].astype(np.uint32)

    def luminous_sphere_ids(self) -> np.ndarray:
        ids = [i for i, s in enumerate(self.spheres)
               if self.materials[s.material_id].ty == MaterialType.Light]
        return np.array(ids, dtype=np.uint32)

    def lengths(self) -> np.ndarray:
        """The LengthBuffer (vulkan.rs:492-499)."""
        return np.array([len(self.materials), len(self.spheres), len(self.mesh.aligned_vertices()),
                         len(self.mesh.aligned_faces()), len(self.luminous_sphere_ids()),
                         len(self.luminous_face_ids())], dtype=np.uint32)

    def push_constant(self, time: float) -> np.ndarray:
        return push_constant(self.camera, time)

    @staticmethod
    def default() -> "Scene":
        return cornell_box()


def cornell_box() -> Scene:
    """``impl Default for Scene`` (src/ray_tracer/scene/mod.rs:21-259), in f32."""
    camera = Camera.new(vec3(0.0, 274.0, -1050.0), vec3(0.0, 274.0, 0.0),
                        0.1, 10000.0, 40.0, 150.0, 5.0)                       # mod.rs:23-32

    def s(x):
        return f32(x)

    light = (s(8.0) * vec3(s(0.747) + s(0.058), s(0.747) + s(0.258), s(0.747))).astype(f32)
    light = (light + (s(15.6) * vec3(s(0.740) + s(0.287), s(0.740) + s(0.160), s(0.740))).astype(f32)).astype(f32)
    light = (light + (s(18.4) * vec3(s(0.737) + s(0.642), s(0.737) + s(0.159), s(0.737))).astype(f32)).astype(f32)
    materials = [
        Material.new_lambertian(vec3(0.725, 0.71, 0.68)),    # white
        Material.new_lambertian(vec3(0.63, 0.065, 0.05)),    # red
        Material.new_lambertian(vec3(0.14, 0.45, 0.091)),    # green
        Material.new_light(light),                            # mod.rs:38-40
    ]

    H = s(548.8)          # cornel_height
    W = s(275.0)          # cornel_width
    LW = s(60.0)          # cornel_light_width
    tall_h = s(330.0)
    tv = [vec3(423.0, 0.0, 247.0), vec3(265.0, 0.0, 296.0), vec3(314.0, 0.0, 456.0),
          vec3(472.0, 0.0, 406.0)]
    short_h = s(165.0)
    sv = [vec3(130.0, 0.0, 65.0), vec3(82.0, 0.0, 225.0), vec3(240.0, 0.0, 272.0),
          vec3(290.0, 0.0, 114.0)]

    def side_normal(a, b):
        return normalize(cross((b - a).astype(f32), Y))

    delta = vec3(-W, 0.0, -W)
    up_n, down_n = vec3(0.0, 1.0, 0.0), vec3(0.0, -1.0, 0.0)
    V = []

    def quad(ps, n):
        for p in ps:
            V.append(Vertex(np.asarray(p, dtype=f32), np.asarray(n, dtype=f32)))

    ly = s(H - s(0.01))
    quad([vec3(-LW, ly, -LW), vec3(-LW, ly, LW), vec3(LW, ly, LW), vec3(LW, ly, -LW)], down_n)   # light
    quad([vec3(-W, H, -W), vec3(-W, H, W), vec3(W, H, W), vec3(W, H, -W)], down_n)               # top
    quad([vec3(-W, 0.0, -W), vec3(-W, 0.0, W), vec3(-W, H, W), vec3(-W, H, -W)], vec3(1, 0, 0))  # left
    quad([vec3(W, 0.0, -W), vec3(W, 0.0, W), vec3(W, H, W), vec3(W, H, -W)], vec3(-1, 0, 0))     # right
    quad([vec3(-W, 0.0, W), vec3(W, 0.0, W), vec3(W, H, W), vec3(-W, H, W)], vec3(0, 0, -1))     # front
    quad([vec3(-W, 0.0, -W), vec3(W, 0.0, -W), vec3(W, H, -W), vec3(-W, H, -W)], vec3(0, 0, 1))  # back
    quad([vec3(-W, 0.0, -W), vec3(-W, 0.0, W), vec3(W, 0.0, W), vec3(W, 0.0, -W)], up_n)         # bottom

    def box(v, h):
        lift = vec3(0.0, h, 0.0)
        quad([(delta + vec3(p[0], h, p[2])).astype(f32) for p in v], up_n)                       # top
        for a, b in ((0, 1), (1, 2), (2, 3), (3, 0)):                                            # sides
            n = side_normal(v[a], v[b])
            quad([(delta + v[a]).astype(f32), (delta + v[b]).astype(f32),
                  ((delta + v[b]).astype(f32) + lift).astype(f32),
                  ((delta + v[a]).astype(f32) + lift).astype(f32)], n)

    box(tv, tall_h)
    box(sv, short_h)

    F = []

    def qf(base, mat):
        F.append(Face((base, base + 1, base + 2), mat))
        F.append(Face((base, base + 2, base + 3), mat))

    qf(0, 3)     # top light
    qf(4, 0)     # top
    qf(8, 2)     # left (green)
    qf(12, 1)    # right (red)
    qf(16, 0)    # front
    # back (20..23) is commented out in mod.rs:201-203
    qf(24, 0)    # bottom
    for base in range(28, 68, 4):   # tall box top + 4 sides, short box top + 4 sides
        qf(base, 0)
    return Scene(camera, materials, [], Mesh(V, F))


def rotated_scene(base: Scene, yaw_deg: float = 23.0, pitch_deg: float = 17.0,
                  roll_deg: float = 11.0, center=(0.0, 274.4, 0.0)) -> Scene:
    """`base` with its mesh AND camera turned by R = Rz(roll) Rx(pitch) Ry(yaw) about `center` (the
    Cornell box's middle): every vertex p -> f32(c + R (p - c)) and normal n ->
    normalize(f32(R n)) (rotation in float64, one rounding), the camera re-built by
    Camera::new from its turned position and look-at point.  The camera keeps the world up
    axis (camera.rs:62-68), so the box appears turned in the frame, with the same content.
    No triangle of the Cornell box keeps an exact-zero position or edge component, so the
    scene-specialised scan has no product to drop: this is the bench's
    off-axis workload (`bench.py --workload c3rot`)."""
    a, b, g = np.radians(yaw_deg), np.radians(pitch_deg), np.radians(roll_deg)
    ry = np.array([[np.cos(a), 0.0, np.sin(a)], [0.0, 1.0, 0.0], [-np.sin(a), 0.0, np.cos(a)]])
    rx = np.array([[1.0, 0.0, 0.0], [0.0, np.cos(b), -np.sin(b)], [0.0, np.sin(b), np.cos(b)]])
    rz = np.array([[np.cos(g), -np.sin(g), 0.0], [np.sin(g), np.cos(g), 0.0], [0.0, 0.0, 1.0]])
    R = rz @ rx @ ry
    c = np.asarray(center, dtype=np.float64)

    def turn(p):
        return (c + R @ (np.asarray(p, dtype=np.float64) - c)).astype(f32)

    bv = base.mesh.aligned_vertices().copy()
    pos = bv["position"][:, :3].astype(np.float64)
    bv["position"][:, :3] = (c + (pos - c) @ R.T).astype(f32)
    nr = (bv["normal"][:, :3].astype(np.float64) @ R.T).astype(f32)
    bv["normal"][:, :3] = np.stack([normalize(n) for n in nr])
    cam = base.camera
    look = (cam.position.astype(np.float64) + 1050.0 * cam.forward.astype(np.float64))
    camera = Camera.new(turn(cam.position), turn(look), cam.t_near, cam.t_far, cam.vertical_fov,
                        cam.move_speed, cam.rotate_speed)
    mesh = ArrayMesh(bv, base.mesh.aligned_faces().copy())
    return Scene(camera, list(base.materials), list(base.spheres), mesh)


# --------------------------------------------------------------------------------------
# Synthetic large-mesh workload (BASELINE.json configs[4]; SURVEY.md §8(d) "C5 generator")
# --------------------------------------------------------------------------------------
C5_SEED = 0x5256435020241022


def splitmix64(seed: int, n: int) -> np.ndarray:
    """First n outputs of splitmix64 seeded with `seed` (vectorised: output i mixes
    seed + (i+1) * golden_gamma mod 2^64)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform(bits: np.ndarray, lo: float, hi: float) -> np.ndarray:
    u = (bits >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)   # [0, 1)
    return (np.float32(lo) + np.float32(hi - lo) * u).astype(np.float32)


class ArrayMesh(Mesh):
    """A mesh held directly as upload arrays (VERTEX_DTYPE / FACE_DTYPE records)."""

    def __init__(self, vertices: np.ndarray, faces: np.ndarray):
        super().__init__([], [])
        self._v = np.ascontiguousarray(vertices, dtype=VERTEX_DTYPE)
        self._f = np.ascontiguousarray(faces, dtype=FACE_DTYPE)

    def aligned_vertices(self) -> np.ndarray:
        return self._v

    def aligned_faces(self) -> np.ndarray:
        return self._f

    @property
    def n_vertices(self):
        return len(self._v)

    @property
    def n_faces(self):
        return len(self._f)


def with_random_triangles(base: Scene, n: int, seed: int = C5_SEED) -> Scene:
    """Append n random small triangles to `base` (material 0, white Lambertian):
    centroid c ~ U([-265,265] x [10,538] x [-265,265]), v_k = c + U([-5,5]^3), per-vertex
    normal = normalize(cross(v1 - v0, v2 - v0)); 12 splitmix64 draws per triangle in the
    order c.xyz, d0.xyz, d1.xyz, d2.xyz."""
    bits = splitmix64(seed, 12 * n).reshape(n, 12)
    c = np.stack([_uniform(bits[:, 0], -265, 265), _uniform(bits[:, 1], 10, 538),
                  _uniform(bits[:, 2], -265, 265)], axis=1)
    d = _uniform(bits[:, 3:], -5, 5).reshape(n, 3, 3)
    p = (c[:, None, :] + d).astype(np.float32)                     # [n, 3 verts, xyz]
    e1 = (p[:, 1] - p[:, 0]).astype(np.float32)
    e2 = (p[:, 2] - p[:, 0]).astype(np.float32)
    cr = np.stack([(e1[:, 1] * e2[:, 2]).astype(np.float32) - (e2[:, 1] * e1[:, 2]).astype(np.float32),
                   (e1[:, 2] * e2[:, 0]).astype(np.float32) - (e2[:, 2] * e1[:, 0]).astype(np.float32),
                   (e1[:, 0] * e2[:, 1]).astype(np.float32) - (e2[:, 0] * e1[:, 1]).astype(np.float32)],
                  axis=1).astype(np.float32)
    dd = ((cr[:, 0] * cr[:, 0]).astype(np.float32) + (cr[:, 1] * cr[:, 1]).astype(np.float32)).astype(np.float32)
    dd = (dd + (cr[:, 2] * cr[:, 2]).astype(np.float32)).astype(np.float32)
    inv = (np.float32(1.0) / np.sqrt(dd).astype(np.float32)).astype(np.float32)
    nrm = (cr * inv[:, None]).astype(np.float32)

    bv = base.mesh.aligned_vertices()
    bf = base.mesh.aligned_faces()
    nv = np.zeros(3 * n, dtype=VERTEX_DTYPE)
    nv["position"][:, :3] = p.reshape(3 * n, 3)
    nv["normal"][:, :3] = np.repeat(nrm, 3, axis=0)
    nf = np.zeros(n, dtype=FACE_DTYPE)
    nf["vertices"] = len(bv) + np.arange(3 * n, dtype=np.uint32).reshape(n, 3)
    nf["material_id"] = 0
    mesh = ArrayMesh(np.concatenate([bv, nv]), np.concatenate([bf, nf]))
    sc = Scene(base.camera, list(base.materials), list(base.spheres), mesh)
    return sc


# --------------------------------------------------------------------------------------
# Sphere scene of the deprecated host (integrator mode 2 fixture)
# --------------------------------------------------------------------------------------
def sphere_scene() -> Scene:
    """``impl Default for Scene`` of src/ray_tracer_deprecated/scene/mod.rs:21-185: 8 spheres,
    11 materials (Lambertian, metal, dielectric, light), an open-front room of 12 faces."""
    camera = Camera.new(vec3(0.0, 1.0, 3.0), vec3(0.0, 0.0, 0.0), 0.1, 1000.0, 120.0, 3.0, 10.0)
    materials = [
        Material.new_lambertian(vec3(1.0, 1.0, 1.0)),
        Material.new_lambertian(vec3(0.8, 0.3, 0.3)),
        Material.new_lambertian(vec3(0.3, 0.7, 0.3)),
        Material.new_metal(vec3(0.8, 0.8, 0.8), 0.3),
        Material.new_metal(vec3(1.0, 1.0, 1.0), 0.0),
        Material.new_metal(vec3(0.5, 0.4, 0.9), 0.3),
        Material.new_dielectric(1.3),
        Material.new_dielectric(2.5),
        Material.new_light(vec3(1.0, 1.0, 1.0)),
        Material.new_lambertian(vec3(1.0, 0.0, 0.0)),     # red
        Material.new_lambertian(vec3(0.0, 1.0, 0.0)),     # green
    ]
    spheres = [Sphere(vec3(*c), float(np.float32(r)), m) for c, r, m in [
        ((0.0, 1.0, 0.0), 1.0, 1), ((-1.5, 0.5, 2.0), 0.5, 2), ((-2.0, 1.0, 0.0), 1.0, 3),
        ((0.0, 0.25, 1.75), 0.25, 4), ((1.5, 0.25, 1.75), 0.25, 5), ((1.25, 0.25, 1.25), 0.25, 6),
        ((2.0, 1.0, 0.0), 1.0, 7), ((-1.0, 0.25, 1.0), 0.25, 8)]]
    Hh, Ww, LW = f32(5.0), f32(5.0), f32(5.0)
    ly = f32(Hh - f32(0.01))
    V = []

    def quad(ps, n):
        for p in ps:
            V.append(Vertex(np.asarray(p, dtype=f32), np.asarray(n, dtype=f32)))

    quad([vec3(-LW, ly, -LW), vec3(-LW, ly, LW), vec3(LW, ly, LW), vec3(LW, ly, -LW)], vec3(0, 1, 0))
    quad([vec3(-Ww, Hh, -Ww), vec3(-Ww, Hh, Ww), vec3(Ww, Hh, Ww), vec3(Ww, Hh, -Ww)], vec3(0, -1, 0))
    quad([vec3(-Ww, 0, -Ww), vec3(-Ww, 0, Ww), vec3(-Ww, Hh, Ww), vec3(-Ww, Hh, -Ww)], vec3(1, 0, 0))
    quad([vec3(Ww, 0, -Ww), vec3(Ww, 0, Ww), vec3(Ww, Hh, Ww), vec3(Ww, Hh, -Ww)], vec3(-1, 0, 0))
    quad([vec3(-Ww, 0, Ww), vec3(Ww, 0, Ww), vec3(Ww, Hh, Ww), vec3(-Ww, Hh, Ww)], vec3(0, 0, -1))
    quad([vec3(-Ww, 0, -Ww), vec3(Ww, 0, -Ww), vec3(Ww, Hh, -Ww), vec3(-Ww, Hh, -Ww)], vec3(0, 0, 1))
    quad([vec3(-Ww, 0, -Ww), vec3(-Ww, 0, Ww), vec3(Ww, 0, Ww), vec3(Ww, 0, -Ww)], vec3(0, 1, 0))
    F = []
    for base, mat in ((0, 8), (4, 0), (8, 9), (12, 10), (20, 0), (24, 0)):   # front commented out
        F.append(Face((base, base + 1, base + 2), mat))
        F.append(Face((base, base + 2, base + 3), mat))
    return Scene(camera, materials, spheres, Mesh(V, F))
