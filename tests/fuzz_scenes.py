"""Seeded adversarial scenes for the scene-specialised scan's exactness proof (VERDICT r4 item 3;
rvcp_jit.cpp).

The specialised scan drops products with exact-zero triangle components and skips the
reciprocal's class check where an interval/grain analysis proves the denominator zero or
normal.  Those proofs depend on the triangles' magnitudes and lowest set bits, so the scenes
here span them: a room of axis-aligned quads (many exact zeros, coarse grains) at a scale of
2^-20 .. 2^22, for a third of the seeds translated (with its camera) by up to 2^38 -- so that
coordinates span 2^-20 .. 2^38 while the distances a path covers stay below the 2^24 that
rvcp_config_t.ray_t_max allows (the shader's miss test writes t_max + 1, :287) -- plus a mix
of off-axis triangles with random bits, slivers, point- and
line-degenerate triangles, coplanar overlapping and duplicated triangles, tiny and huge
triangles relative to the room, and cameras inside the geometry.  Each scene stays within the
specialisation's range (|v0| <= 2^40, |e| <= 2^41: jit_scene_in_range), has at most 64 faces
(kJitMaxFaces) and a luminous quad, and comes with a config whose ray_t_min / ray_t_max / eps
are scaled with it (or not: a fixed eps at a huge scale is one more case).

Pure numpy (test infrastructure); the scene follows ray_tracer_games101_branch.comp's inputs
(:74-111) through the package's Scene / ArrayMesh records.
"""
import numpy as np

import rvcp_amd

N_FUZZ = 36


def _normal(p0, p1, p2):
    n = np.cross((p1 - p0).astype(np.float64), (p2 - p0).astype(np.float64))
    ln = np.linalg.norm(n)
    return (n / ln).astype(np.float32) if ln > 0 and np.isfinite(ln) else np.float32([0, 1, 0])


def fuzz_scene(seed):
    """(scene, config kwargs, description) for fuzz case `seed`."""
    rng = np.random.default_rng(0x5EC0 + seed)
    e = int(rng.integers(-20, 23)) if seed >= 4 else [-20, 22, 0, 20][seed]
    s = np.float32(2.0 ** e)
    # a translation of the whole scene: none, or 2^20 .. 2^38 per axis (seeds 1 and 3 at 2^38)
    e_off = 38 if seed in (1, 3) else (int(rng.integers(20, 39)) if rng.random() < 0.34 else None)
    off = (np.zeros(3, np.float32) if e_off is None else
           (rng.choice([-1.0, 1.0], 3) * 2.0 ** e_off * rng.uniform(1, 1.9, 3)).astype(np.float32))
    if e_off is not None and e < e_off - 14:
        # the room at least 2^9 ulps of the offset across (else it collapses to a point and the
        # camera's rays to a few directions), within the 2^22 cap (seeds 1 and 3: 2^7 ulps)
        e = min(e_off - 14, 22)
        s = np.float32(2.0 ** e)
    tris, mats = [], []

    def add(p0, p1, p2, mat):
        tris.append(np.array([p0, p1, p2], np.float32))
        mats.append(mat)

    def quad(c, u, v, mat):
        c, u, v = (np.asarray(x, np.float32) for x in (c, u, v))
        a, b, cc, d = c - u - v, c + u - v, c + u + v, c - u + v
        add(a, b, cc, mat)
        add(a, cc, d, mat)

    # the room: floor, ceiling, back and side walls on axis planes, coordinates on a grid of
    # s / 8 (exact zeros in the edges, coarse lowest set bits); the light on the ceiling
    g = s / np.float32(8)
    walls = [((0, -8 * g, 0), (8 * g, 0, 0), (0, 0, 8 * g), 0),     # floor
             ((0, 8 * g, 0), (8 * g, 0, 0), (0, 0, -8 * g), 0),     # ceiling
             ((0, 0, 8 * g), (8 * g, 0, 0), (0, 8 * g, 0), 0),      # back wall
             ((-8 * g, 0, 0), (0, 0, 8 * g), (0, 8 * g, 0), 1),     # red wall
             ((8 * g, 0, 0), (0, 8 * g, 0), (0, 0, 8 * g), 0)]
    for c, u, v, m in walls[:int(rng.integers(3, 6))]:
        quad(c, u, v, m)
    quad((0, 7.875 * g, 0), (2 * g, 0, 0), (0, 0, 2 * g), 2)       # light, just below the ceiling
    kinds = []
    while len(tris) < int(rng.integers(20, 63)):
        kind = rng.choice(["offaxis", "sliver", "point", "line", "coplanar", "dup", "box",
                           "tiny", "huge_edge", "grain"])
        c = rng.uniform(-6, 6, 3).astype(np.float32) * g
        if kind == "offaxis":
            p = c + rng.normal(size=(3, 3)).astype(np.float32) * g
            add(p[0], p[1], p[2], int(rng.integers(0, 2)))
        elif kind == "sliver":              # v2 within a few ulps of the edge v0-v1
            p0 = c
            p1 = c + rng.normal(size=3).astype(np.float32) * 2 * g
            p2 = (p0 + (p1 - p0) * np.float32(rng.uniform(0.2, 0.8))).astype(np.float32)
            k = int(rng.integers(0, 3))
            p2[k] = np.nextafter(p2[k], np.float32(np.inf) * np.sign(rng.normal()))
            add(p0, p1, p2, 0)
        elif kind == "point":               # all three vertices equal
            add(c, c, c, 0)
        elif kind == "line":                # exactly collinear: v2 - v0 = 2 (v1 - v0) on the grid
            d = np.round(rng.normal(size=3) * 4).astype(np.float32) * g / np.float32(4)
            add(c, c + d, c + 2 * d, 0)
        elif kind == "coplanar":            # two overlapping triangles in one floor-parallel plane
            y = np.float32(-8 * g + g * np.float32(rng.integers(1, 4)))
            for _ in range(2):
                q = rng.uniform(-4, 4, (3, 2)).astype(np.float32) * g
                add(np.float32([q[0, 0], y, q[0, 1]]), np.float32([q[1, 0], y, q[1, 1]]),
                    np.float32([q[2, 0], y, q[2, 1]]), 0)
        elif kind == "dup" and tris:        # an exact duplicate: ties in t, the later face wins
            j = int(rng.integers(0, len(tris)))
            add(*tris[j], 1 - mats[j] if mats[j] < 2 else 0)
        elif kind == "box":                 # an axis-aligned box face pair, off-grid centre
            u = np.zeros(3, np.float32)
            v = np.zeros(3, np.float32)
            a, b = rng.choice(3, 2, replace=False)
            u[a] = np.float32(rng.uniform(0.5, 2)) * g
            v[b] = np.float32(rng.uniform(0.5, 2)) * g
            quad(c, u, v, 0)
        elif kind == "tiny":                # 2^-12 of the room: small denominators
            p = c + rng.normal(size=(3, 3)).astype(np.float32) * g * np.float32(2.0 ** -12)
            add(p[0], p[1], p[2], 0)
        elif kind == "huge_edge":           # edges up to 4 rooms long, off-axis
            p = c + rng.normal(size=(3, 3)).astype(np.float32) * g * np.float32(16)
            add(p[0], p[1], p[2], 1)
        else:                               # "grain": components with one or two set bits
            p = (np.float32(2.0) ** rng.integers(-6, 3, (3, 3)).astype(np.float32)) * g
            p *= rng.choice([-1, 1], (3, 3)).astype(np.float32)
            add(p[0], p[1], p[2], 0)
        kinds.append(str(kind))
    tris = tris[:64]
    mats = mats[:64]
    # every vertex within 30 rooms of the origin: |v0| <= 2^40 and |e| <= 2^41 at 2^38, the
    # specialisation's range (jit_scene_in_range), so every case takes the specialised scan
    lim = np.float32(30) * g
    tris = [(np.clip(p, -lim, lim) + off).astype(np.float32) for p in tris]

    V = rvcp_amd.scene.VERTEX_DTYPE
    F = rvcp_amd.scene.FACE_DTYPE
    verts = np.zeros(3 * len(tris), V)
    faces = np.zeros(len(tris), F)
    for i, p in enumerate(tris):
        verts["position"][3 * i:3 * i + 3, :3] = p
        verts["normal"][3 * i:3 * i + 3, :3] = _normal(*p)
        faces[i]["vertices"] = [3 * i, 3 * i + 1, 3 * i + 2]
        faces[i]["material_id"] = mats[i]
    M = rvcp_amd.scene.Material
    materials = [M.new_lambertian([0.73, 0.71, 0.68]), M.new_lambertian([0.63, 0.065, 0.05]),
                 M.new_light([17.0, 12.0, 4.0])]

    # the camera: inside the room (often inside the clutter) or outside the open front
    inside = rng.random() < 0.5
    pos = (rng.uniform(-6, 6, 3).astype(np.float32) * g if inside
           else np.float32([0, 0, -12]) * g + rng.uniform(-2, 2, 3).astype(np.float32) * g)
    look = rng.uniform(-4, 4, 3).astype(np.float32) * g
    if np.allclose(look, pos):
        look = pos + np.float32([0, 0, 1]) * g
    t_cap = 16777214.0                      # below 2^24 (rvcp_config_t.ray_t_max)
    pos, look = (pos + off).astype(np.float32), (look + off).astype(np.float32)
    # (the primary ray's t_far x t_coef stays below 2^24 too: t_coef < 1.7 at these fields of
    # view, rvcp_host.cpp primary_t_range_ok; 2^23 still reaches across a 2^22 room)
    cam = rvcp_amd.Camera.new(pos, look, float(np.float32(0.1) * g),
                              min(float(np.float32(1e5) * s), 2.0 ** 23),
                              float(rng.uniform(35, 80)), 1.0, 1.0)
    mesh = rvcp_amd.scene.ArrayMesh(verts, faces)
    sc = rvcp_amd.Scene(cam, materials, [], mesh)

    t_min = float(np.float32(rng.choice([1e-2, 1e-3, 0.3])) * g)
    kw = dict(spp=2, ray_t_min=t_min, ray_t_max=min(float(np.float32(1e4) * s), t_cap),
              eps=float(rng.choice([1e-3 * float(g), 1e-2 * float(g), 1e-3])),
              max_bounces=int(rng.choice([3, 15])), lum_id_std140_quirk=int(rng.random() < 0.7))
    desc = (f"seed {seed}: scale 2^{e}, offset 2^{e_off}, {len(tris)} faces, camera {'inside' if inside else 'outside'}"
            f", t_min {t_min:.3g}, eps {kw['eps']:.3g}, kinds {sorted(set(kinds))}")
    return sc, kw, desc


def positions(sc):
    """[F, 3, 3] vertex positions of a scene's faces (float32)."""
    v = sc.mesh.aligned_vertices()["position"][:, :3]
    return v[sc.mesh.aligned_faces()["vertices"]].astype(np.float32)
