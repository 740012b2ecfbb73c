"""The scene-specialised scan of rvcp_jit.cpp, checked on the CPU.

1. The generated source (librvcp's rvcp_internal_jit_scan_source) is compiled with g++ and a
   plain-C prelude (the reciprocal = the IEEE quotient, commits as no-ops) and run against the CPU
   oracle's ray-triangle test (oracle/rvcp_oracle.c is_intersect_with_face, with the nearest-
   hit rule of get_intersection_with_scene): the nearest (t, face) of every ray must be
   bit-identical.  Rays: random, axis-aligned, parallel to walls, aimed at shared edges and
   vertices; scenes: the Cornell box and random triangles whose components are mostly +0 / -0.
2. hipRTC compiles the generated module for gfx950 here (no GPU needed).

Tolerance: bit-exact (t bitwise equal, face index equal)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import rvcp_amd

HERE = os.path.dirname(os.path.abspath(__file__))
TRI_DTYPE = np.dtype([("v0", "<f4", 3), ("e1", "<f4", 3), ("e2", "<f4", 3), ("pad", "<f4", 3)])

PRELUDE = r"""
#include <cmath>
#include <cstdint>
#include <cstring>
#define __device__
#define __forceinline__ inline
struct f3 { float x, y, z; };
static inline float RVCP_F32(uint32_t b) { float f; std::memcpy(&f, &b, 4); return f; }
#define RVCP_SPEC_RCP(d) (1.0f / (d))
// RVCP_SPEC_RCP_FAST: the kernel's reciprocal without the class check, which equals the IEEE
// quotient for +-0 (rejected either way) and for |den| in [2^-126, 2^126] (tools/rcp_check2.hip);
// the generator emits it only where that holds for every ray passing dir_grain_ok -- counted
// here: a denominator outside that set while the current rays pass the guard is a violation
static long g_fast_calls = 0, g_fast_bad = 0;
static bool g_grain_ok = true;
static inline float rcp_fast_check(float d) {
    if (g_grain_ok) {
        g_fast_calls++;
        const float a = std::fabs(d);
        if (!(d == 0.0f || (a >= 0x1p-126f && a <= 0x1p126f))) g_fast_bad++;
    }
    return 1.0f / d;
}
#define RVCP_SPEC_RCP_FAST(d) rcp_fast_check(d)
static inline bool dir_grain_ok(f3 d) {       // the kernel's guard (rvcp_kernels.hip)
    const float c[3] = {d.x, d.y, d.z};
    for (float x : c)
        if (x != 0.0f && !(std::fabs(x) >= 0x1p-40f)) return false;
    return true;
}
#define RVCP_SPEC_COMMIT(t, i) ((void)0)
#define RVCP_SPEC_ANY(q) (q)          // one lane: the block runs iff this ray's mask holds
#define RVCP_SPEC_COMMIT1(t) ((void)0)
"""
DRIVER = r"""
extern "C" void scan_all(const float *rays, int n, float tmin, float tmax, float *bt_out,
                         int *best_out, int dual) {
    for (int r = 0; r < n; r++) {
        const float *q = rays + 6 * r;
        f3 o{q[0], q[1], q[2]}, d{q[3], q[4], q[5]};
        g_grain_ok = dir_grain_ok(d);
        float bt = tmax; int best = -1;
        if (dual) {
            // the two-ray form: the ray in slot B (nearest t and face), a different ray in
            // slot A; then the ray in slot A (its t and hit flag), the other ray in slot B
            f3 o2{q[0] + 1.0f, q[1], q[2]}, d2{q[4], q[5], q[3]};
            // (slot A keeps only its t: t_max after the scan is a miss or a hit at exactly
            // t_max, which the kernel settles with the generic scan)
            float bt2 = tmax;
            spec_scan2(o2, d2, o, d, tmin, bt2, bt, best);
            float btA = tmax, bt3 = tmax; int best3 = -1;
            spec_scan2(o, d, o2, d2, tmin, btA, bt3, best3);
            if (btA != bt || (btA != tmax && best < 0) || bt3 != bt2 || (bt2 != tmax && best3 < 0))
                best = -2;        // the slots disagree: reported as a mismatch
        } else {
            spec_scan1(o, d, tmin, bt, best);
        }
        bt_out[r] = bt; best_out[r] = best;
    }
}
extern "C" long fast_rcp_calls() { return g_fast_calls; }
extern "C" long fast_rcp_violations() { return g_fast_bad; }
"""


def _tri_records(positions):
    """TriRecords (v0, e1 = v1 - v0, e2 = v2 - v0 in float32) of [n, 3, 3] vertex positions."""
    p = np.asarray(positions, dtype=np.float32)
    rec = np.zeros(len(p), dtype=TRI_DTYPE)
    rec["v0"] = p[:, 0]
    rec["e1"] = (p[:, 1] - p[:, 0]).astype(np.float32)
    rec["e2"] = (p[:, 2] - p[:, 0]).astype(np.float32)
    return rec


def _scan_source(rec, opts=0):
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_jit_scan_source_opt
    fn.restype = ctypes.c_size_t
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    n = fn(rec.ctypes.data, len(rec), int(opts), None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    fn(rec.ctypes.data, len(rec), int(opts), buf, n + 1)
    return buf.value.decode()


def _build(tmp_path, rec, name, opts=0):
    src = tmp_path / f"{name}.cpp"
    src.write_text(PRELUDE + _scan_source(rec, opts) + DRIVER)
    so = tmp_path / f"{name}.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                    "-mfma", "-fno-fast-math", "-o", str(so), str(src)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.scan_all.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.fast_rcp_calls.restype = ctypes.c_long
    lib.fast_rcp_violations.restype = ctypes.c_long
    return lib


def _oracle_nearest(positions, ray, tmin, tmax):
    bt, best = np.float32(tmax), -1
    for i, tri in enumerate(positions):
        hit, out = O.intersect(list(ray) + [tmin, float(bt)], tri.reshape(9))
        if hit and out[0] <= bt:                       # :291 (NaN t is dropped here)
            bt, best = out[0], i
    return np.float32(bt), best


def _check(lib, positions, rays, tmin=0.01, tmax=10000.0):
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = len(rays)
    bt = np.zeros(n, np.float32)
    best = np.zeros(n, np.int32)
    lib.scan_all(rays.ctypes.data, n, tmin, tmax, bt.ctypes.data, best.ctypes.data, 0)
    hits = 0
    for r in range(n):
        obt, ob = _oracle_nearest(positions, rays[r], tmin, tmax)
        assert best[r] == ob and bt[r].view(np.uint32) == obt.view(np.uint32), \
            (r, rays[r].tolist(), (float(bt[r]), int(best[r])), (float(obt), ob))
        hits += ob >= 0
    # the two-ray entry point gives slot A the same answers
    bt2 = np.zeros(n, np.float32)
    best2 = np.zeros(n, np.int32)
    lib.scan_all(rays.ctypes.data, n, tmin, tmax, bt2.ctypes.data, best2.ctypes.data, 1)
    assert np.array_equal(best2, best) and np.array_equal(bt2.view(np.uint32), bt.view(np.uint32))
    assert lib.fast_rcp_violations() == 0
    return hits


def _norm(d):
    d = np.asarray(d, np.float32)
    return (d / np.sqrt((d.astype(np.float64) ** 2).sum(-1, keepdims=True))).astype(np.float32)


def _cornell_positions():
    sc = rvcp_amd.Scene.default()
    V = sc.mesh.aligned_vertices()
    return np.array([[V[j]["position"][:3] for j in f["vertices"]] for f in sc.mesh.aligned_faces()],
                    dtype=np.float32)


def _adversarial_rays(positions, rng, n):
    """Random rays inside the scene's box, axis-aligned rays, rays parallel to axis planes
    and rays aimed exactly at triangle vertices and at the midpoints of shared edges."""
    lo, hi = positions.reshape(-1, 3).min(0), positions.reshape(-1, 3).max(0)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = _norm(rng.normal(size=(n, 3)))
    k = n // 5
    axes = np.eye(3, dtype=np.float32)
    d[:k] = (axes[rng.integers(0, 3, k)] * rng.choice([-1, 1], (k, 1))).astype(np.float32)
    d[k:2 * k, 1] = 0.0                                  # parallel to the floor / ceiling
    d[k:2 * k] = _norm(d[k:2 * k] + 1e-30)
    d[k:2 * k, 1] = 0.0
    tgt = positions[rng.integers(0, len(positions), n - 2 * k), rng.integers(0, 3, n - 2 * k)]
    mid = (positions[:, 0] + positions[:, 2]) * np.float32(0.5)     # rectangle diagonals
    half = (n - 2 * k) // 2
    tgt[:half] = mid[rng.integers(0, len(mid), half)]
    d[2 * k:] = _norm(tgt - o[2 * k:])
    return np.concatenate([np.concatenate([o, d], axis=1), _exact_edge_rays(positions)])


def _exact_edge_rays(positions):
    """Axis-aligned rays at vertices and edge midpoints of the triangles from 50 units along
    each axis: on axis-aligned faces they land exactly on an edge or vertex, b1 or b2 = 0 or
    b1 + b2 = 1 exactly (the inclusive bounds of :259-260)."""
    pts = np.concatenate([positions.reshape(-1, 3),
                          ((positions + np.roll(positions, 1, axis=1)) * np.float32(0.5)).reshape(-1, 3)])
    rays = []
    for p in pts:
        for a in range(3):
            for sgn in (-1.0, 1.0):
                o = p.copy()
                o[a] += np.float32(50.0 * sgn)
                d = np.zeros(3, np.float32)
                d[a] = -sgn
                rays.append(np.concatenate([o, d]))
    return np.array(rays, dtype=np.float32)


def test_generated_scan_cornell_bitexact(tmp_path):
    pos = _cornell_positions()
    rec = _tri_records(pos)
    src = _scan_source(rec)
    # one commit per test (the single-ray scan's and slot B's with the face, slot A's t only),
    # except that the first test of a quad whose two triangles share t shares its partner's
    # commit (a deferred acceptance flag, "bool t<i><ray>_c;")
    import re
    deferred = re.findall(r"^    bool t\d+([AB]?)_c;$", src, re.M)
    dA = sum(1 for r in deferred if r == "A")
    assert 0 < dA and src.count("spec_scan1") == 1
    assert src.count("RVCP_SPEC_COMMIT(") + len(deferred) - dA == 2 * len(pos)
    assert src.count("RVCP_SPEC_COMMIT1(") + dA == len(pos)
    # zero components are dropped: 2544 arithmetic temporaries against 3552 for 32 triangles
    # with no zero component (-28 %)
    dense = _scan_source(_tri_records(np.random.default_rng(0).uniform(-5, 5, pos.shape)))
    assert src.count("const float ") < 0.75 * dense.count("const float ")
    # every reciprocal of the Cornell scans skips the class check
    assert "RVCP_SPEC_RCP(" not in src and src.count("RVCP_SPEC_RCP_FAST(") > 0
    lib = _build(tmp_path, rec, "cornell")
    hits = _check(lib, pos, _adversarial_rays(pos, np.random.default_rng(1), 2500))
    assert hits > 1500
    assert lib.fast_rcp_calls() > 0
    _check(lib, pos, _grain_edge_rays(pos, np.random.default_rng(7), 600))


def _grain_edge_rays(positions, rng, n):
    """Rays whose direction components sit at dir_grain_ok's bound: 0, +-2^-40 and a few ulps
    above it, the rest random (the smallest denominators the fast reciprocal may meet)."""
    lo, hi = positions.reshape(-1, 3).min(0), positions.reshape(-1, 3).max(0)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = _norm(rng.normal(size=(n, 3)))
    tiny = np.float32(2.0 ** -40) * (1 + rng.integers(0, 4, (n, 3)) * np.float32(2.0 ** -23))
    pick = rng.random((n, 3)) < 0.4
    d = np.where(pick, tiny * rng.choice([-1, 1], (n, 3)), d).astype(np.float32)
    d[rng.random((n, 3)) < 0.2] = 0.0
    d[(d == 0).all(1), 0] = 1.0
    return np.concatenate([o, d], axis=1)


def test_fast_reciprocal_grain_rule(tmp_path):
    """The generator emits the class-check-free reciprocal only where its grain bound proves the
    denominator zero or normal for every ray dir_grain_ok admits: triangles at unit scale get it,
    triangles at 2^-10 scale (denominators down to 2^-129) do not; the premise holds on rays at
    the guard's bound and the scan stays bit-exact vs the oracle."""
    rng = np.random.default_rng(11)
    unit = rng.uniform(-5, 5, (6, 3, 3)).astype(np.float32)
    unit[:, :, 1] = np.float32(1.25)                   # horizontal: a zero denominator term
    small = (rng.uniform(-5, 5, (6, 3, 3)) * 2.0 ** -10).astype(np.float32)
    pos = np.concatenate([unit, small])
    src = _scan_source(_tri_records(pos))
    assert src.count("RVCP_SPEC_RCP_FAST(") > 0 and src.count("RVCP_SPEC_RCP(") > 0
    lib = _build(tmp_path, _tri_records(pos), "grain")
    _check(lib, pos, _grain_edge_rays(pos, rng, 800))
    _check(lib, pos, _adversarial_rays(pos, rng, 400))
    assert lib.fast_rcp_calls() > 0


def test_generated_scan_sparse_random_bitexact(tmp_path):
    """Triangles whose components are mostly signed zeros (every drop rule of the generator,
    including identically-zero denominators and vanished b1/b2/t terms), small and huge."""
    rng = np.random.default_rng(2)
    n = 40
    pos = rng.uniform(-50, 50, (n, 3, 3)).astype(np.float32)
    mask = rng.random((n, 3, 3)) < 0.55
    pos[mask] = np.where(rng.random(mask.sum()) < 0.5, np.float32(0.0), np.float32(-0.0))
    pos[:4] *= np.float32(1e-30)
    pos[4:8] *= np.float32(1e30)
    rec = _tri_records(pos)
    lib = _build(tmp_path, rec, "sparse")
    rays = _adversarial_rays(pos[8:], rng, 1500)
    rays[:100, :3] = 0.0                       # origins at the (zero) vertices
    _check(lib, pos, rays)
    _check(lib, pos, rays, tmin=1e-3, tmax=1e30)


def test_hiprtc_compiles_specialised_module():
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_jit_compile_check
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t),
                   ctypes.c_char_p, ctypes.c_size_t]
    rec = _tri_records(_cornell_positions())
    size = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(4096)
    rc = fn(rec.ctypes.data, len(rec), ctypes.byref(size), err, 4096)
    if rc != 0 and b"libhiprtc not found" in err.value:
        pytest.skip("hipRTC not installed")
    assert rc == 0, err.value.decode()
    assert size.value > 10000


def test_code_object_disk_cache(tmp_path):
    """the specialised module's code object goes through the on-disk cache
    (rvcp_set_code_cache_dir): compiled and stored once, then read back (a second process does
    the same: tests/test_gpu_specialize.py); a damaged, truncated or foreign entry is rejected
    and recompiled, never used."""
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_jit_cached_code
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                   ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
    rec = _tri_records(_cornell_positions())
    cache = tmp_path / "cache" / "nested"
    rvcp_amd.abi.set_code_cache_dir(str(cache))

    def get():
        disk, size = ctypes.c_int(-1), ctypes.c_size_t(0)
        err = ctypes.create_string_buffer(4096)
        rc = fn(rec.ctypes.data, len(rec), 0, ctypes.byref(disk), ctypes.byref(size), err, 4096)
        if rc != 0 and b"libhiprtc not found" in err.value:
            pytest.skip("hipRTC not installed")
        assert rc == 0, err.value.decode()
        return disk.value, size.value
    try:
        c0 = rvcp_amd.abi.code_cache_counts()
        disk, size = get()
        assert disk == 0 and size > 10000                         # compiled, stored
        files = list(cache.glob("*.rvcpco"))
        assert len(files) == 1 and not list(cache.glob("*.tmp.*"))
        assert get() == (1, size)                                 # read back
        blob = files[0].read_bytes()
        # a file cut inside its key whose code length is the wrapped difference, so that
        # header + key + code "adds up" to the file size modulo 2^64 (must be rejected before
        # the key is compared: the comparison would read past the end of the file's bytes)
        key_len = int.from_bytes(blob[8:16], "little")
        cut = 40 + key_len // 2
        wrapped = (cut - 40 - key_len) % (1 << 64)
        cut_key = blob[:16] + wrapped.to_bytes(8, "little") + blob[24:cut]
        for bad in (blob[:-1] + bytes([blob[-1] ^ 1]),            # code bit flipped
                    blob[: len(blob) // 2],                       # truncated
                    b"RVCPCO01" + blob[8:40] + b"X" + blob[41:],  # key text altered
                    cut_key,                                      # length wraps past 2^64
                    b"garbage"):
            files[0].write_bytes(bad)
            assert get() == (0, size)                             # rejected -> recompiled
            assert files[0].read_bytes() == blob                  # ... and rewritten
            assert get() == (1, size)
        c1 = rvcp_amd.abi.code_cache_counts()
        assert c1["rejects"] - c0["rejects"] == 5
        assert c1["loads"] - c0["loads"] == 6 and c1["compiles"] - c0["compiles"] == 6
        rvcp_amd.abi.set_code_cache_dir("")                       # off: compiles, stores nothing
        files[0].unlink()
        assert get() == (0, size) and not list(cache.glob("*.rvcpco"))
        # a cache path that cannot be a directory (a regular file on the way): the module is
        # still compiled, nothing is written, nothing fails
        blocker = tmp_path / "not_a_dir"
        blocker.write_text("x")
        rvcp_amd.abi.set_code_cache_dir(str(blocker / "cache"))
        assert get() == (0, size)
        assert blocker.read_text() == "x"
    finally:
        rvcp_amd.abi.set_code_cache_dir("")


def test_hiprtc_compiles_specialised_mode2_module():
    """The mode-2 (ray_tracer.comp) kernel with the specialised triangle scan, compiled for the
    sphere room's 12 faces (RVCP_JIT_LEGACY)."""
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_jit_compile_check_mode
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t),
                   ctypes.c_char_p, ctypes.c_size_t]
    sc = rvcp_amd.scene.sphere_scene()
    verts = sc.mesh.aligned_vertices()["position"][:, :3]
    faces = sc.mesh.aligned_faces()["vertices"]
    rec = _tri_records(verts[faces].astype(np.float32))
    size = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(4096)
    rc = fn(rec.ctypes.data, len(rec), 1, ctypes.byref(size), err, 4096)
    if rc != 0 and b"libhiprtc not found" in err.value:
        pytest.skip("hipRTC not installed")
    assert rc == 0, err.value.decode()
    assert size.value > 10000


def test_mode2_sphere_literals():
    """Mode 2's spheres as literals (rvcp_jit.cpp jit_sphere_source): the X-macro carries every
    sphere's center and radius bit for bit, in index order; the mode-2 module compiles with it
    (the kernel's unrolled sphere tests, rvcp_kernels.hip legacy_spheres); none for a scene
    without spheres or with more than 64 (the kernel keeps its loop over the records)."""
    import re
    L = rvcp_amd.abi.load()
    src = L.rvcp_internal_jit_sphere_source
    src.restype = ctypes.c_size_t
    src.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]

    def text(sph):
        n = src(sph.ctypes.data if len(sph) else None, len(sph), None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        src(sph.ctypes.data if len(sph) else None, len(sph), buf, n + 1)
        return buf.value.decode()
    sc = rvcp_amd.scene.sphere_scene()
    sph = np.ascontiguousarray(sc.aligned_spheres())
    rng = np.random.default_rng(5)
    odd = sph.copy()                     # signed zeros, subnormals, huge and negative values
    odd["center"][:, 0] = np.array([-0.0, 1e-40, -3e38, 7.25, 0.0, -1.5, 2.0 ** -126, 1e30][:len(odd)], np.float32)
    odd["radius"] = rng.standard_normal(len(odd)).astype(np.float32)
    for recs in (sph, odd):
        t = text(recs)
        rows = re.findall(r"X\((\d+), ([^X]*)\)", t)
        assert [int(i) for i, _ in rows] == list(range(len(recs)))
        for (_, args), rec in zip(rows, recs):
            bits = [int(b, 16) for b in re.findall(r"RVCP_F32\(0x([0-9a-f]{8})u\)", args)]
            want = np.concatenate([rec["center"], [rec["radius"]]]).astype(np.float32).view(np.uint32)
            assert bits == want.tolist()
    assert text(sph[:0]) == ""
    big = np.zeros(65, dtype=sph.dtype)
    assert text(big) == "" and text(big[:64]).count("X(") == 64
    fn = L.rvcp_internal_jit_compile_check_spheres
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                   ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
    verts = sc.mesh.aligned_vertices()["position"][:, :3]
    faces = sc.mesh.aligned_faces()["vertices"]
    rec = _tri_records(verts[faces].astype(np.float32))
    size = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(4096)
    rc = fn(rec.ctypes.data, len(rec), sph.ctypes.data, len(sph), ctypes.byref(size), err, 4096)
    if rc != 0 and b"libhiprtc not found" in err.value:
        pytest.skip("hipRTC not installed")
    assert rc == 0, err.value.decode()
    assert size.value > 10000


def _in_range(rec):
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_jit_scene_in_range
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    return bool(fn(rec.ctypes.data, len(rec)))


def _huge_box(scale):
    """An axis-aligned box of side 2*scale around the origin (12 triangles, a third of their
    edge components exact zeros), the camera inside it."""
    s = np.float32(scale)
    c = np.array([[x, y, z] for x in (-s, s) for y in (-s, s) for z in (-s, s)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris = []
    for a, b, cc, d in quads:
        tris += [[c[a], c[b], c[cc]], [c[a], c[cc], c[d]]]
    return np.array(tris, np.float32)


def test_specialisation_range_guard(tmp_path):
    """The zero-dropping premise: no intermediate of the generic test may
    overflow, else the generic inf * 0 = NaN rejects where the dropped term does not.  Upload
    specialises only scenes with |v0| <= 2^40 and |e1|, |e2| <= 2^41 (jit_scene_in_range); the
    Cornell box is in range, a 1e20-scale box is routed to the generic kernels.  Inside the
    range the generated scan stays bit-exact vs the oracle on that box scaled to 2^39."""
    assert _in_range(_tri_records(_cornell_positions()))
    big = _huge_box(1e20)
    assert not _in_range(_tri_records(big))
    assert not _in_range(_tri_records(_huge_box(2.0 ** 40.5)))
    edge = _huge_box(2.0 ** 39)
    assert _in_range(_tri_records(edge))
    rng = np.random.default_rng(5)
    rays = _adversarial_rays(edge, rng, 600)
    lib = _build(tmp_path, _tri_records(edge), "edge")
    _check(lib, edge, rays, tmin=0.01, tmax=1e30)
    # outside the range the premise fails: from a point inside the 1e20 box the generic
    # test's s2 = s x e1 overflows to inf (and inf * 0 = NaN would meet a dropped zero term)
    T = _tri_records(big)[0]
    o = np.float32([1.0, 2.0, -1e20 + 1e14])
    sv = (o - T["v0"]).astype(np.float32)
    with np.errstate(over="ignore", invalid="ignore"):
        s2 = np.cross(sv, T["e1"]).astype(np.float32)
    assert not np.isfinite(s2).all()


DEN_SRC = r"""
#include <cmath>
// the generic test's denominator, dot(cross(d, e2), e1) with the fused builtins of DESIGN.md §3.1
extern "C" long den_violations(const float *tri, int n, const float *dirs, int m) {
    long bad = 0;
    for (int i = 0; i < n; i++) {
        const float *e1 = tri + 12 * i + 3, *e2 = tri + 12 * i + 6;
        for (int j = 0; j < m; j++) {
            const float *d = dirs + 3 * j;
            const float s1x = std::fma(d[1], e2[2], -(d[2] * e2[1]));
            const float s1y = std::fma(d[2], e2[0], -(d[0] * e2[2]));
            const float s1z = std::fma(d[0], e2[1], -(d[1] * e2[0]));
            const float den = std::fma(s1z, e1[2], std::fma(s1y, e1[1], s1x * e1[0]));
            const float a = std::fabs(den);
            if (!(den == 0.0f || (a >= 0x1p-126f && a <= 0x1p126f))) bad++;
        }
    }
    return bad;
}
"""


def _rcp_fast_scene(rec):
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_scan_rcp_fast_scene
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    return bool(fn(rec.ctypes.data, len(rec)))


def test_generic_scan_fast_reciprocal_scene_rule(tmp_path):
    """FrameArgs::rcp_fast (scan_rcp_fast_scene): the generic scans drop the reciprocal's class
    check only for scenes whose every denominator is +-0 or within [2^-126, 2^126] for all
    directions passing dir_fast_ok.  The Cornell box, its rotated copy and unit-scale random
    meshes pass; 2^-40-scale and 1e30-scale triangles and non-finite edges do not; on the scenes
    that pass, the denominators of directions at the guard's bound stay in range (C, the fused
    builtins)."""
    src = tmp_path / "den.cpp"
    src.write_text(DEN_SRC)
    so = tmp_path / "den.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-mfma",
                    "-fno-fast-math", "-o", str(so), str(src)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.den_violations.restype = ctypes.c_long
    lib.den_violations.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    rng = np.random.default_rng(12)
    cornell = _cornell_positions()
    scenes_ok = [cornell, rng.uniform(-5, 5, (40, 3, 3)).astype(np.float32)]
    rot = np.float32(np.linalg.qr(rng.normal(size=(3, 3)))[0])
    scenes_ok.append((cornell @ rot).astype(np.float32))
    for pos in scenes_ok:
        rec = _tri_records(pos)
        assert _rcp_fast_scene(rec)
        d = _grain_edge_rays(pos, rng, 4000)[:, 3:].copy()
        d = np.concatenate([d, _norm(rng.normal(size=(2000, 3)))]).astype(np.float32)
        assert lib.den_violations(rec.ctypes.data, len(rec), d.ctypes.data, len(d)) == 0
    assert not _rcp_fast_scene(_tri_records(cornell * np.float32(2.0 ** -40)))
    assert not _rcp_fast_scene(_tri_records(cornell * np.float32(1e30)))
    bad = cornell.copy()
    bad[3, 1, 0] = np.inf
    assert not _rcp_fast_scene(_tri_records(bad))


def _rcp_fast_scene_ref(rec):
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_scan_rcp_fast_scene_ref
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    return bool(fn(rec.ctypes.data, len(rec)))


def test_rcp_fast_scene_rule_numeric_equals_generator():
    """the scene rule now tracks grain and magnitude as integers instead of building
    every triangle's expression strings.  It must decide exactly as the generator-based form
    (the same zero-dropping rules) on scenes at every scale and mix of exact-zero components,
    and a C5-size mesh (100 032 triangles) must cost milliseconds, not the 0.3 s of upload the
    string form took."""
    import time
    rng = np.random.default_rng(2024)
    cornell = _cornell_positions()
    cases = [cornell, (cornell * np.float32(2.0 ** -40)).astype(np.float32),
             (cornell * np.float32(1e30)).astype(np.float32)]
    for scale in [2.0 ** -60, 2.0 ** -30, 2.0 ** -10, 1.0, 2.0 ** 20, 2.0 ** 40, 2.0 ** 60]:
        for zeros in (0.0, 0.3, 0.7):
            p = rng.uniform(-1, 1, (30, 3, 3)) * scale
            p[rng.random(p.shape) < zeros] = 0.0       # exact zeros, as on axis-aligned walls
            # snap some components onto coarse grains (small lowest set bits)
            k = rng.random(p.shape) < 0.3
            p[k] = np.round(p[k] / scale * 8) * scale / 8
            cases.append(p.astype(np.float32))
    decided = set()
    for pos in cases:
        rec = _tri_records(pos)
        a, b = _rcp_fast_scene(rec), _rcp_fast_scene_ref(rec)
        assert a == b, pos.max()
        decided.add(a)
    assert decided == {True, False}
    import rvcp_amd as R
    big = R.scene.with_random_triangles(R.Scene.default(), 100000)
    v = big.mesh.aligned_vertices()["position"][:, :3]
    pos = v[big.mesh.aligned_faces()["vertices"]].astype(np.float32)
    rec = _tri_records(pos)
    t0 = time.perf_counter()
    ok = _rcp_fast_scene(rec)
    dt = time.perf_counter() - t0
    assert ok == _rcp_fast_scene_ref(rec) and ok
    assert dt < 0.05, dt


@pytest.mark.parametrize("seed", range(0, 36, 3))
def test_generated_scan_fuzz_scenes_bitexact(tmp_path, seed):
    """The seeded adversarial scenes of tests/fuzz_scenes.py (scales 2^-20 .. 2^38, slivers,
    degenerate / coplanar / duplicated triangles, mixed axis-aligned and off-axis faces; the GPU
    renders all 36 in test_gpu_spec_fuzz.py): the generated scan compiled with g++ equals the
    oracle's nearest hit bit for bit on adversarial and guard-bound rays at the scene's own
    t_min / t_max, and no fast reciprocal meets a denominator outside {+-0} U [2^-126, 2^126]."""
    from fuzz_scenes import fuzz_scene, positions
    sc, kw, desc = fuzz_scene(seed)
    pos = positions(sc)
    rec = _tri_records(pos)
    lib = _build(tmp_path, rec, f"fuzz{seed}")
    rng = np.random.default_rng(seed)
    rays = np.concatenate([_adversarial_rays(pos, rng, 300), _grain_edge_rays(pos, rng, 150)])
    _check(lib, pos, rays, tmin=kw["ray_t_min"], tmax=kw["ray_t_max"])
    assert lib.fast_rcp_violations() == 0, desc


def test_generated_scan_skippable_runs_bitexact(tmp_path):
    """The dual scan's skippable runs (round 5): slot A always, slot B with the experiment knob
    (RVCP_DEBUG_SPEC_SKIP_B).  Every run is split at its first test's range mask; on one lane the
    block runs iff that lane's mask holds, so this checks that the split keeps every value and
    every acceptance: Cornell and two fuzz scenes, adversarial rays, both slots against the oracle."""
    from fuzz_scenes import fuzz_scene, positions
    import re
    cases = [("cornell", _cornell_positions())] + [(f"fuzz{k}", positions(fuzz_scene(k)[0])) for k in (2, 13)]
    for name, pos in cases:
        rec = _tri_records(pos)
        head_ops = {}
        for opts in (0, 1, 2):              # default; + slot B split; eager shadow split (r05h)
            skip_b = bool(opts & 1)
            src = _scan_source(rec, opts)
            runs_a = len(re.findall(r"RVCP_SPEC_ANY\(t\d+A_q\)", src))
            runs_b = len(re.findall(r"RVCP_SPEC_ANY\(t\d+B_q\)", src))
            assert runs_a > 0 and (runs_b > 0) == skip_b, (name, opts, runs_a, runs_b)
            head_ops[opts] = _unskippable_ops(src)
            lib = _build(tmp_path, rec, f"{name}_{opts}", opts)
            _check(lib, pos, _adversarial_rays(pos, np.random.default_rng(5), 300))
        # the default computes s1 / s2 components only n1 and n2 read inside the skippable block
        assert head_ops[0] < head_ops[2], (name, head_ops)


def _unskippable_ops(src):
    """Arithmetic statements of the dual scan outside its skippable blocks."""
    body = src[src.index("spec_scan2"):]
    n, inside = 0, False
    for line in body.splitlines():
        if "RVCP_SPEC_ANY(" in line:
            inside = True
        elif line.startswith("    RVCP_SPEC_COMMIT"):
            inside = False
        elif line.strip().startswith("const float") and not inside:
            n += 1
    return n
