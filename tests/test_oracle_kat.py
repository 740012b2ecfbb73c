"""Known-answer tests of the CPU oracle's building blocks (no GPU).

The reference has no tests or golden vectors; these KATs pin the oracle's
restatement of each shader function against hand-computed answers, float64 mathematics and
the independent pure-Python restatement in tests/pyref.py."""
import math

import numpy as np
import pytest

import oracle as O
import pyref
import rvcp_amd

F = np.float32


def bits(x):
    return int(np.float32(x).view(np.uint32))


def test_sin_accuracy_vs_float64():
    xs = np.concatenate([np.linspace(-20.0, 2100.0, 40001, dtype=np.float32),
                         np.random.default_rng(1).uniform(0, 1500, 20000).astype(np.float32)])
    ours = np.array([O.sinf(float(x)) for x in xs], dtype=np.float64)
    ref = np.sin(xs.astype(np.float64))
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    err_ulp = np.abs(ours - ref) / np.maximum(ulp, 2.0 ** -149)
    assert err_ulp.max() <= 2.0, err_ulp.max()
    assert np.abs(ours - ref).max() < 2.4e-7


def test_sin_bitexact_vs_pyref():
    rng = np.random.default_rng(2)
    xs = np.concatenate([rng.uniform(0, 1, 100), rng.uniform(0, 2000, 200), [0.0, -0.0, 1.0,
                         math.pi / 2, 123.0, 999.0, 1e4, 3.0e5]]).astype(np.float32)
    for x in xs:
        assert bits(O.sinf(float(x))) == bits(pyref.sinf(x)), x


def test_pyref_fma_single_rounding():
    """pyref's float64+TwoSum fma equals the rational-arithmetic fma, including inputs whose
    float64 sum lands exactly on a float32 rounding midpoint."""
    rng = np.random.default_rng(9)
    cases = [tuple(F(x) for x in rng.uniform(-1e3, 1e3, 3)) for _ in range(3000)]
    cases += [tuple(F(x) for x in rng.standard_normal(3) * 10.0 ** rng.integers(-20, 20, 3))
              for _ in range(3000)]
    # midpoint traps: a*b = 1 + 2^-24 + 2^-35 exactly; with c = -2^-35 +/- 2^-58 the exact sum is
    # 1 + 2^-24 +/- 2^-58, whose float64 rounding is the float32 midpoint 1 + 2^-24
    a, b = F(1.0 + 2.0 ** -12), F(1.0 - 2.0 ** -12 + 2.0 ** -23)
    traps = [(a, b, F(-2.0 ** -35 + 2.0 ** -58)), (a, b, F(-2.0 ** -35 - 2.0 ** -58)),
             (F(-a), b, F(2.0 ** -35 - 2.0 ** -58)), (a, b, F(-2.0 ** -35))]
    assert float(pyref.fma(*traps[0])) == 1.0 + 2.0 ** -23
    assert float(pyref.fma(*traps[1])) == 1.0
    cases += traps
    for a, b, c in cases:
        assert bits(pyref.fma(a, b, c)) == bits(pyref.fma_exact(a, b, c)), (a, b, c)
    assert np.isnan(pyref.fma(F(np.inf), F(0.0), F(1.0)))
    assert pyref.fma(F(np.inf), F(2.0), F(1.0)) == np.inf


def test_sin_special_values():
    assert math.isnan(O.sinf(float("inf"))) and math.isnan(O.sinf(float("nan")))
    assert O.sinf(0.0) == 0.0


@pytest.mark.parametrize("time,u,v", [(123.0, 0.5, 0.5), (0.0, 0.00048828125, 0.99951171875),
                                      (999.0, 0.123, 0.877), (421.25, 0.3, 0.6)])
def test_rand_sequence_vs_pyref(time, u, v):
    seq = O.rand_sequence(time, u, v, 60)
    g = pyref.Rng(F(time), F(u), F(v))
    assert bits(seq[0]) == bits(g.seed)
    for i in range(60):
        assert bits(seq[1 + i]) == bits(g()), i
    assert np.all((seq >= 0) & (seq < 1))


def test_rand_is_uniform():
    seq = O.rand_sequence(123.0, 0.25, 0.75, 20000)[1:]
    hist, _ = np.histogram(seq, bins=20, range=(0, 1))
    assert hist.min() > 800 and hist.max() < 1200          # expected 1000 per bin


def _driver_u8(g):
    """The reference driver's UNORM8 rule on the stored value g."""
    return (math.floor(min(max(g, 0.0), 1.0) * 4096.0) * 255 + 2048) // 4096


@pytest.mark.parametrize("rule", [0, 1], ids=["driver", "nearest"])
def test_gamma_table_and_u8(rule):
    T = [O.gamma_threshold(k, rule) for k in range(256)]
    assert T[0] == 0.0 and all(T[k] < T[k + 1] for k in range(255))
    assert O.gamma_u8(0.0, rule) == 0 and O.gamma_u8(1.0, rule) == 255
    assert O.gamma_u8(7.0, rule) == 255
    assert O.gamma_u8(-1.0, rule) == 0 and O.gamma_u8(float("nan"), rule) == 0
    assert O.gamma_u8(0.1, rule) == 64    # the miss colour: 255 * 0.1^0.6 = 64.05
    rng = np.random.default_rng(3)
    for c in rng.uniform(0, 1, 2000).astype(np.float32):
        g = float(c) ** 0.6
        if rule == 1:
            exact = 255.0 * g
            if abs(exact - math.floor(exact) - 0.5) < 1e-3:
                continue                   # too close to a rounding tie to call
            assert O.gamma_u8(float(c), rule) == int(math.floor(exact + 0.5)), c
        else:
            if abs(g * 4096.0 - round(g * 4096.0)) < 1e-3:
                continue                   # too close to a truncation step to call
            assert O.gamma_u8(float(c), rule) == _driver_u8(g), c


TRI = [0, 0, 0, 1, 0, 0, 0, 1, 0]


@pytest.mark.parametrize("ray,hit,expect", [
    ([0.25, 0.25, -1, 0, 0, 1, 0.01, 100], True, (1.0, 0.25, 0.25)),     # interior, front
    ([0.25, 0.25, 1, 0, 0, -1, 0.01, 100], True, (1.0, 0.25, 0.25)),     # double-sided
    ([0.6, 0.6, -1, 0, 0, 1, 0.01, 100], False, None),                   # b1 + b2 > 1
    ([-0.1, 0.2, -1, 0, 0, 1, 0.01, 100], False, None),                  # b1 < 0
    ([0.2, -0.1, -1, 0, 0, 1, 0.01, 100], False, None),                  # b2 < 0
    ([0.0, 0.0, -1, 0, 0, 1, 0.01, 100], True, (1.0, 0.0, 0.0)),         # vertex (inclusive)
    ([0.5, 0.5, -1, 0, 0, 1, 0.01, 100], True, (1.0, 0.5, 0.5)),         # hypotenuse (inclusive)
    ([0.25, 0.25, -1, 0, 0, 1, 0.01, 0.5], False, None),                 # t > t_max
    ([0.25, 0.25, -1, 0, 0, 1, 1.5, 100], False, None),                  # t < t_min
    ([0.25, 0.25, -1, 1, 0, 0, 0.01, 100], False, None),                 # parallel: f = inf
])
def test_intersect_kat(ray, hit, expect):
    h, out = O.intersect(ray, TRI)
    assert h == hit
    if hit:
        assert tuple(float(x) for x in out) == expect


def test_intersect_in_plane_nan_semantics():
    """In-plane ray: dot(s1, e1) = 0 -> f = inf, t = b1 = b2 = inf * 0 = NaN.  Every rejection
    test of :259-260 compares false on NaN, so is_intersect_with_face returns TRUE with t = NaN;
    only get_intersection_with_scene's `new_inter.time <= ray.t_max` (:291) drops it."""
    h, out = O.intersect([0.25, 0.25, 0, 1, 0, 0, 0.01, 100], TRI)
    assert h and all(math.isnan(float(x)) for x in out)


def test_intersect_vs_pyref_random():
    rng = np.random.default_rng(4)
    sc = pyref.Scene([{"albedo": [1, 1, 1], "ty": 0}],
                     [{"position": [0, 0, 0, 0], "normal": [0, 1, 0, 0]}] * 3,
                     [{"vertices": [0, 1, 2], "material_id": 0}], [])
    n_hits = 0
    for _ in range(400):
        tri = rng.uniform(-5, 5, 9).astype(np.float32)
        o = rng.uniform(-8, 8, 3).astype(np.float32)
        w = rng.uniform(-0.2, 1.0, 2)                   # aim near / inside the triangle
        target = tri[0:3] + w[0] * (tri[3:6] - tri[0:3]) + w[1] * (tri[6:9] - tri[0:3])
        d = (target - o).astype(np.float32)
        d = (d / np.float32(np.sqrt(np.float32(d @ d)))).astype(np.float32)
        sc.pos = [tuple(F(x) for x in tri[3 * k:3 * k + 3]) for k in range(3)]
        ray = np.concatenate([o, d, [0.01, 1e4]]).astype(np.float32)
        h, out = O.intersect(ray, tri)
        p = pyref.intersect(sc, tuple(F(x) for x in o), tuple(F(x) for x in d), F(0.01), F(1e4),
                            sc.faces[0])
        assert h == (p is not None)
        if h:
            n_hits += 1
            assert bits(out[0]) == bits(p[0])
    assert 100 < n_hits < 390


def test_sample_ray_default_camera():
    sc = rvcp_amd.Scene.default()
    push = sc.push_constant(123.0)
    r = O.sample_ray(push, 1025, 1025, 512, 512)          # exact centre pixel (odd size)
    assert r[3] == 0.0 and r[4] == 0.0 and abs(r[5] - 1.0) < 1e-6
    assert tuple(r[:3]) == (0.0, 274.0, -1050.0)
    assert r[6] == np.float32(0.1) and r[7] == np.float32(10000.0)    # t_coef == 1
    # corners: 40 degree vertical fov
    r = O.sample_ray(push, 1024, 1024, 0, 0)
    half = math.degrees(math.atan2(math.hypot(r[3], r[4]) / math.sqrt(2), r[5]))
    assert abs(half - 20.0 * 1023 / 1024) < 0.05
    # pixel (0, 0) is the top-left; u = fwd x up = -x, so image-left is +x (which is why the
    # green x = -275 wall appears on the right of the README screenshot); v = fwd x u = -y
    assert r[3] > 0 and r[4] > 0


def test_o3_timing_copy_same_bits():
    """bench.py's cpu_baseline times the -O3 build of the oracle; it renders
    the same bits as the -O2 checker (the Cornell box and the off-axis rotated box)."""
    from rvcp_amd import scene as S
    for sc in (rvcp_amd.Scene.default(), S.rotated_scene(rvcp_amd.Scene.default())):
        arrays = dict(materials=sc.aligned_materials(), vertices=sc.mesh.aligned_vertices(),
                      faces=sc.mesh.aligned_faces(), lum_face_ids=sc.luminous_face_ids())
        cfg = rvcp_amd.abi.make_config(spp=3)
        a = O.render(arrays, sc.push_constant(123.0), cfg, 48, 40)
        b = O.render(arrays, sc.push_constant(123.0), cfg, 48, 40, o3=True)
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
        assert np.array_equal(a[1], b[1]) and a[2] == b[2]
