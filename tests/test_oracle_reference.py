"""Pinning the CPU oracle (no GPU).

1. Against the reference's only rendered output: the README screenshot (1024^2, SPP=30,
   rendered by ray_tracer_games101_branch.comp on an RTX 3060).  Its driver sin() differs
   from ours, so only statistics can match: 32x32-pixel block means of the 8-bit image
   (fixture tests/golden/readme_blockmeans.npz, made by tests/golden/make_readme_fixture.py),
   and the per-pixel L2 tolerance of north_star (fixture tests/golden/readme_pixels.npz):
   the per-pixel linear-RGB L2 distance between the oracle and the screenshot must equal the
   oracle's own seed-to-seed L2 at the same SPP within 2 % -- i.e. the reference differs from
   us per pixel exactly as much as a second frame of ours with another time seed does.
2. Against tests/pyref.py, an independent pure-Python restatement, bit for bit, per pixel.
"""
import math
import os

import numpy as np
import pytest

import oracle as O
import pyref
import rvcp_amd
from conftest import block_means, readme_blocks, scene_arrays

TIME = 123.0


def _rms_vs_readme(rgba):
    b32, _ = readme_blocks()
    ours = block_means(rgba, 32)
    ok = np.isfinite(b32)
    return float(np.sqrt(np.mean((ours[ok] - b32[ok]) ** 2))), (ours[ok] - b32[ok]).reshape(-1, 3).mean(0)


@pytest.fixture(scope="module")
def oracle_256(cornell_arrays, cornell):
    out = {}
    for quirk in (1, 0):
        cfg = rvcp_amd.abi.make_config(spp=30, lum_id_std140_quirk=quirk)
        out[quirk] = O.render(cornell_arrays, cornell.push_constant(TIME), cfg, 256, 256)
    return out


def test_readme_blocks_quirk_on(oracle_256):
    rms, mean = _rms_vs_readme(oracle_256[1][1])
    assert rms < 0.012, rms                  # measured 0.0084 (resolution-limited at 256^2)
    assert np.all(np.abs(mean) < 0.004), mean


def test_readme_blocks_discriminate_quirk(oracle_256):
    """The std140 luminous-id quirk is visible in the reference's output:
    emulating the intended packed ids lands ~3x further from the screenshot."""
    on, _ = _rms_vs_readme(oracle_256[1][1])
    off, _ = _rms_vs_readme(oracle_256[0][1])
    assert off > 0.02 and off > 2.5 * on, (on, off)


@pytest.fixture(scope="module")
def c3_frame(cornell_arrays, cornell):
    cfg = rvcp_amd.abi.make_config(spp=30)
    _, rgba, trav = O.render(cornell_arrays, cornell.push_constant(TIME), cfg, 1024, 1024,
                             want_linear=False)
    return rgba, trav


def test_readme_blocks_full_resolution(c3_frame):
    rgba, trav = c3_frame
    rms, mean = _rms_vs_readme(rgba)
    assert rms < 0.006, rms                  # measured 0.0033 (quirk off: 0.027)
    # miss pixels outside the open box are exactly 64 in the screenshot and here
    assert (rgba[0, 0, :3] == 64).all() and (rgba[1023, 1023, :3] == 64).all()
    assert 4.85 < trav / (1024 * 1024 * 30) < 5.0


L2_ROWS = list(range(0, 1023, 4))        # every 4th visible row: 256 x 1022 pixels


def _rows(arrays, sc, time, **kw):
    cfg = rvcp_amd.abi.make_config(spp=30, **kw)
    return np.concatenate([O.render(arrays, sc.push_constant(time), cfg, 1024, 1024,
                                    rect=(0, y, 1024, 1), want_linear=False)[1]
                           for y in L2_ROWS])


def _l2(a, b, vis):
    """Per-pixel L2 distance of linear RGB decoded from 8 bits (inverse of the 0.6 gamma),
    RMS over the visible pixels."""
    la = (a[..., :3].astype(np.float64) / 255.0) ** (1.0 / 0.6)
    lb = (b[..., :3].astype(np.float64) / 255.0) ** (1.0 / 0.6)
    return float(np.sqrt(((la - lb) ** 2).sum(-1)[vis].mean()))


def test_readme_per_pixel_l2(c3_frame, cornell_arrays, cornell):
    """north_star's per-pixel L2 tolerance against the reference's own output.  The driver's
    sin() makes the reference's noise a different realisation, so the tolerance is stated
    against the oracle's seed-to-seed L2: L2(screenshot, oracle@123) / L2(oracle@456,
    oracle@123) in [0.98, 1.02] (measured 1.001-1.008 over seeds 123/456/789; full frames:
    0.1431 vs 0.1419-0.1429).  Emulating the intended packed luminous ids instead of the std140
    quirk moves it to ~1.08, outside the band."""
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "readme_pixels.npz"))
    ref = d["rgb"][L2_ROWS]
    vis = d["visible"][L2_ROWS]
    ours = c3_frame[0][L2_ROWS]
    other = _rows(cornell_arrays, cornell, 456.0)
    self_l2 = _l2(ours, other, vis)
    ratio = _l2(ref, ours, vis) / self_l2
    assert 0.98 <= ratio <= 1.02, (ratio, self_l2)
    quirk_off = _rows(cornell_arrays, cornell, TIME, lum_id_std140_quirk=0)
    ratio_off = _l2(ref, quirk_off, vis) / self_l2
    assert ratio_off > 1.05, ratio_off
    print(f"per-pixel L2: self {self_l2:.4f}, ratio {ratio:.4f}, quirk off {ratio_off:.4f}")


def _pyref_check(sc, cfg, W, H, pixels, time=TIME):
    arrays = scene_arrays(sc)
    lin, _, _ = O.render(arrays, sc.push_constant(time), cfg, W, H)
    ps = pyref.Scene(arrays["materials"], arrays["vertices"], arrays["faces"],
                     arrays["lum_face_ids"], quirk=bool(cfg["lum_id_std140_quirk"]),
                     spheres=arrays["spheres"] if int(cfg["integrator"]) == 1 else ())
    P = pyref.params(cfg)
    for (x, y) in pixels:
        c, _ = pyref.render_pixel(ps, P, sc.push_constant(time), W, H, x, y)
        assert np.array_equal(np.array(c, dtype=np.float32).view(np.uint32),
                              lin[y, x].view(np.uint32)), (x, y, c, lin[y, x])


def _pixels(W, H, n, seed):
    rng = np.random.default_rng(seed)
    return list(zip(rng.integers(0, W, n).tolist(), rng.integers(0, H, n).tolist()))


def test_pyref_default(cornell):
    _pyref_check(cornell, rvcp_amd.abi.make_config(spp=2), 24, 24, _pixels(24, 24, 24, 1))


def test_pyref_quirk_off(cornell):
    _pyref_check(cornell, rvcp_amd.abi.make_config(spp=2, lum_id_std140_quirk=0), 24, 24,
                 _pixels(24, 24, 16, 2))


def test_pyref_params(cornell):
    cfg = rvcp_amd.abi.make_config(spp=2, max_bounces=3, rr_probability=1.0,
                                   attenuation_stop_eps=0.01, ray_t_max=1000.0)
    _pyref_check(cornell, cfg, 20, 20, _pixels(20, 20, 12, 3), time=7.5)


def test_pyref_moved_camera_random_mesh(cornell):
    base = rvcp_amd.Scene(rvcp_amd.Camera.new([120.0, 400.0, -700.0], [-50.0, 150.0, 100.0],
                                              0.1, 10000.0, 55.0, 150.0, 5.0),
                          cornell.materials, [], cornell.mesh)
    sc = rvcp_amd.scene.with_random_triangles(base, 40)
    _pyref_check(sc, rvcp_amd.abi.make_config(spp=1), 16, 12, _pixels(16, 12, 8, 4))


# ---- integrator mode 2 (ray_tracer.comp, the file north_star names) ----
def test_pyref_legacy_sphere_scene():
    sc = rvcp_amd.scene.sphere_scene()
    _pyref_check(sc, rvcp_amd.abi.make_config(integrator=1, spp=2), 24, 24,
                 _pixels(24, 24, 24, 5), time=3.25)


def test_pyref_legacy_params():
    sc = rvcp_amd.scene.sphere_scene()
    cfg = rvcp_amd.abi.make_config(integrator=1, spp=1, max_bounces=6, rr_probability=0.8)
    _pyref_check(sc, cfg, 20, 16, _pixels(20, 16, 16, 6), time=11.0)


def test_pyref_legacy_cornell(cornell):
    _pyref_check(cornell, rvcp_amd.abi.make_config(integrator=1, spp=2), 16, 16,
                 _pixels(16, 16, 12, 7))


def test_legacy_oracle_image_statistics():
    """Mode 2 on the deprecated host's sphere scene: the room is lit only by the roof light
    (miss = black, no NEE), every path ends on a light or a miss, and the image is UNORM
    (no gamma): u8 = round-half-up(255 * c) for c in [0, 1]."""
    sc = rvcp_amd.scene.sphere_scene()
    cfg = rvcp_amd.abi.make_config(integrator=1)
    arrays = scene_arrays(sc)
    lin, rgba, trav = O.render(arrays, sc.push_constant(1.0), cfg, 64, 64)
    assert np.isfinite(lin).all() and (lin >= 0).all() and (lin <= 1.0).all()
    exp = np.floor(np.clip(lin, 0, 1) * 255.0 + 0.5).astype(np.uint8)
    assert np.abs(exp.astype(int) - rgba[..., :3]).max() <= 1
    assert (rgba[..., 3] == 255).all()
    spp = int(cfg["spp"])
    assert 64 * 64 * spp <= trav <= 64 * 64 * spp * int(cfg["max_bounces"])
    assert 0.2 < float(lin.mean()) < 0.8


@pytest.mark.parametrize("rule", [0, 1], ids=["driver", "nearest"])
def test_unorm_thresholds(rule):
    for k in range(1, 256):
        if rule == 1:
            t = np.float32((k - 0.5) / 255.0)
        else:   # smallest g with (floor(4096 g) * 255 + 2048) >> 12 >= k
            t = np.float32(math.ceil((4096 * k - 2048) / 255) / 4096)
        assert O.unorm_u8(float(t), rule) == k
        assert O.unorm_u8(float(np.nextafter(t, np.float32(0))), rule) == k - 1
    assert O.unorm_u8(-1.0, rule) == 0 and O.unorm_u8(2.0, rule) == 255
    assert O.unorm_u8(float("nan"), rule) == 0