"""The seeded scenes of the specialiser fuzz (tests/fuzz_scenes.py, rendered on the GPU by
tests/test_gpu_spec_fuzz.py) are meaningful on the CPU oracle: every one renders a frame in
which paths bounce (more traversals than samples, not an all-miss frame), every camera's primary
t range stays below 2^24 (rvcp_host.cpp primary_t_range_ok), and the coordinates span the
magnitudes the fuzz is for (2^-20 .. 2^38)."""
import numpy as np

import oracle as O
import rvcp_amd
from conftest import scene_arrays
from fuzz_scenes import N_FUZZ, fuzz_scene, positions


def test_fuzz_scenes_render_and_span_magnitudes():
    W, H = 48, 40
    lo, hi = np.inf, 0.0
    for seed in range(N_FUZZ):
        sc, kw, desc = fuzz_scene(seed)
        p = np.abs(positions(sc))
        lo, hi = min(lo, float(p[p > 0].min())), max(hi, float(p.max()))
        cam = sc.push_constant(1.0)["camera"]
        t = np.tan(np.radians(float(cam["vertical_fov"]) / 2))
        assert float(cam["t_far"]) * np.sqrt(1 + t * t * (1 + (W / H) ** 2)) * 1.001 < 2 ** 24, desc
        _, _, trav = O.render(scene_arrays(sc), sc.push_constant(100.0 + seed),
                              rvcp_amd.abi.make_config(**kw), W, H)
        assert trav > W * H * kw["spp"], desc
    assert lo <= 2.0 ** -20 and hi >= 2.0 ** 38, (lo, hi)
