"""bench.py host logic on CPU: the workload table against BASELINE.json's configs, the roofline
constants, and the loaders of the committed PMC summaries (no GPU, nothing rendered)."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_workloads_match_baseline_configs():
    """C1-C5 sizes are BASELINE.json configs[0..4]; N=1 defaults to C3, N>1 C4 is strong."""
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        configs = json.load(f)["configs"]
    want = {"c1": (128, 1), "c2": (384, 10), "c3": (1024, 30), "c4": (2048, 64), "c5": (1024, 30)}
    for (name, (side, spp)), text in zip(want.items(), configs):
        wl = bench.workload(name, 1)
        assert (wl["W"], wl["H"], wl["spp"]) == (side, side, spp)
        assert f"{side}" in text and f"SPP={spp}" in text
    assert bench.workload("c5", 1)["extra_tris"] == 100000
    assert bench.workload("c4", 8)["scaling"] == "strong"
    assert bench.workload("c4", 8)["W"] == 2048                 # fixed frame at any N
    assert bench.workload("c3", 1)["workload"] == "cornell_1024sq_spp30"
    assert bench.workload("c3", 4)["W"] == 2048                 # weak-scaled C3 side
    m2 = bench.workload("c3m2", 1)
    assert (m2["W"], m2["spp"], m2["integrator"], m2["scene"]) == (1024, 30, 1, "cornell")
    assert bench.workload("spheres", 1)["scene"] == "spheres"
    with pytest.raises(SystemExit):
        bench.workload("nope", 1)


def test_roofline_constants():
    assert bench.FLOP_PER_TEST == 52 and bench.FP32_PEAK_TFLOPS == 157.3
    assert bench.REFERENCE_MSAMPLES["c3"] == pytest.approx(1024 * 1024 * 30 * 3 / 1e6, rel=0.01)
    assert bench.REFERENCE_MSAMPLES["c2"] == pytest.approx(384 * 384 * 10 * 51 / 1e6, rel=0.01)


def test_committed_pmc_summaries_load():
    """The bench line's traffic / VALU fields come from these summaries: they exist for the
    headline C3 kernel and the C5 tiled kernel, and carry per-launch numbers."""
    for wl, kname in [("cornell_1024sq_spp30", "rvcp_spec_path_kernel5"),
                      ("cornell_plus_100k_tris_1024sq_spp30", "games101_tiled_kernel")]:
        traffic, src = bench.load_traffic(wl, kname)
        assert traffic and traffic > 0 and src.startswith("profiles/")
        busy, frac = bench.load_valu_busy(wl, kname)
        assert 0 < busy <= 1 and 0 < frac <= 1
