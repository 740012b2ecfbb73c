"""bench.py end to end on the GPU (the driver's command, a short run): the JSON line carries
the contract's fields, its roofline is the wall-clock one (frac <= 1, derived from
ms_per_step), the per-launch pass ran with one frame in flight, and the frame it rendered is
bit-identical to the oracle's on sampled rows (--save-frame)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_auto(pixels, spp, hwq, steps):
    sys.path.insert(0, ROOT)
    import bench
    fif, grid, batch = bench.auto_pipeline(pixels, spp, False, True, hwq, "none", steps)
    return fif, (grid if fif >= 3 else 0), batch


@pytest.mark.parametrize("workload,side,spp,steps", [("c2", 384, 10, 26), ("c3", 1024, 30, 13)])
def test_bench_line(tmp_path, workload, side, spp, steps):
    """C2 and C3 (bench.auto_pipeline: batches of frames per path kernel, 2 in flight; step
    counts that leave a shorter last batch); the saved frame -- the first of a batch -- is the
    oracle's."""
    frame_path = tmp_path / "frame.npy"
    env = dict(os.environ)
    env.pop("RVCP_LIB", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload,
                        "--steps", str(steps), "--warmup", "2", "--no-cpu-baseline",
                        "--save-frame", str(frame_path)],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == 2
    W = H = side
    c = d["config"]
    assert (c["frames_in_flight"], c["grid_waves_per_simd"], c["frames_per_launch"]) == \
        bench_auto(W * H, spp, c["gpu_max_hw_queues"], steps)
    assert c["frames_per_launch"] > 1          # batches of 6 / 3, the last one shorter
    assert c["frame_latency_ms_alone"] > 0
    assert d["value"] == pytest.approx(W * H * spp / (d["ms_per_step"] / 1000.0) / 1e6, rel=2e-3)
    rl = d["roofline"]
    assert rl["bound"] == "valu" and rl["peak"] == 157.3
    flop = rl["tests_per_launch"] * 52
    assert rl["achieved"] == pytest.approx(flop / (d["ms_per_step"] / 1000.0) / 1e12, rel=2e-2)
    assert 0 < rl["frac"] <= 1 and 0 < rl["frac_executed"] <= rl["frac"]
    pl = rl["per_launch"]
    assert pl["frames"] >= 1 and 0 < pl["frac"] <= 1
    assert 0 < pl["frac_executed"] <= pl["frac"]
    assert pl["frac_executed"] == pytest.approx(pl["frac"] * rl["frac_executed"] / rl["frac"], rel=2e-3)
    # PMC-derived fields only from a summary of this very build
    pb = rl["profile_binding"]
    assert set(pb["build"]) == {"source", "module"} and pb["build"]["source"]
    assert rl["stale_profile"] == any(pb[k]["build_match"] is False for k in ("valu", "traffic"))
    if pb["valu"]["build_match"] is not True:
        assert rl["valu_issue_frac_pmc_guide"] is None and rl["valu_insts_per_frame_pmc"] is None
    if pb["traffic"]["build_match"] is not True:
        assert rl["traffic"] is None
    assert pl["kernel_ms_min"] <= pl["kernel_ms"]
    # the clock is this run's (the path kernel's own stamps), not a
    # constant; no "ceiling" field that the wall clock exceeds; the reference's loop shape
    assert "valu_issue_frac_pmc_measured_ceiling" not in rl
    assert 1.0 < rl["shader_clock_ghz"] < 3.0 and 1.0 < rl["shader_clock_ghz_isolated"] < 3.0
    if rl["valu_insts_per_frame_pmc"]:
        want = rl["valu_insts_per_frame_pmc"] / (d["ms_per_step"] * 1e-3 * rl["shader_clock_ghz"]
                                                 * 1e9 * 1024 * 0.5)
        assert rl["valu_issue_frac_wall"] == pytest.approx(want, rel=1e-3)
    assert c["interactive_ms_per_step"] > 0 and c["interactive_frames"] == 60
    # one frame in flight per swapchain image, at most the reference's 3 (vulkan.rs:213)
    assert 1 <= c["interactive_frames_in_flight"] <= 3
    assert c["interactive_grid_waves_per_simd"] >= 0
    # one frame per launch cannot beat the batched pipeline by much, nor lose by more than the
    # tail it leaves (C2's frames are mostly tail)
    assert 0.8 * d["ms_per_step"] < c["interactive_ms_per_step"] < 6.0 * d["ms_per_step"]
    # vs_baseline compares the reference's published row with the reference's
    # own loop shape (one frame per launch, pushes stamped at submission), not with the batched
    # pipeline's rate; the batched ratio is reported beside it
    ref = {"c2": 75.2, "c3": 94.4}[workload]
    loop_msps = W * H * spp / (c["interactive_ms_per_step"] / 1000.0) / 1e6
    assert c["interactive_msamples_s"] == pytest.approx(loop_msps, rel=2e-3)
    assert d["vs_baseline"] == pytest.approx(loop_msps / ref, rel=5e-3)
    assert d["vs_baseline_batched"] == pytest.approx(d["value"] / ref, rel=5e-3)
    # every frame has its own seed (123.0 + frame index); the saved frame is the oracle's
    # render of its seed
    assert c["saved_frame_time"] >= 123.0
    assert d["frame_interval_ms_median"] > 0 and "frame_ms_median" not in d
    frame = np.load(frame_path)
    sc = rvcp_amd.Scene.default()
    cfg = rvcp_amd.abi.make_config(spp=spp)
    for y in (0, 131, 200, H - 1):
        _, o_rgba, _ = O.render(scene_arrays(sc), sc.push_constant(c["saved_frame_time"]), cfg, W, H,
                                rect=(0, y, W, 1), want_linear=False)
        assert np.array_equal(frame[y:y + 1], o_rgba), y
