"""The headline pipeline at full size, against the oracle:

* bench.py renders every timed frame with its own time seed (TIME0 + frame index, as the
  reference re-stamps `time` per frame, vulkan.rs:418-421) in batches of frames per path
  kernel (rvcp_render_frames_async).  Here a C3 batch of 3 frames with 3 different seeds
  goes through that entry point and EVERY frame is compared, whole, with the oracle's render
  of its seed: every RGBA8 byte and every linear-RGB bit.
* the off-axis Cornell box (scene.rotated_scene, bench --workload c3rot): no exact-zero
  triangle component, so the scene-specialised scan keeps every product; its frames against
  the oracle, and against the generic scan.
* `python bench.py --gpus 2` started WITHOUT a launcher (the driver's form) starts its ranks
  itself (bench.self_launch) and prints one valid line (one-GPU rehearsal: both ranks on GPU 0,
  gloo gather), whose assembled frame is bit-identical to the one-GPU render."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from rvcp_amd import scene as S
from conftest import scene_arrays

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEEDS = (123.0, 124.0, 611.0)


def test_c3_batch_distinct_seeds_whole_frames_vs_oracle(cornell):
    torch = pytest.importorskip("torch")
    W = H = 1024
    spp = 30
    out = torch.zeros((len(SEEDS), H, W), dtype=torch.int32, device="cuda")
    lin = torch.zeros((len(SEEDS), H, W, 3), dtype=torch.float32, device="cuda")
    with rvcp_amd.RayTracer(spp=spp) as rt:
        rt.upload_scene(cornell)
        rt.render_frames_async([cornell.push_constant(t) for t in SEEDS], W, H, 0, 1,
                               out.data_ptr(), lin.data_ptr())
        st = rt.sync_stats()
        torch.cuda.synchronize()
    assert int(st["kernel_variant"]) & rvcp_amd.abi.VARIANT_SPECIALIZED    # the headline kernel
    got = out.cpu().numpy().view(np.uint8).reshape(len(SEEDS), H, W, 4)
    got_lin = lin.cpu().numpy()
    cfg = rvcp_amd.abi.make_config(spp=spp)
    trav = 0
    for f, t in enumerate(SEEDS):
        o_lin, o_rgba, o_trav = O.render(scene_arrays(cornell), cornell.push_constant(t), cfg, W, H)
        assert np.array_equal(got[f], o_rgba), (f, int(np.count_nonzero(np.any(got[f] != o_rgba, -1))))
        assert np.array_equal(got_lin[f].view(np.uint32), o_lin.view(np.uint32)), f
        trav += o_trav
    assert int(st["traversals"]) == trav
    assert not np.array_equal(got[0], got[1])


@pytest.fixture(scope="module")
def rotated():
    return S.rotated_scene(rvcp_amd.Scene.default())


@pytest.mark.parametrize("W,H,spp", [(256, 256, 8), (97, 61, 5)])
def test_rotated_scene_vs_oracle(rotated, W, H, spp):
    """The specialised scan on a scene without zero components, whole frames, bit-exact."""
    with rvcp_amd.RayTracer(spp=spp) as rt:
        rt.upload_scene(rotated)
        rgba, lin = rt.render(W, H, 123.0, want_linear=True)
        st = rt.last_stats
    assert int(st["kernel_variant"]) & rvcp_amd.abi.VARIANT_SPECIALIZED
    o_lin, o_rgba, o_trav = O.render(scene_arrays(rotated), rotated.push_constant(123.0),
                                     rvcp_amd.abi.make_config(spp=spp), W, H)
    assert np.array_equal(rgba, o_rgba)
    assert np.array_equal(lin.view(np.uint32), o_lin.view(np.uint32))
    assert int(st["traversals"]) == o_trav


def test_rotated_c3_rows_specialised_equals_generic_and_oracle(rotated):
    """At the C3 size: the specialised and the generic scan give the same frame; rows of every
    stripe offset against the oracle."""
    W = H = 1024
    frames = []
    for spec in (rvcp_amd.abi.SPECIALIZE_AUTO, rvcp_amd.abi.SPECIALIZE_OFF):
        with rvcp_amd.RayTracer(spp=30, specialize=spec) as rt:
            rt.upload_scene(rotated)
            rgba, _ = rt.render(W, H, 123.0, want_linear=True)
            frames.append(rgba)
    assert np.array_equal(frames[0], frames[1])
    cfg = rvcp_amd.abi.make_config(spp=30)
    for y in (0, 9, 130, 515, 766, 1023):
        _, o_rgba, _ = O.render(scene_arrays(rotated), rotated.push_constant(123.0), cfg, W, H,
                                rect=(0, y, W, 1), want_linear=False)
        assert np.array_equal(frames[0][y:y + 1], o_rgba), y


def test_bench_self_launch_rehearsal_n2():
    env = dict(os.environ, RVCP_BENCH_REHEARSAL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "RVCP_LIB"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--workload", "c2", "--steps", "8", "--warmup", "2", "--launch-pass", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 8 and d["value"] > 0
    assert "sharded over 2 GPUs" in d["metric"]
    c = d["config"]
    assert c["assembled_frame_bitexact_vs_1gpu"] is True
    assert c["one_gpu_value"] > 0 and c["physical_gpus"] == 1
    assert "torch imported: False" in r.stderr          # the parent never touched the GPU
