"""Every BASELINE.json configuration rendered by the HIP path at its own size and compared
with the CPU oracle (run on an MI355X: pytest -m gpu).

Tolerance: bit-exact, as in test_gpu_parity.py -- every compared pixel's linear float RGB
bitwise equal, every RGBA8 byte equal, and (for whole frames) the reference-algorithm
traversal count equal.  Coverage per config (BASELINE.json `configs`):

  C1 Cornell 128^2 SPP=1        whole frame (also in test_gpu_parity.py)
  C2 Cornell 384^2 SPP=10       whole frame, default schedule
  C3 Cornell 1024^2 SPP=30      whole frame, default schedule (6); ~4 s of oracle on 16 threads
  C4 Cornell 2048^2 SPP=64      128 rows spread over every stripe offset and every shard of 8
                                 (the whole frame is ~30 s of oracle), plus the 8-shard
                                 device assembly == the 1-shard frame
  C5 Cornell + 100k triangles   64^2 SPP=1 whole frame on the default LDS-tiled schedule (5),
                                 on schedule 4 and on the opt-in BVH; at 1024^2 SPP=30 two
                                 256-pixel row segments (tiled and BVH)
  C6 Cornell + 310 triangles    (bench --workload c6: 342 faces / 998 vertices, the largest
                                 unshared-vertex scene the reference's 1000-entry buffers hold,
                                 ray_tracer_games101_branch.comp:18-19) 128^2 SPP=30 whole frame
                                 on every brute-force schedule, and the 1024^2 SPP=30 frame's
                                 rows at every stripe offset (y mod 8) and shard of 8
"""
import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

pytestmark = pytest.mark.gpu
TIME = 123.0


def _oracle(sc, cfg, W, H, rect=None):
    return O.render(scene_arrays(sc), sc.push_constant(TIME), cfg, W, H, rect=rect)


def _gpu(sc, cfg, W, H):
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(W, H, TIME, want_linear=True)
        return rgba, lin, rt.last_stats.copy()


def _assert_rect(gpu, orc, rect):
    x0, y0, w, h = rect
    rgba, lin = gpu[0][y0:y0 + h, x0:x0 + w], gpu[1][y0:y0 + h, x0:x0 + w]
    o_lin, o_rgba, _ = orc
    diff = np.any(lin.view(np.uint32) != o_lin.view(np.uint32), axis=-1)
    assert not diff.any(), f"{int(diff.sum())} pixels differ in linear RGB, first at " \
                           f"{(np.argwhere(diff)[:3] + [y0, x0]).tolist()}"
    assert np.array_equal(rgba, o_rgba)


def _assert_frame(gpu, orc):
    H, W = gpu[0].shape[:2]
    _assert_rect(gpu, orc, (0, 0, W, H))
    assert int(gpu[2]["traversals"]) == orc[2]


# ---------------------------------------------------------------- C2 / C3: whole frames --
@pytest.mark.parametrize("W,H,spp", [(384, 384, 10), (1024, 1024, 30)], ids=["C2", "C3"])
def test_whole_frame_bitexact(cornell, W, H, spp):
    cfg = rvcp_amd.abi.make_config(spp=spp)
    _assert_frame(_gpu(cornell, cfg, W, H), _oracle(cornell, cfg, W, H))


# ---------------------------------------------------------------- C4: 2048^2 SPP=64 ------
C4_ROWS = sorted({16 * i + (5 * i) % 16 for i in range(128)} | {0, 2047})


@pytest.fixture(scope="module")
def c4_render(cornell):
    cfg = rvcp_amd.abi.make_config(spp=64)
    return cfg, _gpu(cornell, cfg, 2048, 2048)


def test_c4_rows_bitexact(cornell, c4_render):
    cfg, g = c4_render
    assert len(C4_ROWS) >= 128
    assert {y % 8 for y in C4_ROWS} == set(range(8))            # every row of a stripe
    assert {(y // 8) % 8 for y in C4_ROWS} == set(range(8))     # every shard of 8
    for y in C4_ROWS:
        _assert_rect(g, _oracle(cornell, cfg, 2048, 2048, rect=(0, y, 2048, 1)), (0, y, 2048, 1))


def test_c4_traversals_per_sample(c4_render):
    _, g = c4_render
    per_sample = int(g[2]["traversals"]) / (2048 * 2048 * 64)
    assert 4.7 < per_sample < 5.1


def test_c4_eight_shards_assemble(cornell, c4_render):
    """The BASELINE 8-GPU form of C4: 8 shards of 8-row stripes, gathered into one buffer and
    assembled on the device, equal the 1-shard frame (all shards on this one GPU)."""
    torch = pytest.importorskip("torch")
    cfg, g = c4_render
    W = H = 2048
    n = 8
    slot = max(rvcp_amd.shard_rows(H, k, n) for k in range(n))
    gathered = torch.zeros((n, slot, W), dtype=torch.int32, device="cuda")
    frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(cornell)
        push = cornell.push_constant(TIME)
        for k in range(n):
            rt.render_shard_async(push, W, H, k, n, gathered[k].data_ptr(), stream=stream)
            rt.sync_stats()
        rt.assemble_frame_async(gathered.data_ptr(), slot, W, H, n, frame.data_ptr(), stream=stream)
        torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().view(np.uint8).reshape(H, W, 4), g[0])


# ---------------------------------------------------------------- C5: + 100k triangles ---
@pytest.fixture(scope="module")
def c5_scene(cornell):
    return rvcp_amd.scene.with_random_triangles(cornell, 100000)


@pytest.fixture(scope="module")
def c5_small_oracle(c5_scene):
    cfg = rvcp_amd.abi.make_config(spp=1)
    return cfg, _oracle(c5_scene, cfg, 64, 64)


@pytest.mark.parametrize("kw", [dict(), dict(kernel_variant=4), dict(kernel_variant=10),
                                dict(kernel_variant=3), dict(accel=1)],
                         ids=["default", "tiled4", "tiledpool10", "scalar3", "bvh"])
def test_c5_small_bitexact(c5_scene, c5_small_oracle, kw):
    """64^2 SPP=1 of the C5 mesh, whole frame: the default schedule for 100k faces is the
    LDS-tiled single-ray kernel (5); the BVH is compared with the oracle directly, not with
    the brute-force HIP path."""
    cfg, orc = c5_small_oracle
    g = _gpu(c5_scene, rvcp_amd.abi.make_config(spp=1, **kw), 64, 64)
    _assert_frame(g, orc)


C5_RECTS = [(384, 512, 256, 1), (640, 200, 256, 1)]


@pytest.mark.parametrize("kw", [dict(), dict(kernel_variant=10), dict(accel=1)],
                         ids=["tiled", "tiledpool10", "bvh"])
def test_c5_full_size_segments(c5_scene, kw):
    """The C5 frame at its own size (1024^2 SPP=30): two 256-pixel row segments through the
    middle of the room (floor, boxes, back wall) against the oracle."""
    cfg = rvcp_amd.abi.make_config(spp=30, **kw)
    g = _gpu(c5_scene, cfg, 1024, 1024)
    for rect in C5_RECTS:
        _assert_rect(g, _oracle(c5_scene, rvcp_amd.abi.make_config(spp=30), 1024, 1024, rect=rect), rect)


# ---------------------------------------------------------------- C6: the reference's limit --
@pytest.fixture(scope="module")
def c6_scene(cornell):
    import bench
    sc = rvcp_amd.scene.with_random_triangles(cornell, bench.C6_EXTRA_TRIS)
    assert len(sc.mesh.aligned_faces()) == 342 and len(sc.mesh.aligned_vertices()) == 998
    return sc


@pytest.fixture(scope="module")
def c6_small_oracle(c6_scene):
    cfg = rvcp_amd.abi.make_config(spp=30)
    return cfg, _oracle(c6_scene, cfg, 128, 128)


@pytest.mark.parametrize("kw", [dict(), dict(kernel_variant=3), dict(kernel_variant=4),
                                dict(kernel_variant=5), dict(kernel_variant=6),
                                dict(kernel_variant=10), dict(accel=1)],
                         ids=["default", "scalar3", "tiled4", "tiled5", "scalar6", "tiledpool10", "bvh"])
def test_c6_small_bitexact(c6_scene, c6_small_oracle, kw):
    """128^2 SPP=30 of the c6 scene (342 faces), whole frame, every brute-force schedule and
    the BVH, against the oracle: linear bits, RGBA8 and the traversal count."""
    cfg, orc = c6_small_oracle
    _assert_frame(_gpu(c6_scene, rvcp_amd.abi.make_config(spp=30, **kw), 128, 128), orc)


C6_ROWS = sorted({8 * (13 * i % 128) + i % 8 for i in range(24)} | {0, 1023})


def test_c6_full_size_rows(c6_scene):
    """The bench's c6 frame at its own size (1024^2 SPP=30, the default schedule): rows at
    every stripe offset and every shard of 8, against the oracle."""
    assert {y % 8 for y in C6_ROWS} == set(range(8))
    assert {(y // 8) % 8 for y in C6_ROWS} == set(range(8))
    cfg = rvcp_amd.abi.make_config(spp=30)
    g = _gpu(c6_scene, cfg, 1024, 1024)
    for y in C6_ROWS:
        _assert_rect(g, _oracle(c6_scene, cfg, 1024, 1024, rect=(0, y, 1024, 1)), (0, y, 1024, 1))


# ---------------------------------------------------------------- UNORM8 rules -------------
@pytest.mark.parametrize("integrator", [0, 1], ids=["games101", "mode2"])
@pytest.mark.parametrize("rule", [0, 1], ids=["driver", "nearest"])
def test_unorm_rules_bitexact(cornell, integrator, rule):
    """rvcp_config_t.unorm_rule: the driver's 12-bit conversion (default) and round-to-nearest,
    through the gamma store (games101) and the gamma-free store (mode 2), C1 size."""
    sc = cornell if integrator == 0 else rvcp_amd.scene.sphere_scene()
    cfg = rvcp_amd.abi.make_config(spp=2, integrator=integrator, unorm_rule=rule)
    _assert_frame(_gpu(sc, cfg, 128, 128), _oracle(sc, cfg, 128, 128))
