"""HIP kernel vs CPU oracle parity (run on an MI355X: pytest -m gpu).

Tolerance: bit-exact.  The kernel and the oracle implement the same numeric contract
(DESIGN.md §3), so every pixel's linear float RGB must be bitwise equal, every RGBA8 byte
equal, and the traversal counts (control-flow fingerprint) equal.  Here the full-size C3
frame (1024^2 SPP=30) is checked on sampled rows plus size-independent properties
(determinism, sharding invariance, README statistics); the whole C2 / C3 frames, C4 rows and
the C5 mesh are compared with the oracle in test_gpu_configs.py.
"""
import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import block_means, readme_blocks, scene_arrays

pytestmark = pytest.mark.gpu
TIME = 123.0


def _oracle(sc, cfg, W, H, rect=None, time=TIME):
    return O.render(scene_arrays(sc), sc.push_constant(time), cfg, W, H, rect=rect)


def _gpu(sc, cfg, W, H, time=TIME):
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(W, H, time, want_linear=True)
        return rgba, lin, rt.last_stats


def _assert_same(gpu, orc):
    rgba, lin, stats = gpu
    o_lin, o_rgba, o_trav = orc
    diff = np.any(lin.view(np.uint32) != o_lin.view(np.uint32), axis=-1)
    assert not diff.any(), f"{int(diff.sum())} pixels differ in linear RGB, first at " \
                           f"{np.argwhere(diff)[:3].tolist()}"
    assert np.array_equal(rgba, o_rgba)
    assert int(stats["traversals"]) == o_trav


VARIANTS = [1, 2, 3, 4, 5, 6, 10]  # kernel schedules (rvcp_config_t::kernel_variant); 0 = default


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("W,H,spp", [(64, 64, 4), (128, 128, 1), (37, 23, 3), (8, 8, 30),
                                     (1, 1, 7), (130, 3, 2)])
def test_bitexact_cornell(cornell, W, H, spp, variant):
    cfg = rvcp_amd.abi.make_config(spp=spp, kernel_variant=variant)
    _assert_same(_gpu(cornell, cfg, W, H), _oracle(cornell, cfg, W, H))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", ["quirk_off", "params", "no_lights", "random_mesh", "rr1"])
def test_variants_bitexact(cornell, variant, case):
    sc, kw = cornell, dict(spp=3)
    if case == "quirk_off":
        kw["lum_id_std140_quirk"] = 0
    elif case == "params":
        kw.update(max_bounces=2, attenuation_stop_eps=0.2, eps=0.01)
    elif case == "rr1":
        kw.update(rr_probability=1.0, max_bounces=4)
    elif case == "no_lights":
        mats = list(cornell.materials)
        mats[3] = rvcp_amd.Material.new_lambertian([0.5, 0.5, 0.5])
        sc = rvcp_amd.Scene(cornell.camera, mats, [], cornell.mesh)
    elif case == "random_mesh":
        sc = rvcp_amd.scene.with_random_triangles(cornell, 200)
    cfg = rvcp_amd.abi.make_config(kernel_variant=variant, **kw)
    _assert_same(_gpu(sc, cfg, 40, 36), _oracle(sc, cfg, 40, 36))


@pytest.mark.parametrize("variant", [4, 5, 10])
def test_multi_tile_bitexact(cornell, variant):
    """LDS-tiled schedules over several triangle tiles (732 faces = 2 full tiles of 256 and a
    partial one), nearest hits spread across tiles."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, 700)
    cfg = rvcp_amd.abi.make_config(kernel_variant=variant, spp=2)
    _assert_same(_gpu(sc, cfg, 48, 40), _oracle(sc, cfg, 48, 40))


@pytest.mark.parametrize("variant", [4, 5, 10])
@pytest.mark.parametrize("extra", [201, 225, 259])
def test_tiled_odd_remainder_bitexact(cornell, variant, extra):
    """The tiled scans take two triangles per step and the last one of an
    odd tile alone: 233 faces (one odd tile), 257 (a full tile, then a single triangle) and
    291 (a full tile, then 35)."""
    sc = rvcp_amd.scene.with_random_triangles(cornell, extra)
    cfg = rvcp_amd.abi.make_config(kernel_variant=variant, spp=2)
    _assert_same(_gpu(sc, cfg, 40, 32), _oracle(sc, cfg, 40, 32))


def test_bitexact_quirk_off(cornell):
    cfg = rvcp_amd.abi.make_config(spp=4, lum_id_std140_quirk=0)
    _assert_same(_gpu(cornell, cfg, 64, 64), _oracle(cornell, cfg, 64, 64))


@pytest.mark.parametrize("kw", [dict(spp=5, max_bounces=3, rr_probability=1.0,
                                     attenuation_stop_eps=0.01, ray_t_max=1000.0),
                                dict(spp=2, max_bounces=1), dict(spp=3, rr_probability=0.5),
                                dict(spp=2, eps=0.01, ray_t_min=0.5)])
def test_bitexact_params(cornell, kw):
    cfg = rvcp_amd.abi.make_config(**kw)
    _assert_same(_gpu(cornell, cfg, 48, 40), _oracle(cornell, cfg, 48, 40))


@pytest.mark.parametrize("time", [0.0, 1.5, 999.0, 421.25])
def test_bitexact_time_seeds(cornell, time):
    cfg = rvcp_amd.abi.make_config(spp=2)
    _assert_same(_gpu(cornell, cfg, 40, 40, time=time), _oracle(cornell, cfg, 40, 40, time=time))


def test_bitexact_moved_camera(cornell):
    sc = rvcp_amd.Scene(rvcp_amd.Camera.new([120.0, 400.0, -700.0], [-50.0, 150.0, 100.0],
                                            0.1, 10000.0, 55.0, 150.0, 5.0),
                        cornell.materials, [], cornell.mesh)
    cfg = rvcp_amd.abi.make_config(spp=3)
    _assert_same(_gpu(sc, cfg, 64, 48), _oracle(sc, cfg, 64, 48))


def test_trivial_configs_black(cornell):
    for kw in (dict(max_bounces=0), dict(attenuation_stop_eps=1.5)):
        cfg = rvcp_amd.abi.make_config(spp=3, **kw)
        g = _gpu(cornell, cfg, 16, 8)
        o = _oracle(cornell, cfg, 16, 8)
        _assert_same(g, o)
        assert o[2] == 0 and (g[0][..., :3] == 0).all()


def test_no_lights(cornell):
    mats = list(cornell.materials)
    mats[3] = rvcp_amd.Material.new_lambertian([0.5, 0.5, 0.5])
    sc = rvcp_amd.Scene(cornell.camera, mats, [], cornell.mesh)
    assert len(sc.luminous_face_ids()) == 0
    cfg = rvcp_amd.abi.make_config(spp=3)
    _assert_same(_gpu(sc, cfg, 32, 32), _oracle(sc, cfg, 32, 32))


def test_random_mesh(cornell):
    sc = rvcp_amd.scene.with_random_triangles(cornell, 300)
    cfg = rvcp_amd.abi.make_config(spp=2)
    _assert_same(_gpu(sc, cfg, 48, 48), _oracle(sc, cfg, 48, 48))


def test_empty_mesh(cornell):
    sc = rvcp_amd.Scene(cornell.camera, cornell.materials, [], rvcp_amd.Mesh([], []))
    cfg = rvcp_amd.abi.make_config(spp=2)
    g = _gpu(sc, cfg, 16, 16)
    _assert_same(g, _oracle(sc, cfg, 16, 16))
    assert (g[0][..., :3] == 64).all()          # every pixel is the 0.1 miss colour


def test_upload_validation(cornell):
    with rvcp_amd.RayTracer() as rt:
        faces = cornell.mesh.aligned_faces().copy()
        faces[3]["vertices"][1] = 9999
        with pytest.raises(rvcp_amd.abi.RvcpError):
            rt.upload_arrays(cornell.aligned_materials(), cornell.mesh.aligned_vertices(), faces,
                             cornell.luminous_face_ids())
        with pytest.raises(rvcp_amd.abi.RvcpError):
            rt.render_push(cornell.push_constant(TIME), 8, 8)   # no scene uploaded yet


def test_frame_size_limits(cornell):
    """W*H must be in [1, 2^31): rejected with RVCP_E_INVALID before any allocation; the
    context stays usable."""
    torch = pytest.importorskip("torch")
    d = torch.zeros(16, dtype=torch.int32, device="cuda")
    with rvcp_amd.RayTracer(spp=1) as rt:
        rt.upload_scene(cornell)
        push = cornell.push_constant(TIME)
        for W, H in [(65536, 32768), (0, 16), (16, 0)]:
            with pytest.raises(rvcp_amd.abi.RvcpError) as e:
                rt.render_async(push, W, H, d.data_ptr())
            assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID
        assert rt.render(4, 4, TIME).shape == (4, 4, 4)


# ----------------------------------------------------------------------------------------
# Full-size (C3: 1024^2, SPP=30) properties
# ----------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c3_render(cornell):
    cfg = rvcp_amd.abi.make_config(spp=30)
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(cornell)
        a, lin = rt.render(1024, 1024, TIME, want_linear=True)
        stats = rt.last_stats.copy()
        b = rt.render(1024, 1024, TIME)
    return cfg, a, lin, b, stats


@pytest.mark.parametrize("variant", VARIANTS)
def test_c3_variants_identical(cornell, c3_render, variant):
    """Every kernel schedule renders the identical full-size frame."""
    cfg = rvcp_amd.abi.make_config(spp=30, kernel_variant=variant)
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(cornell)
        img = rt.render(1024, 1024, TIME)
        trav = int(rt.last_stats["traversals"])
    assert np.array_equal(img, c3_render[1])
    assert trav == int(c3_render[4]["traversals"])


def test_c3_deterministic(c3_render):
    _, a, _, b, _ = c3_render
    assert np.array_equal(a, b)


def test_c3_rows_bitexact(cornell, c3_render):
    cfg, a, lin, _, _ = c3_render
    rng = np.random.default_rng(7)
    for y in sorted(rng.choice(1024, 6, replace=False).tolist()) + [0, 1023]:
        o_lin, o_rgba, _ = _oracle(cornell, cfg, 1024, 1024, rect=(0, y, 1024, 1))
        assert np.array_equal(lin[y:y + 1].view(np.uint32), o_lin.view(np.uint32)), y
        assert np.array_equal(a[y:y + 1], o_rgba), y


def test_c3_traversals_per_sample(c3_render):
    *_, stats = c3_render
    per_sample = int(stats["traversals"]) / (1024 * 1024 * 30)
    assert 4.7 < per_sample < 5.1          # 4.91 measured on the model


def test_c3_matches_reference_screenshot(c3_render):
    """Statistical parity with the reference's own output (README screenshot, 1024^2 SPP=30,
    different sin() implementation so only block statistics can match)."""
    _, a, _, _, _ = c3_render
    b32, _ = readme_blocks()
    ours = block_means(a, 32)
    ok = np.isfinite(b32)
    rms = float(np.sqrt(np.mean((ours[ok] - b32[ok]) ** 2)))
    assert rms < 0.006, rms


@pytest.mark.parametrize("n_shards", [2, 3, 8])
def test_shard_assembly_bitexact(cornell, n_shards):
    """Sharded render (8-row stripes dealt round-robin) + device assembly == 1-shard render."""
    torch = pytest.importorskip("torch")
    W, H = 96, 83
    cfg = rvcp_amd.abi.make_config(spp=3)
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(cornell)
        full = rt.render(W, H, TIME)
        push = cornell.push_constant(TIME)
        slot = max(rvcp_amd.shard_rows(H, k, n_shards) for k in range(n_shards))
        gathered = torch.zeros((n_shards, slot, W), dtype=torch.int32, device="cuda")
        for k in range(n_shards):
            rt.render_shard_async(push, W, H, k, n_shards, gathered[k].data_ptr(),
                                  stream=torch.cuda.current_stream().cuda_stream)
            rt.sync_stats()
        frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
        rt.assemble_frame_async(gathered.data_ptr(), slot, W, H, n_shards, frame.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    got = frame.cpu().numpy().view(np.uint8).reshape(H, W, 4)
    assert np.array_equal(got, full)


def test_render_async_wait(cornell):
    """rvcp_render_async / rvcp_wait (device output, caller's stream) == rvcp_render."""
    torch = pytest.importorskip("torch")
    W, H = 77, 45
    cfg = rvcp_amd.abi.make_config(spp=3)
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(cornell)
        full, lin = rt.render(W, H, TIME, want_linear=True)
        st_sync = rt.last_stats
        d_rgba = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        d_lin = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
        rt.render_async(cornell.push_constant(TIME), W, H, d_rgba.data_ptr(), d_lin.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream)
        st = rt.wait()
        with pytest.raises(rvcp_amd.abi.RvcpError):
            rt.wait()                   # nothing in flight any more
    assert np.array_equal(d_rgba.cpu().numpy().view(np.uint8).reshape(H, W, 4), full)
    assert np.array_equal(d_lin.cpu().numpy().view(np.uint32), lin.view(np.uint32))
    assert int(st["traversals"]) == int(st_sync["traversals"])
    with rvcp_amd.RayTracer(rvcp_amd.abi.make_config(spp=1, n_gpus=2)) as rt:
        rt.upload_scene(cornell)
        with pytest.raises(rvcp_amd.abi.RvcpError) as e:
            rt.render_async(cornell.push_constant(TIME), W, H, d_rgba.data_ptr())
        assert e.value.code == rvcp_amd.abi.RVCP_E_UNSUPPORTED


@pytest.mark.parametrize("n_gpus", [2, 3, 8])
@pytest.mark.parametrize("W,H,spp", [(64, 64, 2), (37, 29, 3), (130, 3, 2), (256, 200, 1)])
def test_single_process_multi_gpu(cornell, n_gpus, W, H, spp):
    """rvcp_config_t.n_gpus > 1 (single process, strided peer copies of the stripes into the
    frame's GPU): bit-identical to one GPU.  On a 1-GPU box every shard runs on device 0,
    which exercises the sharding and the copy geometry."""
    one = _gpu(cornell, rvcp_amd.abi.make_config(spp=spp), W, H)
    many = _gpu(cornell, rvcp_amd.abi.make_config(spp=spp, n_gpus=n_gpus), W, H)
    assert np.array_equal(many[0], one[0])
    assert np.array_equal(many[1].view(np.uint32), one[1].view(np.uint32))
    assert int(many[2]["traversals"]) == int(one[2]["traversals"])
    assert int(many[2]["samples"]) == int(one[2]["samples"])


def test_single_process_multi_gpu_legacy():
    sc = rvcp_amd.scene.sphere_scene()
    one = _gpu(sc, rvcp_amd.abi.make_config(integrator=1), 96, 80)
    many = _gpu(sc, rvcp_amd.abi.make_config(integrator=1, n_gpus=4), 96, 80)
    assert np.array_equal(many[1].view(np.uint32), one[1].view(np.uint32))
