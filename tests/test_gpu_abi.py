"""C-ABI contract on the GPU: one frame in flight per context, and the one-process-per-GPU
RCCL gather (rvcp_rccl_init / rvcp_gather_frame_async) at world size 1 -- the form every
rank of the multi-GPU bench runs (include/rvcp.h)."""
import numpy as np
import pytest

import rvcp_amd

pytestmark = pytest.mark.gpu
TIME = 123.0


def test_one_frame_in_flight(cornell):
    """A second async frame, an upload or a Mandelbrot call while a frame is pending on the
    context is rejected (RVCP_E_INVALID) instead of overwriting the pending frame's surface
    list, counters and events; after rvcp_wait the context renders again, and both frames
    equal the synchronous render."""
    torch = pytest.importorskip("torch")
    W, H = 96, 64
    with rvcp_amd.RayTracer(spp=3) as rt:
        rt.upload_scene(cornell)
        ref = rt.render(W, H, TIME)
        push = cornell.push_constant(TIME)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        a = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        b = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        rt.render_async(push, W, H, a.data_ptr(), stream=s1.cuda_stream)
        for call in (lambda: rt.render_async(push, W, H, b.data_ptr(), stream=s2.cuda_stream),
                     lambda: rt.render_shard_async(push, W, H, 0, 2, b.data_ptr(), stream=s2.cuda_stream),
                     lambda: rt.render(W, H, TIME),
                     lambda: rt.upload_scene(cornell),
                     lambda: rt.mandelbrot(rvcp_amd.mandelbrot.Config().push_constant(), 16, 16)):
            with pytest.raises(rvcp_amd.abi.RvcpError) as e:
                call()
            assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID
            assert "in flight" in str(e.value)
        st = rt.wait()
        rt.render_async(push, W, H, b.data_ptr(), stream=s2.cuda_stream)
        st2 = rt.wait()
        torch.cuda.synchronize()
    for t in (a, b):
        assert np.array_equal(t.cpu().numpy().view(np.uint8).reshape(H, W, 4), ref)
    assert int(st["traversals"]) == int(st2["traversals"])


def test_destroy_with_frame_pending(cornell):
    """rvcp_destroy waits for a frame still in flight on the caller's stream before it frees
    the buffers that frame reads."""
    torch = pytest.importorskip("torch")
    W, H = 256, 256
    a = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    rt = rvcp_amd.RayTracer(spp=8)
    rt.upload_scene(cornell)
    rt.render_async(cornell.push_constant(TIME), W, H, a.data_ptr(), stream=s.cuda_stream)
    rt.close()
    torch.cuda.synchronize()
    with rvcp_amd.RayTracer(spp=8) as rt2:
        rt2.upload_scene(cornell)
        ref = rt2.render(W, H, TIME)
    assert np.array_equal(a.cpu().numpy().view(np.uint8).reshape(H, W, 4), ref)


@pytest.mark.parametrize("W,H", [(128, 96), (77, 45)])
def test_rccl_gather_world1(cornell, W, H):
    """rvcp_rccl_init + rvcp_render_shard_async + rvcp_gather_frame_async (ncclGather to
    rank 0 and device assembly) with one rank == the direct render."""
    torch = pytest.importorskip("torch")
    uid = rvcp_amd.rccl_unique_id()
    assert len(uid) == 128
    stream = torch.cuda.current_stream().cuda_stream
    with rvcp_amd.RayTracer(spp=2) as rt:
        rt.upload_scene(cornell)
        ref = rt.render(W, H, TIME)
        rt.rccl_init(uid, 1, 0)
        slot = rvcp_amd.shard_rows(H, 0, 1)
        shard = torch.zeros((slot, W), dtype=torch.int32, device="cuda")
        gathered = torch.zeros((1, slot, W), dtype=torch.int32, device="cuda")
        frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        for _ in range(2):
            rt.render_shard_async(cornell.push_constant(TIME), W, H, 0, 1, shard.data_ptr(), stream=stream)
            rt.gather_frame_async(shard.data_ptr(), W, H, gathered.data_ptr(), frame.data_ptr(), stream=stream)
            rt.sync_stats()
        torch.cuda.synchronize()
        with pytest.raises(rvcp_amd.abi.RvcpError):
            rt.rccl_init(uid, 1, 0)                     # one communicator per context
    assert np.array_equal(frame.cpu().numpy().view(np.uint8).reshape(H, W, 4), ref)


def test_two_frames_in_flight_with_two_communicators(cornell):
    """bench.py's frames-in-flight pattern: two contexts, each with its own RCCL communicator
    and its own stream, render and gather alternate frames without a host sync between
    enqueues; every assembled frame equals the direct render."""
    torch = pytest.importorskip("torch")
    W, H = 160, 72
    rts = [rvcp_amd.RayTracer(spp=3) for _ in range(2)]
    try:
        for rt in rts:
            rt.upload_scene(cornell)
            rt.rccl_init(rvcp_amd.rccl_unique_id(), 1, 0)
        ref = rts[0].render(W, H, TIME)
        slot = rvcp_amd.shard_rows(H, 0, 1)
        shards = [torch.zeros((slot, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        gath = [torch.zeros((1, slot, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        frames = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        pending = [False, False]
        push = cornell.push_constant(TIME)
        for f in range(6):
            i = f % 2
            if pending[i]:
                rts[i].sync_stats()
            rts[i].render_shard_async(push, W, H, 0, 1, shards[i].data_ptr())
            rts[i].gather_frame_async(shards[i].data_ptr(), W, H, gath[i].data_ptr(),
                                      frames[i].data_ptr())
            pending[i] = True
        for i in range(2):
            rts[i].sync_stats()
        torch.cuda.synchronize()
        for fr in frames:
            assert np.array_equal(fr.cpu().numpy().view(np.uint8).reshape(H, W, 4), ref)
    finally:
        for rt in rts:
            rt.close()


def test_gather_without_communicator(cornell):
    torch = pytest.importorskip("torch")
    d = torch.zeros(64, dtype=torch.int32, device="cuda")
    with rvcp_amd.RayTracer(spp=1) as rt:
        with pytest.raises(rvcp_amd.abi.RvcpError) as e:
            rt.gather_frame_async(d.data_ptr(), 8, 8, d.data_ptr(), d.data_ptr())
        assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID


def test_gather_checks_the_rendered_shard(cornell):
    """rvcp_gather_frame_async refuses to gather after a render of another shard or frame
    size (rank 0 would assemble a scrambled frame); rvcp_gather_wait reports the gather's
    device time and fails when no gather is in flight."""
    torch = pytest.importorskip("torch")
    W, H = 64, 40
    slot = rvcp_amd.shard_rows(H, 0, 1)
    shard = torch.zeros((slot, W), dtype=torch.int32, device="cuda")
    gathered = torch.zeros((1, slot, W), dtype=torch.int32, device="cuda")
    frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    push = cornell.push_constant(TIME)
    with rvcp_amd.RayTracer(spp=1) as rt:
        rt.upload_scene(cornell)
        rt.rccl_init(rvcp_amd.rccl_unique_id(), 1, 0)
        with pytest.raises(rvcp_amd.abi.RvcpError) as e:
            rt.gather_wait()
        assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID
        rt.render_shard_async(push, W, H, 0, 2, shard.data_ptr())        # shard 0 of 2
        rt.sync_stats()
        with pytest.raises(rvcp_amd.abi.RvcpError) as e:
            rt.gather_frame_async(shard.data_ptr(), W, H, gathered.data_ptr(), frame.data_ptr())
        assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID
        big = torch.zeros((H + 8, W), dtype=torch.int32, device="cuda")
        rt.render_shard_async(push, W, H + 8, 0, 1, big.data_ptr())      # another frame size
        rt.sync_stats()
        with pytest.raises(rvcp_amd.abi.RvcpError):
            rt.gather_frame_async(shard.data_ptr(), W, H, gathered.data_ptr(), frame.data_ptr())
        rt.render_shard_async(push, W, H, 0, 1, shard.data_ptr())
        rt.gather_frame_async(shard.data_ptr(), W, H, gathered.data_ptr(), frame.data_ptr())
        rt.sync_stats()
        g_ms, f_ms = rt.gather_wait()
        assert 0.0 <= g_ms <= f_ms
        ref = rt.render(W, H, TIME)
    assert np.array_equal(frame.cpu().numpy().view(np.uint8).reshape(H, W, 4), ref)


def test_stats_report_schedule(cornell):
    """rvcp_stats_t.kernel_variant names the schedule that ran (bench.py picks the rocprof
    kernel name from it)."""
    spec = rvcp_amd.abi.VARIANT_SPECIALIZED
    with rvcp_amd.RayTracer(spp=30) as rt:          # Cornell: the scene-specialised kernels
        rt.upload_scene(cornell)
        rt.render(1024, 1024, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 3 | spec      # 5 waves beats 6 here
        rt.render(64, 64, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 3 | spec
    with rvcp_amd.RayTracer(spp=64) as rt:          # C4's frame (>= 256 Msamples): 6 waves
        rt.upload_scene(cornell)
        rt.render(2048, 2048, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 6 | spec
    with rvcp_amd.RayTracer(spp=30, specialize=rvcp_amd.abi.SPECIALIZE_OFF) as rt:
        rt.upload_scene(cornell)
        rt.render(1024, 1024, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 6
        rt.render(64, 64, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 3
    with rvcp_amd.RayTracer(spp=1) as rt:
        rt.upload_scene(rvcp_amd.scene.with_random_triangles(cornell, 300))
        rt.render(32, 32, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 5         # large mesh, small frame
        rt.render(1024, 512, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 10        # large mesh, >= 512 Ki samples
    with rvcp_amd.RayTracer(spp=1) as rt:
        rt.upload_scene(rvcp_amd.scene.with_random_triangles(cornell, 40))     # 72 faces
        rt.render(64, 64, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 3
        rt.render(1024, 512, TIME)
        assert int(rt.last_stats["kernel_variant"]) == 10
    with rvcp_amd.RayTracer(spp=2, integrator=1) as rt:                         # mode 2
        rt.upload_scene(rvcp_amd.scene.sphere_scene())
        rt.render(64, 64, TIME)
        v = int(rt.last_stats["kernel_variant"])
        assert v == 8 | spec and rvcp_amd.abi.KERNEL_NAMES[v] == "rvcp_spec_legacy_kernel"


@pytest.mark.parametrize("integrator,spp", [(0, 6), (1, 3)])
def test_grid_waves_per_simd_keeps_the_frame(cornell, integrator, spp):
    """rvcp_config_t.grid_waves_per_simd only sizes the persistent grid of a frame's path
    kernel (1 wave per SIMD, the 3 bench.py uses for C3-sized frames, more than the occupancy):
    every frame and the traversal count equal the full-grid render, in both integrators."""
    W, H = 320, 200
    outs = []
    for g in (0, 1, 3, 64):
        with rvcp_amd.RayTracer(spp=spp, integrator=integrator, grid_waves_per_simd=g) as rt:
            rt.upload_scene(cornell)
            img = rt.render(W, H, TIME)
            outs.append((img, int(rt.last_stats["traversals"])))
    for img, trav in outs[1:]:
        assert np.array_equal(img, outs[0][0])
        assert trav == outs[0][1]


def test_primary_t_range_below_2_24_is_enforced(cornell):
    """The shader writes a miss as t_max + 1 and tests t > t_max (:287, :424): at a primary-ray
    t_max (camera t_far x t_coef) of 2^24 or more the +1 is lost and the reference takes a miss
    for a hit.  Such a camera is refused (RVCP_E_INVALID) like rvcp_config_t.ray_t_max >= 2^24;
    the largest accepted t_far renders the oracle's frame (found by tests/test_gpu_spec_fuzz.py)."""
    import oracle as O
    from conftest import scene_arrays
    cam = cornell.camera
    with rvcp_amd.RayTracer(spp=1) as rt:
        for t_far, ok in [(2.0 ** 24, False), (1.5e7, False), (float("inf"), False),
                          (float("nan"), False), (1.0e7, True)]:
            sc = rvcp_amd.Scene(rvcp_amd.Camera.new(cam.position, cam.position + cam.forward,
                                                    cam.t_near, t_far, cam.vertical_fov, 1.0, 1.0),
                                cornell.materials, [], cornell.mesh)
            rt.upload_scene(sc)
            if not ok:
                with pytest.raises(rvcp_amd.abi.RvcpError) as e:
                    rt.render(64, 48, 123.0)
                assert e.value.code == rvcp_amd.abi.RVCP_E_INVALID and "2^24" in str(e.value)
            else:
                rgba = rt.render(64, 48, 123.0)
                _, o_rgba, _ = O.render(scene_arrays(sc), sc.push_constant(123.0),
                                        rvcp_amd.abi.make_config(spp=1), 64, 48)
                assert np.array_equal(rgba, o_rgba)
