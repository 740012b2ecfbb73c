"""rvcp_render_frames_async (include/rvcp.h): a batch of frames in one path kernel is, frame
by frame, bit-identical to rendering each frame alone -- with a different time seed per frame
(the reference's per-frame `time`, vulkan.rs:418-421), for whole frames and for shards whose
rows differ (the padded slot layout), on the schedules that share one surface list; the stats
cover the whole batch; integrator mode 2 batches too (per-frame cameras); the schedules
without a pre-pass refuse a batch."""
import numpy as np
import pytest

import rvcp_amd

pytestmark = pytest.mark.gpu
TIMES = (123.0, 7.5, 123.0, 301.25)


def _single(rt, sc, W, H, k, n, t, torch):
    rows = rvcp_amd.shard_rows(H, k, n)
    out = torch.zeros((rows, W), dtype=torch.int32, device="cuda")
    lin = torch.zeros((rows, W, 3), dtype=torch.float32, device="cuda")
    rt.render_shard_async(sc.push_constant(t), W, H, k, n, out.data_ptr(), lin.data_ptr())
    st = rt.sync_stats()
    torch.cuda.synchronize()
    return out.cpu().numpy(), lin.cpu().numpy(), st


@pytest.mark.parametrize("W,H,spp,k,n,variant", [
    (160, 96, 5, 0, 1, 0),        # whole frames, the automatic (specialised) schedule
    (200, 83, 4, 2, 3, 0),        # shard 2 of 3 has fewer rows than the slot: padded layout
    (200, 83, 4, 0, 3, 0),
    (96, 64, 3, 0, 1, 4),         # LDS-tiled scan
    (96, 64, 3, 1, 2, 10),        # tiled + workgroup ray pool
    (128, 72, 3, 0, 1, 3),        # generic schedule 3
])
def test_batch_equals_single_frames(cornell, W, H, spp, k, n, variant):
    torch = pytest.importorskip("torch")
    kw = dict(spp=spp)
    if variant:
        kw["kernel_variant"] = variant
        if variant == 3:
            kw["specialize"] = rvcp_amd.abi.SPECIALIZE_OFF
    slot = rvcp_amd.shard_rows(H, 0, n)
    rows = rvcp_amd.shard_rows(H, k, n)
    with rvcp_amd.RayTracer(**kw) as rt:
        rt.upload_scene(cornell)
        singles = [_single(rt, cornell, W, H, k, n, t, torch) for t in TIMES]
        out = torch.zeros((len(TIMES), slot, W), dtype=torch.int32, device="cuda")
        lin = torch.zeros((len(TIMES), slot, W, 3), dtype=torch.float32, device="cuda")
        rt.render_frames_async([cornell.push_constant(t) for t in TIMES], W, H, k, n,
                               out.data_ptr(), lin.data_ptr())
        st = rt.sync_stats()
        torch.cuda.synchronize()
    out, lin = out.cpu().numpy(), lin.cpu().numpy()
    for f, (o1, l1, _) in enumerate(singles):
        assert np.array_equal(out[f, :rows], o1), f
        assert np.array_equal(lin[f, :rows].view(np.uint32), l1.view(np.uint32)), f
    assert not np.array_equal(singles[0][0], singles[1][0])      # the seeds differ
    assert int(st["samples"]) == len(TIMES) * rows * W * spp
    assert int(st["traversals"]) == sum(int(s["traversals"]) for _, _, s in singles)
    assert int(st["traversals_executed"]) == sum(int(s["traversals_executed"]) for _, _, s in singles)


def test_batch_bvh_equals_single_frames(cornell):
    torch = pytest.importorskip("torch")
    sc = rvcp_amd.scene.with_random_triangles(cornell, 300)
    W, H = 96, 80
    with rvcp_amd.RayTracer(spp=3, accel=rvcp_amd.abi.ACCEL_BVH) as rt:
        rt.upload_scene(sc)
        singles = [_single(rt, sc, W, H, 0, 1, t, torch)[0] for t in TIMES[:3]]
        out = torch.zeros((3, H, W), dtype=torch.int32, device="cuda")
        rt.render_frames_async([sc.push_constant(t) for t in TIMES[:3]], W, H, 0, 1, out.data_ptr())
        rt.sync_stats()
        torch.cuda.synchronize()
    for f in range(3):
        assert np.array_equal(out[f].cpu().numpy(), singles[f]), f


@pytest.mark.parametrize("scene,W,H,spp,k,n,spec", [
    ("spheres", 128, 96, 3, 0, 1, 0),     # the sphere room, scene-specialised mode-2 kernel
    ("spheres", 128, 96, 3, 0, 1, 1),     # ... the generic one
    ("cornell", 150, 83, 4, 1, 3, 0),     # Cornell box, shard 1 of 3 (padded slots)
])
def test_mode2_batch_equals_single_frames(cornell, scene, W, H, spp, k, n, spec):
    """Integrator mode 2 (ray_tracer.comp) batches: one kernel queues the frames' pixels frame
    after frame, each frame with its own camera and time (FrameArgs::batch_cams); every frame
    equals its single render."""
    torch = pytest.importorskip("torch")
    sc = cornell if scene == "cornell" else rvcp_amd.scene.sphere_scene()
    slot = rvcp_amd.shard_rows(H, 0, n)
    rows = rvcp_amd.shard_rows(H, k, n)
    times = TIMES[:3]
    pushes = [sc.push_constant(t) for t in times]
    # a moved camera for the last frame: the batch carries per-frame cameras, not only times
    cam = pushes[2]["camera"]
    cam["position"][0] += 7.0
    with rvcp_amd.RayTracer(spp=spp, integrator=1, specialize=spec) as rt:
        rt.upload_scene(sc)
        singles = []
        for p in pushes:
            o = torch.zeros((rows, W), dtype=torch.int32, device="cuda")
            rt.render_shard_async(p, W, H, k, n, o.data_ptr())
            singles.append((o, rt.sync_stats()))
        out = torch.zeros((3, slot, W), dtype=torch.int32, device="cuda")
        rt.render_frames_async(pushes, W, H, k, n, out.data_ptr())
        st = rt.sync_stats()
        torch.cuda.synchronize()
    for f, (o, _) in enumerate(singles):
        assert np.array_equal(out[f, :rows].cpu().numpy(), o.cpu().numpy()), f
    assert not np.array_equal(singles[0][0].cpu().numpy(), singles[2][0].cpu().numpy())
    assert int(st["samples"]) == 3 * rows * W * spp
    assert int(st["traversals"]) == sum(int(x["traversals"]) for _, x in singles)


def test_batch_refused_where_unsupported(cornell):
    torch = pytest.importorskip("torch")
    out = torch.zeros((2, 32, 32), dtype=torch.int32, device="cuda")
    push = [cornell.push_constant(1.0), cornell.push_constant(2.0)]
    for kw in (dict(kernel_variant=2), dict(kernel_variant=1)):
        with rvcp_amd.RayTracer(spp=2, **kw) as rt:
            rt.upload_scene(cornell)
            with pytest.raises(rvcp_amd.abi.RvcpError) as e:
                rt.render_frames_async(push, 32, 32, 0, 1, out.data_ptr())
            assert e.value.code == rvcp_amd.abi.RVCP_E_UNSUPPORTED
            # a batch of one is rvcp_render_shard_async
            rt.render_frames_async(push[:1], 32, 32, 0, 1, out.data_ptr())
            rt.sync_stats()


def test_batch_with_rccl_gathers(cornell):
    """bench.py's N>1 pattern with batches, at world size 1: two contexts, each with its own
    communicator, alternate batches of 3 frames (different seeds) and gather every frame of a
    batch (one rvcp_gather_frame_async per frame, sharing the gather buffer in stream order);
    every assembled frame equals the direct render of its seed."""
    torch = pytest.importorskip("torch")
    W, H = 120, 64
    times = TIMES[:3]
    rts = [rvcp_amd.RayTracer(spp=3) for _ in range(2)]
    try:
        for rt in rts:
            rt.upload_scene(cornell)
            rt.rccl_init(rvcp_amd.rccl_unique_id(), 1, 0)
        refs = [rts[0].render(W, H, t) for t in times]
        slot = rvcp_amd.shard_rows(H, 0, 1)
        shards = [torch.zeros((3, slot, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        gath = [torch.zeros((1, slot, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        frames = [torch.zeros((3, H, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        pending = [False, False]
        pushes = [cornell.push_constant(t) for t in times]
        for c in range(5):
            i = c % 2
            if pending[i]:
                rts[i].sync_stats()
                rts[i].gather_wait()
            rts[i].render_frames_async(pushes, W, H, 0, 1, shards[i].data_ptr())
            for j in range(3):
                rts[i].gather_frame_async(shards[i][j].data_ptr(), W, H, gath[i].data_ptr(),
                                          frames[i][j].data_ptr())
            pending[i] = True
        for i in range(2):
            rts[i].sync_stats()
            rts[i].gather_wait()
        torch.cuda.synchronize()
        for fr in frames:
            for j in range(3):
                assert np.array_equal(fr[j].cpu().numpy().view(np.uint8).reshape(H, W, 4), refs[j]), j
    finally:
        for rt in rts:
            rt.close()


def test_eight_shard_batches_assemble(cornell):
    """The N=8 bench pattern with batches on one GPU: each of 8 shards renders a batch of 3
    frames (different seeds) in one call, the slots of each frame are gathered (here: copied
    into the gather layout) and assembled on the device; every assembled frame equals the
    1-shard render of its seed."""
    torch = pytest.importorskip("torch")
    W, H, n, spp = 160, 203, 8, 2
    times = TIMES[:3]
    pushes = [cornell.push_constant(t) for t in times]
    slot = rvcp_amd.shard_rows(H, 0, n)
    with rvcp_amd.RayTracer(spp=spp) as rt:
        rt.upload_scene(cornell)
        refs = [rt.render(W, H, t) for t in times]
        shards = torch.zeros((n, len(times), slot, W), dtype=torch.int32, device="cuda")
        for k in range(n):
            rt.render_frames_async(pushes, W, H, k, n, shards[k].data_ptr())
            rt.sync_stats()
        frames = torch.zeros((len(times), H, W), dtype=torch.int32, device="cuda")
        for j in range(len(times)):
            gathered = shards[:, j].contiguous()               # (n, slot, W): the gather layout
            rt.assemble_frame_async(gathered.data_ptr(), slot, W, H, n, frames[j].data_ptr())
        torch.cuda.synchronize()
    for j in range(len(times)):
        assert np.array_equal(frames[j].cpu().numpy().view(np.uint8).reshape(H, W, 4), refs[j]), j
