#!/usr/bin/env python3
"""Rank 0's share of an N-GPU job, timed on ONE GPU (the budget for >= 7x at 8).

At N ranks, rank 0 renders shard 0 of the frame (every N-th 8-row stripe: the largest shard)
with bench.py's pipeline for that shard (bench.auto_pipeline: frames in flight, grid, frames
per launch) and bench.CallSchedule's call order.  This renders that shard alone on one GPU for
each N and reports ms per frame and the speedup (strong) or aggregate rate (weak) the N-rank
job would reach if every rank ran at this rate.

  --workload c4 (default): the 2048^2 SPP=64 frame sharded over N (strong scaling, bench.py's
                 N>1 default); speedup_if_alone = one-GPU frame ms / share ms.
  --workload c3: the weak-scaling frame, side round8(1024 sqrt(N)) at SPP=30 (bench.py
                 --workload c3 at N>1); efficiency_if_alone = share rate / one-GPU C3 rate.
  --gather:      each context also issues, per frame, the rvcp_gather_frame_async bench.py's
                 enqueue() issues at N>1 (bench.py: gather on the context's high-priority
                 gather stream, joined to the render by events; assembly of the N-slot frame on
                 rank 0) -- over a world-1 RCCL communicator attached with world = N, rank = 0
                 (rvcp_rccl_attach takes the caller's world / rank), so that rank 0's streams,
                 hardware queues, events and assembly run as at N; what a one-GPU box cannot
                 show is the N-1 peers' shards arriving over xGMI (N-1 x 4 B x the share's pixels,
                 14 MB per C4 frame at N = 8) and the peers' own jitter.
The hardware queues are the process's (GPU_MAX_HW_QUEUES as set, else HIP's default of 4; the
box runs 4): no override here.

  python tools/rank_share.py [--workload c4|c3] [--ns 1,2,4,8] [--gather] [--frames 24]
"""
import argparse
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import rvcp_amd  # noqa: E402
import bench  # noqa: E402


def frame_of(workload, n):
    """(W, H, spp) of bench.py's frame at n ranks."""
    if workload == "c4":
        return 2048, 2048, 64
    side = 1024 if n == 1 else int(round(1024 * math.sqrt(n) / 8.0)) * 8
    return side, side, 30


def time_share(torch, rts, sc, W, H, rank, world, frames, batch, gather):
    """ms per frame of `frames` timed frames (after a warm-up of at least one full batch per
    context), the call schedule of bench.py (bench.CallSchedule: frames round-robin over the
    contexts, each with its own time seed); with `gather`, bench.py's per-frame gather."""
    fif = len(rts)
    slot = rvcp_amd.shard_rows(H, 0, world)
    shard_bufs = [torch.zeros((batch, slot, W), dtype=torch.int32, device="cuda") for _ in range(fif)]
    frames_buf = [torch.zeros((batch, H, W), dtype=torch.int32, device="cuda") if gather else None
                  for _ in range(fif)]
    gat = [torch.zeros((world, slot, W), dtype=torch.int32, device="cuda") if gather else None
           for _ in range(fif)]
    gather_ms = []

    def enqueue(i, pushes, nb):
        r = rts[i]
        if batch == 1:
            r.render_shard_async(pushes[0], W, H, rank, world, shard_bufs[i].data_ptr())
        else:
            r.render_frames_async(pushes, W, H, rank, world, shard_bufs[i].data_ptr())
        if gather:      # bench.py enqueue(): one gather per frame, behind the render
            for j in range(nb):
                r.gather_frame_async(shard_bufs[i][j].data_ptr(), W, H, gat[i].data_ptr(),
                                     frames_buf[i][j].data_ptr())

    def finish(i, nb):
        st = rts[i].sync_stats()
        if gather:
            gather_ms.append(rts[i].gather_wait()[0])
        return st

    sched = bench.CallSchedule(fif, batch, enqueue, finish, lambda t: sc.push_constant(t))
    warm = -(-max(3, fif * batch) // batch) * batch
    sched.run(warm)
    gather_ms.clear()
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    stats = sched.run(frames)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1000.0 / frames
    kern = sum(float(s["main_kernel_ms"]) for s in stats) / len(stats)
    return wall, kern, (sum(gather_ms) / len(gather_ms) if gather_ms else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=["c4", "c3"])
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--gather", action="store_true")
    a = ap.parse_args()
    import torch
    sys.path.insert(0, HERE)
    import rccl_comm
    hwq = os.environ.get("GPU_MAX_HW_QUEUES", "4")
    sc = rvcp_amd.Scene.default()
    one = None
    for n in [int(x) for x in a.ns.split(",")]:
        W, H, spp = frame_of(a.workload, n)
        rows = rvcp_amd.shard_rows(H, 0, n)
        fif, grid, batch = bench.auto_pipeline(W * rows, spp, False, True, hwq, "none", a.frames)
        grid = grid if fif >= 3 else 0
        rts = [rvcp_amd.RayTracer(spp=spp, grid_waves_per_simd=grid) for _ in range(fif)]
        for r in rts:
            r.upload_scene(sc)
        gather = a.gather and n > 1
        comms = []
        if gather:
            for r in rts:
                comms.append(rccl_comm.make_comm(1, 0))
                r.rccl_attach(comms[-1], n, 0)
        wall, kern, gms = time_share(torch, rts, sc, W, H, 0, n, a.frames, batch, gather)
        share = W * rows * spp
        out = dict(workload=a.workload, n=n, frame=f"{W}x{H} spp={spp}", rows=rows, fif=fif,
                   grid=grid, batch=batch, gather=gather, gpu_max_hw_queues=hwq,
                   ms_per_frame=round(wall, 3), path_kernel_ms=round(kern, 3),
                   gather_ms=None if gms is None else round(gms, 4),
                   msamples_s=round(share / wall / 1e3, 1))
        if n == 1:
            one = (wall, share / wall)
        if one is not None and a.workload == "c4":
            out["speedup_if_alone"] = round(one[0] / wall, 3)
        elif one is not None:
            out["aggregate_msamples_s_if_alone"] = round(n * share / wall / 1e3, 1)
            out["efficiency_if_alone"] = round((share / wall) / one[1], 3)
        print(json.dumps(out), flush=True)
        for r in rts:
            r.close()
        torch.cuda.synchronize()
        for c in comms:
            rccl_comm.destroy_comm(c)


if __name__ == "__main__":
    main()
