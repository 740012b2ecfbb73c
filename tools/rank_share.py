#!/usr/bin/env python3
"""Per-rank share of the N-GPU C4 frame, timed on ONE GPU (DESIGN.md §5 budget for >= 7x).

At N ranks, rank 0 renders shard 0 of 2048^2 SPP=64 (every N-th 8-row stripe, the largest
shard) with `fif` frames in flight, exactly the loop bench.py times at N>1 minus the gather.
This renders that shard alone on one GPU for N = 1, 2, 4, 8 and prints ms per frame and the
speedup the N-rank job would reach if each rank ran alone at this rate (no gather, no
barrier jitter): the one-GPU side of the 8-GPU scaling line, measurable on a 1-GPU box.

  python tools/rank_share.py [--ns 1,2,4,8] [--fif 0] [--frames 24] [--schedule 0] [--grid 0]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import rvcp_amd  # noqa: E402
import bench  # noqa: E402


def time_share(torch, rts, push, W, H, rank, world, frames, batch=1):
    """ms per frame of `frames` frames (rounded up to whole batches of `batch` frames per
    rvcp_render_frames_async call), round-robin over the contexts."""
    fif = len(rts)
    slot = rvcp_amd.shard_rows(H, 0, world)
    bufs = [torch.zeros((batch, slot, W), dtype=torch.int32, device="cuda") for _ in range(fif)]
    pushes = [push] * batch

    def enqueue(i):
        if batch == 1:
            rts[i].render_shard_async(push, W, H, rank, world, bufs[i].data_ptr())
        else:
            rts[i].render_frames_async(pushes, W, H, rank, world, bufs[i].data_ptr())
    for i in range(fif):                                   # warm-up, one per context
        enqueue(i)
    for i in range(fif):
        rts[i].sync_stats()
    torch.cuda.synchronize()
    pending = [False] * fif
    kms = []
    calls = (frames + batch - 1) // batch
    frames = calls * batch
    t0 = time.perf_counter()
    for f in range(calls):
        i = f % fif
        if pending[i]:
            kms.append(float(rts[i].sync_stats()["main_kernel_ms"]))
        enqueue(i)
        pending[i] = True
    for i in range(fif):
        if pending[i]:
            kms.append(float(rts[i].sync_stats()["main_kernel_ms"]))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1000.0 / frames
    return wall, sum(kms) / len(kms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--fif", type=int, default=0, help="0 = bench.py's automatic choice")
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--schedule", type=int, default=0)
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per rvcp_render_frames_async call (1 = rvcp_render_shard_async, "
                         "0 = bench.py's automatic choice)")
    ap.add_argument("--grid", type=int, default=-1,
                    help="rvcp_config_t.grid_waves_per_simd (0 = every resident slot, -1 = "
                         "bench.py's automatic choice)")
    a = ap.parse_args()
    import torch
    sc = rvcp_amd.Scene.default()
    push = sc.push_constant(123.0)
    W = H = a.size
    kw = dict(spp=a.spp)
    if a.schedule:
        kw["kernel_variant"] = a.schedule
    one = None
    for n in [int(x) for x in a.ns.split(",")]:
        rank_samples = W * a.spp * rvcp_amd.shard_rows(H, 0, n)
        fif, grid, batch = bench.auto_pipeline(W * rvcp_amd.shard_rows(H, 0, n), a.spp, False, True,
                                               os.environ["GPU_MAX_HW_QUEUES"], "none", a.frames)
        fif = a.fif or fif
        grid = a.grid if a.grid >= 0 else (grid if fif >= 3 else 0)
        batch = a.batch or batch
        rts = [rvcp_amd.RayTracer(grid_waves_per_simd=grid, **kw) for _ in range(fif)]
        for r in rts:
            r.upload_scene(sc)
        wall, kern = time_share(torch, rts, push, W, H, 0, n, a.frames, batch)
        if n == 1:
            one = wall
        out = dict(n=n, rows=rvcp_amd.shard_rows(H, 0, n), fif=fif, grid=grid, batch=batch,
                   ms_per_frame=round(wall, 3),
                   path_kernel_ms=round(kern, 3),
                   msamples_s=round(rank_samples / wall / 1e3, 1))
        if one is not None:
            out["speedup_if_alone"] = round(one / wall, 3)
        print(json.dumps(out), flush=True)
        for r in rts:
            r.close()


if __name__ == "__main__":
    main()
