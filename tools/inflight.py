#!/usr/bin/env python3
"""Frames in flight: K frames of one workload rendered (a) one at a time
(enqueue, wait) and (b) with two contexts on two streams, the next frame enqueued before the
previous one is waited for, so that a frame's pre-pass and path kernel can fill the CUs the
previous frame's tail leaves idle.  Prints ms per frame of both and checks the frames equal.

  python tools/inflight.py [--size 1024] [--spp 30] [--frames 40]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rvcp_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=30)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--ctx-streams", action="store_true",
                    help="render on each context's own stream instead of two torch streams")
    a = ap.parse_args()
    import torch
    W = H = a.size
    sc = rvcp_amd.Scene.default()
    push = sc.push_constant(123.0)
    rts = [rvcp_amd.RayTracer(spp=a.spp) for _ in range(2)]
    for rt in rts:
        rt.upload_scene(sc)
    bufs = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    sid = [0, 0] if a.ctx_streams else [s.cuda_stream for s in streams]
    for _ in range(3):                                     # warm-up
        rts[0].render_async(push, W, H, bufs[0].data_ptr(), stream=sid[0])
        rts[0].wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        rts[0].render_async(push, W, H, bufs[0].data_ptr(), stream=sid[0])
        rts[0].wait()
    torch.cuda.synchronize()
    serial = (time.perf_counter() - t0) * 1000.0 / a.frames
    ref = bufs[0].clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pending = [False, False]
    for f in range(a.frames):
        i = f % 2
        if pending[i]:
            rts[i].wait()
        rts[i].render_async(push, W, H, bufs[i].data_ptr(), stream=sid[i])
        pending[i] = True
    for i in range(2):
        if pending[i]:
            rts[i].wait()
    torch.cuda.synchronize()
    inflight = (time.perf_counter() - t0) * 1000.0 / a.frames
    same = bool(torch.equal(bufs[0], ref) and torch.equal(bufs[1], ref))
    print(f"queues {os.environ.get('GPU_MAX_HW_QUEUES', '-')} ctx-streams {a.ctx_streams} size {W} spp {a.spp}: one at a time {serial:.3f} ms/frame, two in flight "
          f"{inflight:.3f} ms/frame, frames equal {same}", flush=True)
    for rt in rts:
        rt.close()


if __name__ == "__main__":
    main()
