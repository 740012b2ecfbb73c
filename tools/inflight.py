#!/usr/bin/env python3
"""Frames in flight: throughput of K frames rendered one after another (host waits for each)
versus with D frames in flight (D contexts, one stream each; frame i waits only for frame i-D),
and a bit-exact check of every in-flight frame against the sequential one.

  python tools/inflight.py [--size 1024] [--spp 30] [--frames 20] [--depth 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import rvcp_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=30)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--tris", type=int, default=0)
    a = ap.parse_args()
    sc = rvcp_amd.Scene.default()
    if a.tris:
        sc = rvcp_amd.scene.with_random_triangles(sc, a.tris)
    push = sc.push_constant(123.0)
    W = H = a.size
    dev = torch.device("cuda", 0)
    rts = [rvcp_amd.RayTracer(spp=a.spp) for _ in range(a.depth)]
    for rt in rts:
        rt.upload_scene(sc)
    streams = [torch.cuda.Stream(device=dev) for _ in range(a.depth)]
    outs = [torch.zeros((H, W), dtype=torch.int32, device=dev) for _ in range(a.depth)]

    def sequential(n):
        s = streams[0].cuda_stream
        for _ in range(n):
            rts[0].render_async(push, W, H, outs[0].data_ptr(), stream=s)
            rts[0].wait()

    def inflight(n):
        pending = []
        for i in range(n):
            k = i % a.depth
            if len(pending) == a.depth:
                rts[pending.pop(0)].wait()
            rts[k].render_async(push, W, H, outs[k].data_ptr(), stream=streams[k].cuda_stream)
            pending.append(k)
        while pending:
            rts[pending.pop(0)].wait()

    sequential(3)
    inflight(3)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("sequential", sequential), ("inflight", inflight), ("sequential2", sequential),
                     ("inflight2", inflight)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(a.frames)
        torch.cuda.synchronize()
        res[name + "_ms_per_frame"] = round((time.perf_counter() - t0) * 1000.0 / a.frames, 4)
    sequential(1)
    torch.cuda.synchronize()
    ref = outs[0].clone()
    inflight(a.depth)
    torch.cuda.synchronize()
    res["bitexact"] = all(bool(torch.equal(o, ref)) for o in outs)
    res.update(size=a.size, spp=a.spp, depth=a.depth, frames=a.frames, tris=a.tris)
    print(json.dumps(res), flush=True)
    for rt in rts:
        rt.close()


if __name__ == "__main__":
    main()
