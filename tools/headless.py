#!/usr/bin/env python3
"""Headless interactive loop (the reference's winit main loop without a window):

  python tools/headless.py [--scene cornell|spheres] [--integrator 0|1] [--size 384]
                           [--spp N] [--frames 60] [--script walk|orbit|none]
                           [--dump DIR] [--format ppm|png] [--fixed-dt 0.016]

Prints `Rendering FPS: n` once a second like ray_tracer.rs:80-87 and a JSON summary.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rvcp_amd  # noqa: E402


def script(name, frames, size):
    if name == "walk":          # forward, strafe right, rise
        third = max(1, frames // 3)
        return [(0, "key", ("W", True)), (third, "key", ("W", False)),
                (third, "key", ("D", True)), (2 * third, "key", ("D", False)),
                (2 * third, "key", ("E", True))]
    if name == "orbit":         # hold the right button and drag right
        return [(0, "mouse_right", (True,))] + [(i, "cursor", (size / 2 + 8, size / 2))
                                                for i in range(frames)]
    return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell", choices=["cornell", "spheres"])
    ap.add_argument("--integrator", type=int, default=None)
    ap.add_argument("--size", type=int, default=384)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--script", default="walk", choices=["walk", "orbit", "none"])
    ap.add_argument("--dump", default="")
    ap.add_argument("--format", default="ppm", choices=["ppm", "png"])
    ap.add_argument("--fixed-dt", type=float, default=None)
    a = ap.parse_args()
    integ = a.integrator if a.integrator is not None else (1 if a.scene == "spheres" else 0)
    sc = rvcp_amd.Scene.default() if a.scene == "cornell" else rvcp_amd.scene.sphere_scene()
    kw = dict(integrator=integ)
    if a.spp:
        kw["spp"] = a.spp
    with rvcp_amd.RayTracer(**kw) as rt:
        rt.upload_scene(sc)
        out = rvcp_amd.interactive.run_headless(
            rt, sc, a.frames, a.size, a.size, events=script(a.script, a.frames, a.size),
            fixed_dt=a.fixed_dt, dump_dir=a.dump or None, dump_format=a.format)
    ms = np.array(out["frame_ms"])
    print(json.dumps({"frames": a.frames, "size": a.size, "integrator": integ,
                      "median_frame_ms": round(float(np.median(ms)), 3),
                      "fps_reports": out["fps_reports"],
                      "final_camera": {"position": out["camera"].position.tolist(),
                                       "forward": out["camera"].forward.tolist()}}))


if __name__ == "__main__":
    main()
