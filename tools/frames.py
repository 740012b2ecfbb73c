#!/usr/bin/env python3
"""Render N frames of a workload with one kernel variant (profiling driver for rocprofv3).

  python tools/frames.py [--variant V] [--frames N] [--size S] [--spp P] [--tris T]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rvcp_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=30)
    ap.add_argument("--tris", type=int, default=0)
    ap.add_argument("--integrator", type=int, default=0)
    ap.add_argument("--accel", type=int, default=0)
    ap.add_argument("--scene", default="cornell", choices=["cornell", "spheres"])
    ap.add_argument("--generic", action="store_true", help="specialize = OFF (generic scan)")
    ap.add_argument("--grid", type=int, default=0, help="rvcp_config_t.grid_waves_per_simd (0: full)")
    a = ap.parse_args()
    sc = rvcp_amd.Scene.default() if a.scene == "cornell" else rvcp_amd.scene.sphere_scene()
    if a.tris:
        sc = rvcp_amd.scene.with_random_triangles(sc, a.tris)
    with rvcp_amd.RayTracer(spp=a.spp, kernel_variant=a.variant, integrator=a.integrator,
                            accel=a.accel, specialize=1 if a.generic else 0,
                            grid_waves_per_simd=a.grid) as rt:
        rt.upload_scene(sc)
        for _ in range(a.frames):
            rt.render(a.size, a.size, 123.0)
            st = rt.last_stats
            print(json.dumps({"variant": a.variant, "integrator": a.integrator, "grid": a.grid,
                              "traversals": int(st["traversals"]), "kernel_ms": round(float(st["kernel_ms"]), 3),
                              "executed": int(st["traversals_executed"]),
                              "wave_iterations": int(st["wave_iterations"]),
                              # path-kernel rays per ray slot (2 per lane per wave iteration;
                              # the pre-pass traced one primary ray per pixel)
                              "slot_util": round((int(st["traversals_executed"]) - a.size * a.size)
                                                 / max(1, 128 * int(st["wave_iterations"])), 4)
                              if a.integrator == 0 else None}), flush=True)


if __name__ == "__main__":
    main()
