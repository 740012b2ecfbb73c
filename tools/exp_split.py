#!/usr/bin/env python3
"""Experiment: split C3 frame time into scan vs shading by duplicating every face.

Duplicated faces give bit-identical images (ties keep the later, identical face), so the
traversal count is unchanged and only the per-traversal scan grows with F:
frame(F) = shade + F * scan_per_face.  Also prints lane utilisation of the scan."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rvcp_amd  # noqa: E402


def dup_scene(sc, k):
    faces = sc.mesh.aligned_faces()
    # keep the light faces first (ids 0, 1) so the luminous-id table is unchanged
    f = np.concatenate([faces] + [faces[2:]] * (k - 1)) if k > 1 else faces
    mesh = rvcp_amd.scene.ArrayMesh(sc.mesh.aligned_vertices(), f)
    return rvcp_amd.Scene(sc.camera, sc.materials, [], mesh)


def main():
    variant = int(os.environ.get("RVCP_KERNEL_VARIANT", "0"))
    base = rvcp_amd.Scene.default()
    ref = None
    out = []
    for k in (1, 2, 3, 5):
        sc = dup_scene(base, k)
        cfg = rvcp_amd.abi.make_config(spp=30)
        cfg["kernel_variant"] = variant
        with rvcp_amd.RayTracer(cfg) as rt:
            rt.upload_scene(sc)
            img = rt.render(1024, 1024, 123.0)
            ms = []
            for _ in range(5):
                rt.render(1024, 1024, 123.0)
                ms.append(float(rt.last_stats["kernel_ms"]))
            st = rt.last_stats
        if ref is None:
            ref = img
        util = int(st["traversals_executed"]) / (64.0 * max(1, int(st["wave_iterations"])))
        out.append(dict(F=int(st["faces"]), kernel_ms=round(float(np.median(ms)), 3),
                        same_image=bool(np.array_equal(img, ref)), lane_util=round(util, 4),
                        wave_iters=int(st["wave_iterations"]),
                        executed=int(st["traversals_executed"])))
        print(json.dumps(out[-1]), flush=True)
    F = np.array([o["F"] for o in out], float)
    T = np.array([o["kernel_ms"] for o in out], float)
    b, a = np.polyfit(F, T, 1)
    print(json.dumps({"fit_shade_ms": round(a, 3), "fit_scan_ms_per_face": round(b, 4),
                      "scan_share_at_F32": round(b * 32 / (a + b * 32), 3)}))


if __name__ == "__main__":
    main()
