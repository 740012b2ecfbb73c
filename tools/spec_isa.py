#!/usr/bin/env python3
"""Compile the scene-specialised module (rvcp_jit.cpp's hipRTC build) for the Cornell box with
hipcc instead, to read its resource usage and ISA:  python tools/spec_isa.py [--out DIR]
Writes DIR/spec_scan.inc, DIR/spec.s and DIR/resource-usage.txt (default build/spec_isa).
--flags -DRVCP_SPEC_ISA_SKIP_ALL: the code left when every skippable block is skipped."""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rvcp_amd  # noqa: E402

CSRC = os.path.join(ROOT, "rvcp-real-time-path-tracer_amd", "csrc")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(CSRC, "build", "spec_isa"))
    ap.add_argument("--flags", default="")
    ap.add_argument("--scene", default="cornell", choices=["cornell", "spheres"])
    ap.add_argument("--legacy", action="store_true", help="the mode-2 module (RVCP_JIT_LEGACY)")
    ap.add_argument("--opts", type=int, default=0, help="generator options (rvcp_jit.h kScan*)")
    ap.add_argument("--no-sphere-literals", action="store_true",
                    help="--legacy: the module without the spheres as literals (the record loop)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    sc = rvcp_amd.Scene.default() if a.scene == "cornell" else rvcp_amd.scene.sphere_scene()
    V = sc.mesh.aligned_vertices()["position"][:, :3]
    F = sc.mesh.aligned_faces()["vertices"]
    p = V[F].astype(np.float32)
    rec = np.zeros(len(p), dtype=[("v0", "<f4", 3), ("e1", "<f4", 3), ("e2", "<f4", 3), ("pad", "<f4", 3)])
    rec["v0"], rec["e1"], rec["e2"] = p[:, 0], (p[:, 1] - p[:, 0]), (p[:, 2] - p[:, 0])
    L = rvcp_amd.abi.load()
    fn = L.rvcp_internal_jit_scan_source_opt
    fn.restype = ctypes.c_size_t
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    n = fn(rec.ctypes.data, len(rec), a.opts, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    fn(rec.ctypes.data, len(rec), a.opts, buf, n + 1)
    text = buf.value.decode()
    if a.legacy and not a.no_sphere_literals:      # the mode-2 module's sphere literals
        sph = np.ascontiguousarray(sc.aligned_spheres())
        fs = L.rvcp_internal_jit_sphere_source
        fs.restype = ctypes.c_size_t
        fs.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        m = fs(sph.ctypes.data, len(sph), None, 0)
        sb = ctypes.create_string_buffer(m + 1)
        fs(sph.ctypes.data, len(sph), sb, m + 1)
        text += sb.value.decode()
    inc = os.path.join(a.out, "spec_scan.inc")
    with open(inc, "w") as f:
        f.write(text)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math", "-fno-slp-vectorize",
           "-DRVCP_JIT", f'-DRVCP_SPEC_SCAN="{inc}"', "--cuda-device-only", "-S",
           "-o", os.path.join(a.out, "spec.s"), os.path.join(CSRC, "rvcp_kernels.hip"),
           "-Rpass-analysis=kernel-resource-usage"] + (["-DRVCP_JIT_LEGACY"] if a.legacy else []) + \
          a.flags.split()
    with open(os.path.join(a.out, "resource-usage.txt"), "w") as f:
        subprocess.run(cmd, check=True, stderr=f)
    out = open(os.path.join(a.out, "resource-usage.txt")).read()
    for line in out.splitlines():
        if any(k in line for k in ("Function Name", "VGPRs:", "Spill", "Occupancy", "LDS Size")):
            print(line.split("remark: ")[-1])


if __name__ == "__main__":
    main()
