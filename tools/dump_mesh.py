#!/usr/bin/env python3
"""Write a scene's triangles as raw float32 [n][3][3] (input of tools/bvh4_check.cpp).

  python tools/dump_mesh.py OUT.bin [--tris 100000]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rvcp_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--tris", type=int, default=100000)
a = ap.parse_args()
sc = rvcp_amd.scene.with_random_triangles(rvcp_amd.Scene.default(), a.tris)
v = sc.mesh.aligned_vertices()
f = sc.mesh.aligned_faces()
v["position"][:, :3][f["vertices"]].astype(np.float32).tofile(a.out)
