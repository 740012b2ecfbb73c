"""Generate tests/golden/oracle_frames.npz: small frames rendered by the CPU oracle
(oracle/rvcp_oracle.c), committed so that

* the oracle itself is pinned against regressions (tests/test_golden_frames.py, CPU), and
* the HIP kernel is checked against committed vectors, not only against a live oracle
  (tests/test_golden_frames.py, GPU).

The reference ships no golden vectors; these are the oracle's outputs for the
cases SURVEY.md §8(c) lists (64² SPP=4 and the C1 config 128² SPP=1, time 123.0) plus one
integrator-mode-2 frame of the sphere room.  Each case stores the linear RGB (float32), the
RGBA8 frame and the reference-algorithm traversal count, and the SHA-256 of the scene
buffers it was rendered from.

  python tests/golden/make_oracle_fixtures.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
import rvcp_amd  # noqa: E402

OUT = os.path.join(HERE, "oracle_frames.npz")

# name -> (scene factory, config kwargs, W, H, time)
CASES = {
    "cornell_64sq_spp4": ("cornell", dict(spp=4), 64, 64, 123.0),
    "c1_cornell_128sq_spp1": ("cornell", dict(spp=1), 128, 128, 123.0),
    "cornell_48x40_quirk_off": ("cornell", dict(spp=3, lum_id_std140_quirk=0), 48, 40, 7.5),
    "spheres_mode2_64sq_spp5": ("spheres", dict(integrator=1), 64, 64, 3.25),
}


def scene_of(name):
    return rvcp_amd.Scene.default() if name == "cornell" else rvcp_amd.scene.sphere_scene()


def arrays_of(sc):
    return dict(materials=sc.aligned_materials(), vertices=sc.mesh.aligned_vertices(),
                faces=sc.mesh.aligned_faces(), lum_face_ids=sc.luminous_face_ids(),
                spheres=sc.aligned_spheres())


def scene_digest(arrays):
    h = hashlib.sha256()
    for k in ("materials", "vertices", "faces", "lum_face_ids", "spheres"):
        h.update(np.ascontiguousarray(arrays[k]).tobytes())
    return h.hexdigest()


def render(case):
    scn, kw, W, H, t = CASES[case]
    sc = scene_of(scn)
    arrays = arrays_of(sc)
    cfg = rvcp_amd.abi.make_config(**kw)
    lin, rgba, trav = O.render(arrays, sc.push_constant(t), cfg, W, H)
    return sc, cfg, arrays, lin, rgba, trav


def main():
    out = {}
    for case in CASES:
        _, _, arrays, lin, rgba, trav = render(case)
        out[case + "/linear"] = lin
        out[case + "/rgba"] = rgba
        out[case + "/traversals"] = np.array(trav, dtype=np.uint64)
        out[case + "/scene_sha256"] = np.array(scene_digest(arrays))
        print(case, lin.shape, trav, scene_digest(arrays)[:16])
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
