"""The off-axis workload (bench.py --workload c3rot): the Cornell box turned
with its camera by a rotation about three axes (scene.rotated_scene).  No triangle keeps an
exact-zero component for the scene-specialised scan to drop, and the frame has the statistics
of the original (same traversals per sample within a few percent), so its rate measures the
specialised scan without the axis-aligned benchmark's zeros.  (CPU: oracle only.)"""
import numpy as np

import oracle as O
import rvcp_amd
from rvcp_amd import scene as S
from conftest import scene_arrays


def tri_parts(sc):
    v = sc.mesh.aligned_vertices()["position"][:, :3]
    f = sc.mesh.aligned_faces()["vertices"]
    v0 = v[f[:, 0]]
    return v0, (v[f[:, 1]] - v0).astype(np.float32), (v[f[:, 2]] - v0).astype(np.float32)


def test_no_exact_zero_components():
    base, rot = rvcp_amd.Scene.default(), S.rotated_scene(rvcp_amd.Scene.default())
    assert sum(int((p == 0).sum()) for p in tri_parts(base)) > 80      # the axis-aligned box
    for p in tri_parts(rot):
        assert not (p == 0).any()
    n = rot.mesh.aligned_vertices()["normal"][:, :3]
    assert np.allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-6)
    assert len(rot.mesh.aligned_faces()) == 32 and len(rot.luminous_face_ids()) == 2


def test_rotated_frame_statistics():
    """Oracle at 96^2 SPP=4: the turned box shows the same scene -- traversals per sample
    and the mean brightness of the frame within a few percent of the original's."""
    base, rot = rvcp_amd.Scene.default(), S.rotated_scene(rvcp_amd.Scene.default())
    cfg = rvcp_amd.abi.make_config(spp=4)
    res = []
    for sc in (base, rot):
        lin, rgba, trav = O.render(scene_arrays(sc), sc.push_constant(123.0), cfg, 96, 96)
        res.append((trav / (96 * 96 * 4), float(rgba[..., :3].mean())))
    (t0, m0), (t1, m1) = res
    assert abs(t1 / t0 - 1.0) < 0.08, (t0, t1)
    assert abs(m1 / m0 - 1.0) < 0.08, (m0, m1)
