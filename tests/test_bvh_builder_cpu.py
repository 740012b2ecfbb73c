"""Host-side BVH builder + 4-wide collapse (csrc/rvcp_bvh.cpp) on the CPU: tools/bvh4_check.cpp
links the product's builder, checks the traversal-stack bound, and compares the 4-wide
traversal's nearest hit with a brute-force scan on random rays through random meshes."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import rvcp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rvcp-real-time-path-tracer_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("bvh") / "bvh4_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(ROOT, "tools", "bvh4_check.cpp"),
                    os.path.join(CSRC, "rvcp_bvh.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("tris", [0, 3, 200, 5000])
def test_bvh4_matches_brute_force(checker, tmp_path, tris):
    sc = rvcp_amd.Scene.default()
    if tris:
        sc = rvcp_amd.scene.with_random_triangles(sc, tris)
    v = sc.mesh.aligned_vertices()
    f = sc.mesh.aligned_faces()
    mesh = str(tmp_path / "mesh.bin")
    v["position"][:, :3][f["vertices"]].astype(np.float32).tofile(mesh)
    r = subprocess.run([checker, mesh, "400"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0 of 400" in r.stdout


def test_bvh4_tiny_mesh(checker, tmp_path):
    """Fewer triangles than a leaf holds: the root is a leaf, no inner node."""
    p = np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 0, 1], [1, 0, 1], [0, 1, 1]]], np.float32)
    mesh = str(tmp_path / "tiny.bin")
    p.tofile(mesh)
    r = subprocess.run([checker, mesh, "100"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "nodes4=0" in r.stdout


def test_bvh4_builder_sanitized(tmp_path):
    """The builder + collapse under AddressSanitizer / UBSan (host code only), on a degenerate,
    a tiny and a random mesh: no report, and the same answers."""
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "bvh4_asan")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                        "-I", CSRC, os.path.join(ROOT, "tools", "bvh4_check.cpp"),
                        os.path.join(CSRC, "rvcp_bvh.cpp"), "-o", exe],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-200:])
    sc = rvcp_amd.scene.with_random_triangles(rvcp_amd.Scene.default(), 3000)
    v = sc.mesh.aligned_vertices()
    f = sc.mesh.aligned_faces()
    meshes = {"random": v["position"][:, :3][f["vertices"]].astype(np.float32),
              "degenerate": np.zeros((5, 3, 3), np.float32),
              "tiny": np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]]], np.float32)}
    for name, tris in meshes.items():
        path = str(tmp_path / f"{name}.bin")
        tris.tofile(path)
        r = subprocess.run([exe, path, "200"], capture_output=True, text=True)
        assert r.returncode == 0, (name, r.stdout[-500:], r.stderr[-2000:])
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
        assert "mismatches 0 of 200" in r.stdout, (name, r.stdout)
        assert "quantized: violations 0" in r.stdout, (name, r.stdout)


def test_bvh4_split_clipping(checker, tmp_path):
    """Early split clipping (round 5): the Cornell walls among many small triangles enter the
    build as clipped pieces.  Same nearest hits as brute force (a leaf may repeat a triangle),
    and fewer traversal steps per ray than the build without it (-DRVCP_BVH_NO_SPLIT_CLIP)."""
    plain = str(tmp_path / "bvh4_plain")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-DRVCP_BVH_NO_SPLIT_CLIP=1",
                    "-I", CSRC, os.path.join(ROOT, "tools", "bvh4_check.cpp"),
                    os.path.join(CSRC, "rvcp_bvh.cpp"), "-o", plain], check=True)
    sc = rvcp_amd.scene.with_random_triangles(rvcp_amd.Scene.default(), 20000)
    v = sc.mesh.aligned_vertices()
    f = sc.mesh.aligned_faces()
    tris = v["position"][:, :3][f["vertices"]].astype(np.float32)
    # plus a scene-spanning sliver and a big off-axis triangle: pieces of thin and tilted shapes
    extra = np.array([[[-270, 1, -270], [270, 547, 270], [270, 548, 269]],
                      [[-200, 50, 100], [150, 500, -250], [200, 60, 240]]], np.float32)
    mesh = str(tmp_path / "mesh.bin")
    np.concatenate([tris, extra]).tofile(mesh)

    def steps(exe):
        r = subprocess.run([exe, mesh, "3000"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "mismatches 0 of 3000" in r.stdout, r.stdout
        line = [l for l in r.stdout.splitlines() if l.startswith("steps/ray")][0]
        return float(line.split()[1])

    assert steps(checker) < 0.97 * steps(plain)


def test_bvh4_hybrid_prefix(checker, tmp_path):
    """The BVH hybrid (round 5, rvcp_host.cpp upload_one): bvh_big_prefix finds the 32 Cornell
    faces that lead the C5-style mesh, the BVH is built over the rest, and brute force over the
    prefix followed by the BVH gives the brute-force nearest hit on every ray, in fewer node
    steps than the BVH over every face.  No prefix for a mesh of small triangles only, nor for
    the Cornell box alone (fewer than 64 faces)."""
    def run(tris, hybrid):
        mesh = str(tmp_path / "mesh.bin")
        np.ascontiguousarray(tris, np.float32).tofile(mesh)
        r = subprocess.run([checker, mesh, "2000"] + (["hybrid"] if hybrid else []),
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "mismatches 0 of 2000" in r.stdout, r.stdout
        k = int([l for l in r.stdout.splitlines() if l.startswith("prefix")][0].split()[1])
        st = float([l for l in r.stdout.splitlines() if l.startswith("steps/ray")][0].split()[1])
        return k, st

    def positions(sc):
        v = sc.mesh.aligned_vertices()
        return v["position"][:, :3][sc.mesh.aligned_faces()["vertices"]]

    cornell = rvcp_amd.Scene.default()
    sc = rvcp_amd.scene.with_random_triangles(cornell, 20000)
    k0, plain = run(positions(sc), False)
    k1, hyb = run(positions(sc), True)
    assert k0 == 0 and k1 == 32
    assert hyb < 0.95 * plain
    assert run(positions(sc)[32:], True)[0] == 0            # small triangles only
    assert run(positions(cornell), True)[0] == 0            # 32 faces: below 64
