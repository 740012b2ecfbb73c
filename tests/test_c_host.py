"""The drop-in boundary from a host that is neither Python nor torch: examples/rvcp_render.c
drives librvcp through include/rvcp.h alone (create, upload_scene_file, render, destroy), as the
reference's Rust loop would after INTEGRATION.md.  Built by __graft_entry__.build()."""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "build", "rvcp_render")


def _read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    magic, dims, maxv, rest = data.split(b"\n", 3)
    assert magic == b"P6" and maxv == b"255"
    w, h = map(int, dims.split())
    return np.frombuffer(rest, dtype=np.uint8).reshape(h, w, 3)


def test_c_host_built_and_linked():
    """The example exists (build() made it) and resolves librvcp from the tree."""
    assert os.path.exists(EXE), "run __graft_entry__.build() first"
    out = subprocess.run(["ldd", EXE], capture_output=True, text=True).stdout
    assert "librvcp.so" in out and "not found" not in out.split("librvcp.so")[1].split("\n")[0]


def test_c_host_usage_error():
    r = subprocess.run([EXE], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,spp", [("cornell", 96, 64, 4), ("random", 57, 41, 3)])
def test_c_host_render_bitexact(tmp_path, name, W, H, spp):
    sc = rvcp_amd.Scene.default()
    if name == "random":
        sc = rvcp_amd.scene.with_random_triangles(sc, 200)
    scene = str(tmp_path / "s.rvcpscn")
    rvcp_amd.scene_io.save(scene, sc)
    ppm = str(tmp_path / "out.ppm")
    r = subprocess.run([EXE, scene, str(W), str(H), str(spp), "123.0", "2", ppm],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 2 and lines[0]["traversals"] == lines[1]["traversals"] > 0
    got = _read_ppm(ppm)
    cfg = rvcp_amd.abi.make_config(spp=spp)
    _, want, trav = O.render(scene_arrays(sc), sc.push_constant(123.0), cfg, W, H,
                             want_linear=False)
    assert np.array_equal(got, want[..., :3])
    assert lines[1]["traversals"] == trav


@pytest.mark.gpu
def test_c_host_reports_bad_scene(tmp_path):
    bad = tmp_path / "bad.rvcpscn"
    bad.write_bytes(b"not a scene")
    r = subprocess.run([EXE, str(bad), "8", "8", "1", "0", "1", str(tmp_path / "o.ppm")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "rvcp_upload_scene_file failed" in r.stderr
