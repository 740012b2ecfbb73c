import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
CSRC = os.path.join(ROOT, "rvcp-real-time-path-tracer_amd", "csrc")
for p in (ROOT, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = os.path.join(CSRC, "build", "librvcp.so")
    orc = os.path.join(ORACLE_DIR, "build", "librvcp_oracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-j8", "-C", CSRC], check=True)
    if not os.path.exists(orc):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def cornell():
    import rvcp_amd
    return rvcp_amd.Scene.default()


def scene_arrays(sc):
    return dict(materials=sc.aligned_materials(), vertices=sc.mesh.aligned_vertices(),
                faces=sc.mesh.aligned_faces(), lum_face_ids=sc.luminous_face_ids(),
                spheres=sc.aligned_spheres())


@pytest.fixture(scope="session")
def cornell_arrays(cornell):
    return scene_arrays(cornell)


def readme_blocks():
    d = np.load(os.path.join(ROOT, "tests", "golden", "readme_blockmeans.npz"))
    return d["blocks32"].astype(np.float64), d["blocks16"].astype(np.float64)


def block_means(rgba, nblocks):
    """Mean of 8-bit RGB (scaled to [0,1]) over an nblocks x nblocks grid of a square image."""
    h = rgba.shape[0]
    k = h // nblocks
    x = rgba[:nblocks * k, :nblocks * k, :3].astype(np.float64) / 255.0
    return x.reshape(nblocks, k, nblocks, k, 3).mean(axis=(1, 3))
