"""Committed golden frames (tests/golden/oracle_frames.npz, made by
tests/golden/make_oracle_fixtures.py).

CPU: the oracle still renders every committed frame bit for bit (a regression pin of the
checker itself) from scene buffers whose SHA-256 matches the one recorded at generation.
GPU: the HIP kernel (librvcp, through the C-ABI) renders the same frames bit for bit --
tolerance: linear RGB bitwise equal, RGBA8 equal, traversal count equal.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_oracle_fixtures as G  # noqa: E402
import rvcp_amd  # noqa: E402

GOLDEN = np.load(os.path.join(HERE, "golden", "oracle_frames.npz"))
CASES = list(G.CASES)


def _expected(case):
    return (GOLDEN[case + "/linear"], GOLDEN[case + "/rgba"],
            int(GOLDEN[case + "/traversals"]), str(GOLDEN[case + "/scene_sha256"]))


@pytest.mark.parametrize("case", CASES)
def test_scene_buffers_unchanged(case):
    scn = G.CASES[case][0]
    assert G.scene_digest(G.arrays_of(G.scene_of(scn))) == _expected(case)[3]


@pytest.mark.parametrize("case", CASES)
def test_oracle_reproduces_golden(case):
    lin, rgba, trav, _ = _expected(case)
    _, _, _, o_lin, o_rgba, o_trav = G.render(case)
    assert np.array_equal(o_lin.view(np.uint32), lin.view(np.uint32))
    assert np.array_equal(o_rgba, rgba)
    assert o_trav == trav


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_hip_matches_golden(case):
    lin, rgba, trav, _ = _expected(case)
    scn, kw, W, H, t = G.CASES[case]
    sc = G.scene_of(scn)
    with rvcp_amd.RayTracer(rvcp_amd.abi.make_config(**kw)) as rt:
        rt.upload_scene(sc)
        g_rgba, g_lin = rt.render(W, H, t, want_linear=True)
        st = rt.last_stats
    assert np.array_equal(g_lin.view(np.uint32), lin.view(np.uint32))
    assert np.array_equal(g_rgba, rgba)
    assert int(st["traversals"]) == trav
