"""The N>1 path cannot hang: rvcp_rccl_init creates its communicator
non-blocking and polls it against the context's deadline (rvcp_rccl_set_timeout), so a rank
whose peers never join gets RVCP_E_TIMEOUT and an aborted communicator instead of blocking
inside RCCL -- the reference's own recover-not-hang path is the swapchain's OutOfDate ->
recreate (src/ray_tracer/vulkan.rs:355-364).

Each case runs in a child process under its own time limit, so that a regression (a blocking
init) fails this test instead of hanging the suite."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_NO_PEER = r'''
import time
import numpy as np
import rvcp_amd
from rvcp_amd import abi
print("STAGE start", flush=True)
sc = rvcp_amd.Scene.default()
rt = rvcp_amd.RayTracer(spp=2)
rt.upload_scene(sc)
before = rt.render(40, 24, 123.0)
rt.rccl_set_timeout(TIMEOUT_MS)
uid = rvcp_amd.rccl_unique_id()
print("STAGE init", flush=True)
t0 = time.perf_counter()
try:
    rt.rccl_init(uid, 2, 0)               # world 2, and rank 1 never comes
    print("RESULT ok", flush=True)
except abi.RvcpError as e:
    print("RESULT", e.code, round(time.perf_counter() - t0, 3), str(e), flush=True)
# the context outlives the aborted communicator: it still renders, bit-identically
print("STAGE render", flush=True)
after = rt.render(40, 24, 123.0)
print("SAME", bool(np.array_equal(before, after)), flush=True)
# a gather without a communicator is refused, not attempted
try:
    rt.gather_wait()
    print("WAIT ok", flush=True)
except abi.RvcpError as e:
    print("WAIT", e.code, flush=True)
# and a world-1 communicator can still be made on the same context afterwards
print("STAGE reinit", flush=True)
rt.rccl_init(rvcp_amd.rccl_unique_id(), 1, 0)
print("REINIT ok", flush=True)
print("STAGE close", flush=True)
rt.close()
print("DONE", flush=True)
'''


def _run(code, limit):
    try:
        return subprocess.run([sys.executable, "-u", "-c", code], cwd=ROOT, capture_output=True,
                              text=True, timeout=limit)
    except subprocess.TimeoutExpired as e:
        out = e.stdout.decode() if isinstance(e.stdout, bytes) else (e.stdout or "")
        err = e.stderr.decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        raise AssertionError(f"child hung after {limit} s; stdout:\n{out[-3000:]}\nstderr:\n{err[-3000:]}")


@pytest.mark.gpu
def test_rccl_init_without_peer_times_out():
    """rvcp_rccl_init(world = 2, rank = 0) with no rank 1 returns RVCP_E_TIMEOUT within the
    deadline (+ a bounded abort), the process keeps its context usable and exits cleanly."""
    timeout_ms = 3000
    r = _run(_NO_PEER.replace("TIMEOUT_MS", str(timeout_ms)), 120)
    out = r.stdout
    assert r.returncode == 0, (r.returncode, out[-2000:], r.stderr[-3000:])
    res = [l for l in out.splitlines() if l.startswith("RESULT")]
    assert res, out
    parts = res[0].split()
    assert parts[1] == "-7", res[0]                     # RVCP_E_TIMEOUT
    elapsed = float(parts[2])
    assert timeout_ms / 1000.0 <= elapsed < timeout_ms / 1000.0 + 20.0, res[0]
    assert "SAME True" in out
    assert "WAIT -1" in out                             # RVCP_E_INVALID: no gather in flight
    assert "REINIT ok" in out and "DONE" in out


@pytest.mark.gpu
def test_rccl_set_timeout_validates_context():
    import rvcp_amd
    L = rvcp_amd.abi.load()
    assert L.rvcp_rccl_set_timeout(None, 1000) == rvcp_amd.abi.RVCP_E_INVALID
    with rvcp_amd.RayTracer(spp=1) as rt:
        rt.rccl_set_timeout(0)                          # 0 = no deadline
        rt.rccl_set_timeout(250)
