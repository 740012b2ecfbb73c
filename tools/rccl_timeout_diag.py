"""Diagnostic (GPU box): rvcp_rccl_init(world = 2, rank = 0) with no peer, each stage stamped,
to see where a non-blocking RCCL init / abort spends its time.  Run with NCCL_DEBUG=INFO."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rvcp_amd  # noqa: E402

t00 = time.perf_counter()


def stamp(msg):
    print(f"[{time.perf_counter() - t00:8.3f}] {msg}", flush=True)


stamp("start")
rt = rvcp_amd.RayTracer(spp=1)
stamp("context")
rt.rccl_set_timeout(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)
uid = rvcp_amd.rccl_unique_id()
stamp("unique id")
try:
    rt.rccl_init(uid, 2, 0)
    stamp("init returned ok (unexpected)")
except rvcp_amd.abi.RvcpError as e:
    stamp(f"init raised {e}")
rt.close()
stamp("closed")
