#!/usr/bin/env python3
"""Summarise per-wave timeline dumps of the path kernel (debug build of the library,
RVCP_DEBUG_TIMELINE): {start, queue-exhausted, end, iterations} in s_memrealtime ticks (100 MHz),
{start, end} in s_memtime ticks (shader clock), so `clock_ghz` = the in-kernel clock, and -- with
RVCP_JIT_FLAGS=-DRVCP_REGION_CLOCK, specialised kernels -- the shader cycles each wave spent in
its scans and in its iterations as a whole (`scan_frac`):

  RVCP_LIB=rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so \
      RVCP_DEBUG_TIMELINE=/tmp/tl.bin python tools/frames.py --frames 3
  python tools/timeline.py /tmp/tl.bin --waves N
"""
import argparse
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--waves", type=int, required=True, help="waves per launch (file size / 64 / frames)")
    a = ap.parse_args()
    t = np.fromfile(a.path, dtype=np.uint64).reshape(-1, a.waves, 8).astype(np.float64)
    for k, fr in enumerate(t):
        st, ex, en, it = fr[:, 0], fr[:, 1], fr[:, 2], fr[:, 3]
        ok = (en > st) & (fr[:, 5] > fr[:, 4])
        ghz = (fr[ok, 5] - fr[ok, 4]) / (en[ok] - st[ok]) * 0.1
        t0 = st.min()
        span = en.max() - t0
        ex = np.where(ex > 0, ex, en)
        q = lambda x: [round(float(v), 3) for v in np.percentile((x - t0) / span, [0, 10, 50, 90, 100])]
        print(json.dumps({"frame": k, "span_ms": round(span / 1e5, 3),
                          "start_pct": q(st), "exhausted_pct": q(ex), "end_pct": q(en),
                          "mean_residency": round(float(np.mean((en - st) / span)), 4),
                          "iters_p50": float(np.median(it)), "iters_max": float(it.max()),
                          "us_per_iter_p50": round(float(np.median((en - st)[it > 0] / it[it > 0])) / 100.0, 3),
                          "waves_with_work": int((it > 0).sum()),
                          "scan_frac": round(float(fr[:, 6].sum() / fr[:, 7].sum()), 4)
                          if fr[:, 7].sum() > 0 else None,
                          "clock_ghz_p50": round(float(np.median(ghz)), 4) if ghz.size else None,
                          "clock_ghz_p10_p90": [round(float(np.percentile(ghz, p)), 4) for p in (10, 90)]
                          if ghz.size else None}))


if __name__ == "__main__":
    main()
