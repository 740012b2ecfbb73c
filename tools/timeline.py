#!/usr/bin/env python3
"""Summarise RVCP_DEBUG_TIMELINE dumps (per-wave {start, queue-exhausted, end, iterations} of
the path kernel, s_memrealtime ticks at 100 MHz):

  RVCP_DEBUG_TIMELINE=/tmp/tl.bin python tools/frames.py --frames 3
  python tools/timeline.py /tmp/tl.bin --waves N
"""
import argparse
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--waves", type=int, required=True, help="waves per launch")
    a = ap.parse_args()
    t = np.fromfile(a.path, dtype=np.uint64).reshape(-1, a.waves, 4).astype(np.float64)
    for k, fr in enumerate(t):
        st, ex, en, it = fr[:, 0], fr[:, 1], fr[:, 2], fr[:, 3]
        t0 = st.min()
        span = en.max() - t0
        ex = np.where(ex > 0, ex, en)
        q = lambda x: [round(float(v), 3) for v in np.percentile((x - t0) / span, [0, 10, 50, 90, 100])]
        print(json.dumps({"frame": k, "span_ms": round(span / 1e5, 3),
                          "start_pct": q(st), "exhausted_pct": q(ex), "end_pct": q(en),
                          "mean_residency": round(float(np.mean((en - st) / span)), 4),
                          "iters_p50": float(np.median(it)), "iters_max": float(it.max()),
                          "us_per_iter_p50": round(float(np.median((en - st)[it > 0] / it[it > 0])) / 100.0, 3),
                          "waves_with_work": int((it > 0).sum())}))


if __name__ == "__main__":
    main()
