#!/usr/bin/env python3
"""Overlap of consecutive frames' kernels in a rocprofv3 --kernel-trace CSV: for each path-kernel
launch (in start order) its duration, the pre-pass/tone-map launches around it, and how long it
ran alongside the previous path-kernel launch (frames in flight fill a frame's tail only when
the next frame's kernels start before it ends).

  python tools/trace_overlap.py run_kernel_trace.csv [--skip K]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--last", type=int, default=0, help="only the last N path launches")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        n = r["Kernel_Name"]
        kind = ("path" if ("path_kernel" in n or "legacy_kernel" in n or "tiled" in n) else
                "pre" if "primary_kernel" in n else "tone" if "tonemap" in n else None)
        if kind:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind,
                         r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    path = [r for r in rows if r[2] == "path"][a.skip:]
    if a.last:
        path = path[-a.last:]
    dur, ovl, gap = [], [], []
    for p, c in zip(path, path[1:]):
        dur.append((c[1] - c[0]) / 1e6)
        ovl.append(max(0, p[1] - c[0]) / 1e6)
        gap.append(max(0, c[0] - p[1]) / 1e6)
    for i, (p, c) in enumerate(zip(path, path[1:])):
        if i < 12:
            print(f"launch {i + 1}: start +{(c[0] - path[0][0]) / 1e6:8.3f} ms  dur {(c[1] - c[0]) / 1e6:.3f}"
                  f"  overlap with previous {max(0, p[1] - c[0]) / 1e6:.3f}  gap {max(0, c[0] - p[1]) / 1e6:.3f}"
                  f"  queue {c[3]}")
    if dur:
        span = (path[-1][1] - path[0][0]) / 1e6
        print(f"path launches {len(path)}: median dur {statistics.median(dur):.3f} ms, median overlap "
              f"{statistics.median(ovl):.3f} ms, median gap {statistics.median(gap):.3f} ms, "
              f"span/launch {span / len(path):.3f} ms")
    pre = [r for r in rows if r[2] == "pre"]
    if pre:
        print(f"pre-pass median {statistics.median([(r[1] - r[0]) / 1e6 for r in pre]):.3f} ms, "
              f"tone map median {statistics.median([(r[1] - r[0]) / 1e6 for r in rows if r[2] == 'tone'] or [0]):.3f} ms")


if __name__ == "__main__":
    main()
