#!/usr/bin/env python3
"""Overlap of consecutive frames' kernels in a rocprofv3 --kernel-trace CSV: for each path-kernel
launch (in start order) its duration, the pre-pass/tone-map launches around it, and how long it
ran alongside the previous path-kernel launch (frames in flight fill a frame's tail only when
the next frame's kernels start before it ends).  With gathers in the trace (RCCL kernels and
rank 0's assemble_kernel, rvcp_gather_frame_async), also: which hardware queue each kind of
kernel ran on, and how many gathers started while a path kernel was running (a gather queued
behind a render on a shared queue would start only after it).

  python tools/trace_overlap.py run_kernel_trace.csv [--skip K] [--last N]
"""
import argparse
import collections
import csv
import statistics


def kind_of(name):
    if "path_kernel" in name or "legacy_kernel" in name or "tiled" in name:
        return "path"
    if "primary_kernel" in name:
        return "pre"
    if "tonemap" in name:
        return "tone"
    if "assemble_kernel" in name:
        return "assemble"
    if "nccl" in name.lower():
        return "gather"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--last", type=int, default=0, help="only the last N path launches")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        kind = kind_of(r["Kernel_Name"])
        if kind:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind,
                         r.get("Queue_Id", r.get("Stream_Id", "?")), r.get("Stream_Id", "?")))
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
                  f"  queue {c[3]}  stream {c[4]}")
    if dur:
        span = (path[-1][1] - path[0][0]) / 1e6
        print(f"path launches {len(path)}: median dur {statistics.median(dur):.3f} ms, median overlap "
              f"{statistics.median(ovl):.3f} ms, median gap {statistics.median(gap):.3f} ms, "
              f"span/launch {span / len(path):.3f} ms, launches overlapping the previous one "
              f"{sum(1 for o in ovl if o > 0)}/{len(ovl)}")
    pre = [r for r in rows if r[2] == "pre"]
    if pre:
        print(f"pre-pass median {statistics.median([(r[1] - r[0]) / 1e6 for r in pre]):.3f} ms, "
              f"tone map median {statistics.median([(r[1] - r[0]) / 1e6 for r in rows if r[2] == 'tone'] or [0]):.3f} ms")
    per_q = collections.defaultdict(collections.Counter)
    for r in rows:
        per_q[r[2]][f"q{r[3]}/s{r[4]}"] += 1
    for k in ("path", "pre", "tone", "gather", "assemble"):
        if per_q.get(k):
            print(f"{k:8s} launches by queue/stream: {dict(sorted(per_q[k].items()))}")
    gathers = [r for r in rows if r[2] == "gather"]
    if gathers and path:
        t_lo = path[0][0]
        gathers = [g for g in gathers if g[0] >= t_lo]
        during = sum(1 for g in gathers if any(p[0] < g[0] < p[1] for p in path))
        gq = {g[3] for g in gathers}
        pq = {p[3] for p in path}
        print(f"gathers after the first counted path launch: {len(gathers)}, started while a path "
              f"kernel ran: {during}; median gather {statistics.median([(g[1] - g[0]) / 1e6 for g in gathers]):.4f} ms; "
              f"gather queues {sorted(gq)} vs path queues {sorted(pq)}: "
              f"{'disjoint' if not (gq & pq) else 'SHARED'}")
    asm = [r for r in rows if r[2] == "assemble"]
    if asm:
        print(f"assemble median {statistics.median([(r[1] - r[0]) / 1e6 for r in asm]):.4f} ms")


if __name__ == "__main__":
    main()
