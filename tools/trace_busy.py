#!/usr/bin/env python3
"""GPU-busy time per frame from a rocprofv3 kernel trace (--kernel-trace CSV): the union of the
path-tracing kernels' [start, end] intervals (the pre-pass, path kernel and tone map of every
launch) over the timed frames.  With frames in flight and batches the launches overlap, so their
per-launch durations (kernel_stats "AverageNs") exceed the frame rate; the union of the
intervals is what the device spent, and divided by the frames it covers it is comparable with
bench.py's ms_per_step (it must not exceed it by more than the host-side gaps allow).

  python tools/trace_busy.py run_kernel_trace.csv --frames N

--frames: the frames the traced run rendered.  Trace a run whose every launch is timed
(`bench.py --warmup 0 --launch-pass 0`, gpu_check.sh step `profbusy`), so that the busy time per
frame compares with that run's ms_per_step.  --skip K: leave out the first K path-kernel launches
and everything up to their end -- bench.py warms every frame-in-flight context with one full
batch even at --warmup 0 (its warm-up rule), so K = frames in flight.
"""
import argparse
import csv

KERNELS = ("path_kernel", "primary_kernel", "tonemap_kernel", "legacy_kernel", "tiled")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--skip", type=int, default=0)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"]
        if not any(k in name for k in KERNELS):
            continue
        is_path = "path_kernel" in name or "legacy_kernel" in name or "tiled" in name
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), is_path))
    rows.sort()
    if a.skip:
        # the warm-up launches and what ran with them: everything that starts no later than the
        # last of them ends (their pre-passes before, their tone maps at that end)
        t_cut = max(e for _, e, _ in [r for r in rows if r[2]][:a.skip])
        rows = [r for r in rows if r[0] > t_cut]
    n_path = sum(1 for r in rows if r[2])
    iv = [(s_, e_) for s_, e_, _ in rows]
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0] if iv else 0
    print(f"path-kernel launches {n_path}, frames {a.frames}: busy {busy / 1e6:.3f} ms "
          f"({busy / 1e6 / a.frames:.4f} ms per frame), first-to-last span {span / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
