#!/usr/bin/env python3
"""One line per bench.py log: ms per frame, Msamples/s, frames in flight, grid, roofline fracs.
  python tools/bench_summary.py gpurun_out/r03zq_bench_*.log"""
import json
import sys

for path in sys.argv[1:]:
    try:
        line = [x for x in open(path) if x.startswith("{")][-1]
    except (OSError, IndexError):
        print(f"{path}: no JSON line")
        continue
    d = json.loads(line)
    c, r = d["config"], d.get("roofline") or {}
    pl = r.get("per_launch") or {}
    extra = {k: c[k] for k in ("speedup_vs_one_gpu_same_frame", "one_gpu_ms",
                               "assembled_frame_bitexact_vs_1gpu", "gather") if k in c}
    print(f"{path}: {c['workload']} n={d['n_gpus']} ms {d['ms_per_step']} value {d['value']} "
          f"fif {c.get('frames_in_flight')} grid {c.get('grid_waves_per_simd')} frac {r.get('frac')} "
          f"per_launch {pl.get('kernel_ms')} {extra if extra else ''}")
