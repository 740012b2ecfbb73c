#!/bin/bash
# bench.py lines with the path kernel's grid per frame (rvcp_config_t.grid_waves_per_simd,
# --grid-waves) and frames in flight varied: "workload:steps:fif:grid" per argument.
#   tools/grid_bench_ab.sh c3:40:2:0 c3:40:3:3 ...
set -o pipefail
for spec in "$@"; do
  IFS=: read -r w n f g <<< "$spec"
  line=$(timeout -k 10 200 python -u bench.py --workload $w --steps $n --warmup 4 --no-cpu-baseline \
         --launch-pass 0 --frames-in-flight $f --grid-waves $g 2>/dev/null | tail -1) || exit 1
  python - "$spec" "$line" <<'PY'
import json, sys
d = json.loads(sys.argv[2])
print(f"{sys.argv[1]:>16}  ms/frame {d['ms_per_step']:.4f}  Msamples/s {d['value']:.1f}", flush=True)
PY
done
