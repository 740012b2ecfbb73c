#!/usr/bin/env bash
# Same-box A/B of librvcp builds through bench.py (ms_per_step, frames in flight as the bench
# picks them unless BENCH_ARGS says otherwise), interleaved passes.
#   tools/bench_ab.sh LIB... ; BENCH_ARGS="--workload c2" PASSES=3
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pass in $(seq ${PASSES:-2}); do
  for lib in "$@"; do
    RVCP_LIB=$lib timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --launch-pass 0 ${BENCH_ARGS:-} > /tmp/bab.log 2>/dev/null
    python3 - "$lib" "$pass" <<'PY'
import json, sys
d = json.loads([l for l in open("/tmp/bab.log") if l.startswith("{")][-1])
print(f"pass {sys.argv[2]} {sys.argv[1][-44:]:>44}  ms_per_step {d['ms_per_step']:.4f}  Msamples/s {d['value']:.1f}  fif {d['config']['frames_in_flight']}", flush=True)
PY
  done
done
