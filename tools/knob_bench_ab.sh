#!/usr/bin/env bash
# Same-box A/B of debug-build environment knobs through bench.py (C3 unless BENCH_ARGS says
# otherwise; ms_per_step, interleaved passes):  tools/knob_bench_ab.sh "VAR=v" "VAR=w" ...
# ("-" = no knob).  Uses the debug build of the library (knobs exist only there).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RVCP_LIB=rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so
for pass in $(seq ${PASSES:-2}); do
  for kv in "$@"; do
    if [ "$kv" = "-" ]; then cmd="env"; else cmd="env $kv"; fi
    $cmd timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --launch-pass 0 ${BENCH_ARGS:-} > /tmp/kab.log 2>/dev/null
    python3 - "$kv" "$pass" <<'PY'
import json, sys
d = json.loads([l for l in open("/tmp/kab.log") if l.startswith("{")][-1])
print(f"pass {sys.argv[2]} {sys.argv[1]:>36}  ms_per_step {d['ms_per_step']:.4f}  Msamples/s {d['value']:.1f}", flush=True)
PY
  done
done
