#!/usr/bin/env bash
# mode-2 settle deferral threshold sweep (debug build, RVCP_JIT_FLAGS reaches the hipRTC module)
set -e
export PASSES=${PASSES:-3}
for wl in spheres c3m2; do
  BENCH_ARGS="--workload $wl" timeout -k 10 600 bash tools/knob_bench_ab.sh - \
    RVCP_JIT_FLAGS=-DRVCP_LEGACY_DEFER=12 RVCP_JIT_FLAGS=-DRVCP_LEGACY_DEFER=16 \
    RVCP_JIT_FLAGS=-DRVCP_LEGACY_DEFER=24 RVCP_JIT_FLAGS=-DRVCP_LEGACY_DEFER=32 \
    RVCP_JIT_FLAGS=-DRVCP_LEGACY_DEFER=40
done
