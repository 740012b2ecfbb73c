#!/usr/bin/env bash
# shared-reciprocal divisions (divs_y) on/off, same box (debug build: the hipRTC module takes -D)
set -e
export PASSES=${PASSES:-3}
for wl in c3 c3m2 spheres; do
  BENCH_ARGS="--workload $wl" timeout -k 10 600 bash tools/knob_bench_ab.sh - RVCP_JIT_FLAGS=-DRVCP_DIV_SHARED=0
done
