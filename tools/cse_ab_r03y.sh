#!/usr/bin/env bash
# generator-level common subexpressions in the specialised scan: HEAD build vs this tree
set -e
export PASSES=${PASSES:-3}
for wl in ${WLS:-c3 c3m2 c2 c4}; do
  echo "== $wl"
  BENCH_ARGS="--workload $wl" timeout -k 10 900 bash tools/bench_ab.sh tools/build/var_head/librvcp.so rvcp-real-time-path-tracer_amd/csrc/build/librvcp.so
done
