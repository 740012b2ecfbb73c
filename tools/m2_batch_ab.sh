#!/bin/bash
# Integrator mode 2 pipelines (bench.py lines): "workload:steps:fif:grid:batch" per argument.
set -o pipefail
for spec in "$@"; do
  IFS=: read -r w n f g b <<< "$spec"
  timeout -k 10 200 python -u bench.py --workload $w --steps $n --warmup 6 --no-cpu-baseline \
      --launch-pass 0 --frames-in-flight $f --grid-waves $g --batch $b > /tmp/m2b.log 2>&1 || exit 1
  python tools/bench_summary.py /tmp/m2b.log | sed "s|^|$spec: |"
done
