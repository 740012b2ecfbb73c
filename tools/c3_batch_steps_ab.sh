#!/bin/bash
# C3 bench lines at the driver-like step counts with batches of 3 vs deeper ones.
set -o pipefail
for rep in 1 2; do
  for sb in 20:3 20:5 40:3 40:6 20:4; do
    IFS=: read -r n b <<< "$sb"
    timeout -k 10 200 python -u bench.py --steps $n --warmup 3 --no-cpu-baseline --launch-pass 0 --batch $b > /tmp/c3b.log 2>&1 || exit 1
    python tools/bench_summary.py /tmp/c3b.log | sed "s|^|rep $rep steps $n batch $b: |"
  done
done
