#!/bin/bash
# Frames per launch for the opt-in BVH on C5 (persistent BVH path kernel): bench lines.
set -o pipefail
for b in 1 2 3 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --accel bvh --steps 6 --warmup 2 --no-cpu-baseline \
      --launch-pass 0 --batch $b > /tmp/bvhb.log 2>&1 || exit 1
  python tools/bench_summary.py /tmp/bvhb.log | sed "s|^|batch $b: |"
done
