#!/usr/bin/env bash
# Frames in flight x hardware queues per process (GPU_MAX_HW_QUEUES) for C2 and C3 (bench.py),
# interleaved repetitions on one box.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for cfg in "4 2 c3" "4 3 c3" "4 3 c2" "8 4 c2" "8 3 c2"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python bench.py --workload $3 --steps 60 --warmup 6 --no-cpu-baseline --frames-in-flight $2 > /tmp/h.log 2>&1
    python3 -c "import json; d=json.loads(open('/tmp/h.log').read().strip().splitlines()[-1]); print('rep=$rep hwq=$1 fif=$2 $3', d['value'], d['ms_per_step'])"
  done
done
