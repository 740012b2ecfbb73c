#!/usr/bin/env bash
# Same-box A/B of kernel schedules on Cornell workloads (frames.py kernel ms, one frame at a
# time, median over the frames after the first 3, two interleaved passes).
#   tools/sched_ab.sh "VARIANTS" "frames.py args" ["frames.py args"]...
#   e.g. tools/sched_ab.sh "3 9" "--frames 20" "--size 384 --spp 10 --frames 40"
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS=$1; shift
for pass in 1 2; do
  for args in "$@"; do
    for v in $VARS; do
      timeout -k 10 200 python tools/frames.py --variant "$v" $args > /tmp/sab.log 2>/dev/null
      python3 - "$v" "$args" "$pass" <<'PY'
import json, sys
rows = [json.loads(l) for l in open("/tmp/sab.log") if l.startswith("{")]
ms = sorted(r["kernel_ms"] for r in rows[3:] or rows)
it = rows[-1]["wave_iterations"]
print(f"pass {sys.argv[3]} [{sys.argv[2]:>36}] variant {sys.argv[1]}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}  wave-iters {it}", flush=True)
PY
    done
  done
done
