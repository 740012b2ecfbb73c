#!/usr/bin/env bash
# Plane-cull A/B: which rays' tests get the wave-level sign cull.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pass in 1 2; do
for sz in "1024 30 20" "384 10 40"; do
  set -- $sz
  for c in "none" "A" "AB1" "B"; do
    for v in 3 6; do
      RVCP_JIT_CULL=$c timeout -k 10 120 python tools/frames.py --frames $3 --size $1 --spp $2 --variant $v > /tmp/cab.log 2>/dev/null
      python3 - "$1" "$c" "$v" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/cab.log") if l.startswith("{"))
print(f"pass {sys.argv[4]} size {sys.argv[1]:>4} cull {sys.argv[2]:>4} variant {sys.argv[3]}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}")
PY
    done
  done
done
done
