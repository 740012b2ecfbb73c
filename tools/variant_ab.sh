#!/usr/bin/env bash
# Same-box A/B of kernel schedules (frames.py --variant), three interleaved passes.
#   tools/variant_ab.sh "V1 V2 ..." ["frames.py args"]...
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS=$1; shift
[ $# -gt 0 ] || set -- ""
for pass in 1 2 3; do
  for args in "$@"; do
    for v in $VARS; do
      timeout -k 10 120 python tools/frames.py --frames 20 --variant $v $args > /tmp/vab.log 2>/dev/null
      python3 - "$v" "$args" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/vab.log") if l.startswith("{"))
print(f"pass {sys.argv[3]} [{sys.argv[2]:>30}] variant {sys.argv[1]}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}")
PY
    done
  done
done
