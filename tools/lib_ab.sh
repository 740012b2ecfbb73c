#!/usr/bin/env bash
# Same-box A/B of two librvcp builds (frames.py kernel ms, median of 20 frames, two passes):
#   tools/lib_ab.sh LIB_A LIB_B ["frames.py args"]...
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; B=$2; shift 2
[ $# -gt 0 ] || set -- ""
for pass in 1 2; do
  for args in "$@"; do
    for lib in "$A" "$B"; do
      RVCP_LIB=$lib timeout -k 10 120 python tools/frames.py --frames 20 $args > /tmp/lab.log 2>/dev/null
      python3 - "$lib" "$args" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/lab.log") if l.startswith("{"))
print(f"pass {sys.argv[3]} [{sys.argv[2]:>22}] {sys.argv[1][-40:]:>40}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}")
PY
    done
  done
done
