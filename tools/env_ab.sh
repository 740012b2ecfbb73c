#!/usr/bin/env bash
# Same-box A/B of an environment setting (frames.py kernel ms, median of 20 frames, two
# passes):  tools/env_ab.sh "VAR=value" ["frames.py args"]...
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# environment knobs exist only in the debug build of the library (csrc: make debug)
export RVCP_LIB=${RVCP_LIB:-rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so}
SETTING=$1; shift
[ $# -gt 0 ] || set -- ""
for pass in 1 2; do
  for args in "$@"; do
    for on in 0 1; do
      if [ $on = 1 ]; then cmd="env $SETTING"; else cmd="env"; fi
      $cmd timeout -k 10 120 python tools/frames.py --frames 20 $args > /tmp/eab.log 2>/dev/null
      python3 - "$SETTING" "$on" "$args" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/eab.log") if l.startswith("{"))
print(f"pass {sys.argv[4]} [{sys.argv[3]:>22}] {sys.argv[1] if sys.argv[2] == '1' else 'default':>24}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}")
PY
    done
  done
done
