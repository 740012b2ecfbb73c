#!/usr/bin/env bash
# Specialised-kernel A/B: schedule 3 (5 waves) vs 6 (6 waves), generic vs specialised (§4.7).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# environment knobs exist only in the debug build of the library (csrc: make debug)
export RVCP_LIB=${RVCP_LIB:-rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so}
for sz in "1024 30" "2048 64 6" "384 10"; do
  set -- $sz
  fr=${3:-20}
  for cfg in "6 0" "3 0" "6 1" "3 1"; do
    read v off <<< "$cfg"
    if [ "$off" = 1 ]; then export RVCP_NO_SPECIALIZE=1; else unset RVCP_NO_SPECIALIZE; fi
    timeout -k 10 120 python tools/frames.py --frames $fr --size $1 --spp $2 --variant $v > /tmp/sab.log 2>/dev/null
    python3 - "$1" "$2" "$v" "$off" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/sab.log") if l.startswith("{"))[:max(1, 3 * 5)]
print(f"size {sys.argv[1]:>4} spp {sys.argv[2]:>2} variant {sys.argv[3]} generic {sys.argv[4]}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}")
PY
  done
done
