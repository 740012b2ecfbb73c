#!/usr/bin/env bash
# Same-box A/B of the scan reciprocal: rcp_scan (zero denominators skip the IEEE division)
# vs plain rcp_ieee, for the generic (static) and the specialised (hipRTC) kernels.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pass in 1 2; do
for sz in "1024 30 20" "2048 64 6"; do
  set -- $sz
  for cfg in "base 0" "rcpieee 0" "base 1" "rcpieee 1"; do
    read lib gen <<< "$cfg"
    if [ "$gen" = 1 ]; then export RVCP_NO_SPECIALIZE=1; else unset RVCP_NO_SPECIALIZE; fi
    if [ "$lib" = rcpieee ]; then export RVCP_JIT_FLAGS=-DRVCP_SCAN_RCP_IEEE; else unset RVCP_JIT_FLAGS; fi
    RVCP_LIB=tools/build/var_$lib/librvcp.so timeout -k 10 120 python tools/frames.py --frames $3 --size $1 --spp $2 > /tmp/rab.log 2>/dev/null
    python3 - "$1" "$lib" "$gen" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/rab.log") if l.startswith("{"))
print(f"pass {sys.argv[4]} size {sys.argv[1]:>4} {sys.argv[2]:>8} generic {sys.argv[3]}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}")
PY
  done
done
done
