#!/usr/bin/env bash
# Marginal costs of the specialised path kernel's steps at C3: each
# RVCP_EXP_* knob runs one step a second time (inputs laundered, results discarded) in the
# hipRTC-compiled kernel; frames are unchanged.  Two interleaved passes, 20 frames each.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pass in 1 2; do
  for f in "" "-DRVCP_EXP_SCAN_REPEAT=2" "-DRVCP_EXP_REPEAT_NEE=1" "-DRVCP_EXP_REPEAT_COOP=1" "-DRVCP_EXP_REPEAT_BRDF=1" "-DRVCP_EXP_REPEAT_HIT=1"; do
    RVCP_JIT_FLAGS="$f" timeout -k 10 120 python tools/frames.py --frames 20 > /tmp/sc.log 2>/dev/null
    python3 - "${f:-base}" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/sc.log") if l.startswith("{"))
print(f"pass {sys.argv[2]} {sys.argv[1]:>28}  median {ms[len(ms)//2]:.3f} min {ms[0]:.3f}")
PY
  done
done
