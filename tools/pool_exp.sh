#!/usr/bin/env bash
# Kernel schedules (VARIANTS, default 3 6 9), generic and specialised scans, C3 / C2 / C4
# frames (frames.py kernel ms, one frame at a time, two interleaved passes).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { # label args
  local label=$1; shift
  timeout -k 10 120 python tools/frames.py "$@" > /tmp/pe.log 2>/dev/null
  python3 - "$label" <<'PY'
import json, sys
rows = [json.loads(l) for l in open("/tmp/pe.log") if l.startswith("{")]
ms = sorted(r["kernel_ms"] for r in rows[3:])
print(f"{sys.argv[1]:>28}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f} iters {rows[-1]['wave_iterations']} trav {rows[-1]['traversals']}", flush=True)
PY
}
VARS=${VARS:-"3 6 9"}
for pass in 1 2; do
  for v in $VARS; do run "c3 gen v$v" --frames 20 --generic --variant $v; done
  for v in $VARS; do run "c3 spec v$v" --frames 20 --variant $v; done
  for v in $VARS; do run "c2 spec v$v" --frames 40 --size 384 --spp 10 --variant $v; done
  for v in $VARS; do run "c4 spec v$v" --frames 6 --size 2048 --spp 64 --variant $v; done
done
