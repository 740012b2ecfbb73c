#!/usr/bin/env bash
# Same-box sweep of the LDS-tiled schedules (4 = dual-slot, 5 = single-slot) over mesh and
# frame sizes (frames.py kernel ms, median over the frames, two passes).  Feeds the automatic
# schedule rule in rvcp_host.cpp.
#   tools/variant_sweep.sh [variants...]      default: 4 5
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS=${*:-"4 5"}
for pass in 1 2; do
  for args in "--tris 300 --size 512 --spp 4 --frames 10" "--tris 2000 --size 1024 --spp 8 --frames 6" \
              "--tris 10000 --size 512 --spp 8 --frames 4" "--tris 100000 --size 1024 --spp 8 --frames 3" \
              "--tris 100000 --size 1024 --spp 30 --frames 2"; do
    for v in $VARS; do
      timeout -k 10 200 python tools/frames.py --variant "$v" $args > /tmp/vs.log 2>/dev/null
      python3 - "$v" "$args" "$pass" <<'PY'
import json, sys
ms = sorted(json.loads(l)["kernel_ms"] for l in open("/tmp/vs.log") if l.startswith("{"))
print(f"pass {sys.argv[3]} [{sys.argv[2]:>46}] variant {sys.argv[1]}  median {ms[len(ms)//2]:.4f} min {ms[0]:.4f}", flush=True)
PY
    done
  done
done
