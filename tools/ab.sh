#!/usr/bin/env bash
# A/B timing on the GPU box: tools/ab.sh "<frames.py args>" VARIANT...  (variants built by
# tools/build_variant.sh into tools/build/var_<name>/).  Two interleaved passes per variant,
# 20 frames each; prints the median of the last 15 kernel times of every pass.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args=$1; shift
for pass in 1 2; do
  for v in "$@"; do
    RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 300 python tools/frames.py --frames 20 $args > /tmp/ab_$v.log 2>/dev/null
    python3 - "$v" "$pass" <<'PY'
import json, sys
ms = [json.loads(l)["kernel_ms"] for l in open(f"/tmp/ab_{sys.argv[1]}.log") if l.startswith("{")]
ms = sorted(ms[5:])
print(f"{sys.argv[1]:>12} pass {sys.argv[2]}  median {ms[len(ms)//2]:.3f}  min {ms[0]:.3f}")
PY
  done
done
