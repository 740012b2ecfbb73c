#!/usr/bin/env bash
# BVH A/B on the GPU box: variants named on the command line (tools/build/var_<name>/librvcp.so),
# C3 and C5 frames with the opt-in BVH.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  echo "== $v c3-bvh"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 120 python tools/frames.py --frames 4 --accel 1 | tail -2
  echo "== $v c5-bvh"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 200 python tools/frames.py --frames 3 --tris 100000 --accel 1 | tail -2
done
