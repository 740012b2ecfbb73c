#!/usr/bin/env bash
# Experiments on the GPU box (variants built here by tools/build_variant.sh):
#   repN : C3 / C2 frames with the path kernel's scan run N times (-DRVCP_EXP_SCAN_REPEAT=N);
#          the frames do not change, only the time -- the scan's share of the frame;
#   ww   : the BVH traversal in while-while form (-DRVCP_BVH_WHILE_WHILE=1) vs rep1 on C5.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in rep1 rep2 rep3; do
  echo "== $v c3"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 120 python tools/frames.py --frames 8 | tail -3
  echo "== $v c2"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 120 python tools/frames.py --frames 8 --size 384 --spp 10 | tail -2
done
for v in rep1 ww; do
  echo "== $v c5-bvh"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 200 python tools/frames.py --frames 3 --tris 100000 --accel 1 | tail -2
done
