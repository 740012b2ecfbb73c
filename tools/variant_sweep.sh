#!/usr/bin/env bash
# Kernel-variant sweep over mesh sizes (auto-variant thresholds).  GPU box only.
set -u
for t in ${TRIS:-1024 4096 16384}; do
  for v in ${VARS:-3 4 5}; do
    echo "tris=$t variant=$v"
    timeout -k 10 300 python tools/frames.py --frames 2 --spp 8 --tris $t --variant $v || exit 1
  done
done
