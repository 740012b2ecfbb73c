#!/bin/bash
# Frames per path kernel (rvcp_render_frames_async batches) x frames in flight x grid per frame,
# for the N=8 share of C4 and for C3 (tools/rank_share.py).
#   tools/batch_sweep.sh "1 2 3 4" "2:0 3:3 1:0"
set -o pipefail
for fg in ${2:-2:0 3:3}; do
  IFS=: read -r f g <<< "$fg"
  for b in ${1:-1 2 3}; do
    echo "== batch $b fif $f grid $g"
    timeout -k 10 200 python -u tools/rank_share.py --ns 8 --fif $f --grid $g --batch $b --frames 24 2>/dev/null || exit 1
    timeout -k 10 200 python -u tools/rank_share.py --ns 1 --fif $f --grid $g --batch $b --frames 24 --size 1024 --spp 30 2>/dev/null || exit 1
  done
done
