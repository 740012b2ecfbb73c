#!/bin/bash
# Pipelines of at most 4 frames in flight (frames in flight x frames per launch) and two deeper
# ones, repeated, for the N=8 share of C4, C3, C2 and the one-GPU C4 frame (rank_share.py).
#   each spec fif:grid:batch
set -o pipefail
rs() { timeout -k 10 200 python -u tools/rank_share.py "$@" 2>/dev/null || exit 1; }
for rep in 1 2; do
  for spec in 3:3:1 2:0:2 2:4:2 2:3:2 3:3:2 2:0:3; do
    IFS=: read -r f g b <<< "$spec"
    echo "== rep $rep fif $f grid $g batch $b"
    rs --ns 8 --fif $f --grid $g --batch $b --frames 24
    rs --ns 1 --fif $f --grid $g --batch $b --frames 24 --size 1024 --spp 30
    rs --ns 1 --fif $f --grid $g --batch $b --frames 120 --size 384 --spp 10
  done
done
for spec in 2:0:1 2:0:2 3:0:1; do
  IFS=: read -r f g b <<< "$spec"
  echo "== C4 fif $f grid $g batch $b"
  rs --ns 1 --fif $f --grid $g --batch $b --frames 8
done
