#!/bin/bash
# Three launches in flight on the full grid with batches, against the default 2 x batches.
set -o pipefail
rs() { timeout -k 10 200 python -u tools/rank_share.py "$@" 2>/dev/null || exit 1; }
for rep in 1 2; do
  for fb in 2:3 3:3 3:2 2:6 3:6; do
    IFS=: read -r f b <<< "$fb"
    echo "== rep $rep fif $f batch $b C3"; rs --ns 1 --fif $f --grid 0 --batch $b --frames 48 --size 1024 --spp 30
  done
  for fb in 2:6 3:6 3:4; do
    IFS=: read -r f b <<< "$fb"
    echo "== rep $rep fif $f batch $b N8"; rs --ns 8 --fif $f --grid 0 --batch $b --frames 48
  done
done
