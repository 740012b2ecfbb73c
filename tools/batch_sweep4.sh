#!/bin/bash
# Batches of 2 for the larger shares: the N=2 share of C4 (2 Mpixel) and the whole C4 frame.
set -o pipefail
rs() { timeout -k 10 200 python -u tools/rank_share.py "$@" 2>/dev/null || exit 1; }
for rep in 1 2; do
  for b in 1 2; do
    echo "== rep $rep batch $b"; rs --ns 1,2 --fif 2 --grid 0 --batch $b --frames 12
  done
done
