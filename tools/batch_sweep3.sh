#!/bin/bash
# Deeper batches for the smallest launches (2 in flight, full grid): the N=8 share of C4 and C2.
set -o pipefail
rs() { timeout -k 10 200 python -u tools/rank_share.py "$@" 2>/dev/null || exit 1; }
for rep in 1 2; do
  for b in 3 4 6; do
    echo "== rep $rep N=8 share batch $b"; rs --ns 8 --fif 2 --grid 0 --batch $b --frames 48
  done
  for b in 3 6 10 16; do
    echo "== rep $rep C2 batch $b"; rs --ns 1 --fif 2 --grid 0 --batch $b --frames 480 --size 384 --spp 10
  done
done
